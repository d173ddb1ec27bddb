// fec_raptorq.hpp -- C++ host mirror of the reference's go/fec RaptorQ API, over the rqhip C-ABI.
//
// The reference's host code is Go (go/fec/raptorq_wrap.go:13-124); no Go toolchain exists in
// this image, so the host side above the C-ABI is written in C++ with the same names, argument
// meaning and error behaviour.  Go's (value, error) pairs become a value plus an `Error`
// (empty message == nil).  The cgo shim a Go maintainer would add instead is in INTEGRATION.md.
//
//   Go (reference)                                       C++ (this header)
//   NewRaptorQEncoder(data []byte, K, L int)             fec::NewRaptorQEncoder(data, K, L, &err)
//   (*RaptorQEncoder).GenSymbol(id uint32) []byte        enc->GenSymbol(id)
//   (*RaptorQEncoder).BaseSymbolsNum() uint32            enc->BaseSymbolsNum()
//   NewRaptorQDecoder(dataSize, L int)                   fec::NewRaptorQDecoder(size, L, &err)
//   (*RaptorQDecoder).AddSymbol(id, data) (bool, error)  dec->AddSymbol(id, data, &err)
//   (*RaptorQDecoder).Decode() (bool, []byte, error)     dec->Decode(&out, &err)
//   RaptorQEncodeBlock(data, N, K, L) ([]Packet, error)  fec::RaptorQEncodeBlock(data, N, K, L, &err)
//   RaptorQDecodeBytes(recv, N, K, L, size) ([]byte,bool) fec::RaptorQDecodeBytes(recv, N, K, L, size, &ok)
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rqhip.h"

namespace fec {

using Bytes = std::vector<uint8_t>;

struct Error {
    int code = RQ_OK;
    std::string msg;  // empty == nil
    explicit operator bool() const { return code != RQ_OK; }
};

inline Error last_error(int code) {
    Error e;
    e.code = code;
    const char* d = rq_last_error();
    e.msg = (d && *d) ? d : rq_strerror(code);
    return e;
}

// fec.Packet (go/fec/packet_polar.go:87-90)
struct Packet {
    int Index = 0;
    Bytes Data;
};

class RaptorQEncoder {
  public:
    int K = 0, L = 0;
    ~RaptorQEncoder() { if (h_) rq_encoder_free(h_); }
    RaptorQEncoder(const RaptorQEncoder&) = delete;
    RaptorQEncoder& operator=(const RaptorQEncoder&) = delete;

    // GenSymbol: id < K -> systematic source symbol, else repair symbol (raptorq_wrap.go:44-46).
    Bytes GenSymbol(uint32_t id) const {
        Bytes out(rq_encoder_symbol_size(h_));
        if (rq_encoder_symbol(h_, id, out.data()) != RQ_OK) out.clear();
        return out;
    }
    // Batch extension used by RaptorQEncodeBlock: symbols first..first+count-1, one launch.
    std::vector<Bytes> GenSymbols(uint32_t first, uint32_t count, Error* err) const {
        const uint32_t T = rq_encoder_symbol_size(h_);
        Bytes flat((size_t)T * count);
        std::vector<Bytes> out;
        const int rc = rq_encoder_symbols(h_, first, count, flat.data());
        if (rc != RQ_OK) { if (err) *err = last_error(rc); return out; }
        for (uint32_t i = 0; i < count; ++i) out.emplace_back(flat.begin() + (size_t)i * T, flat.begin() + (size_t)(i + 1) * T);
        return out;
    }
    uint32_t BaseSymbolsNum() const { return rq_encoder_k(h_); }

  private:
    friend std::unique_ptr<RaptorQEncoder> NewRaptorQEncoder(const Bytes&, int, int, Error*);
    RaptorQEncoder() = default;
    rq_enc* h_ = nullptr;
};

// raptorq_wrap.go:29-40
inline std::unique_ptr<RaptorQEncoder> NewRaptorQEncoder(const Bytes& data, int K, int L, Error* err) {
    if (K <= 0 || L <= 0) { if (err) *err = Error{RQ_ERR_BAD_ARG, "bad K or L"}; return nullptr; }
    int rc = RQ_OK;
    rq_enc* h = rq_encoder_create(data.data(), data.size(), (uint32_t)L, &rc);
    if (!h) { if (err) *err = last_error(rc); return nullptr; }
    std::unique_ptr<RaptorQEncoder> e(new RaptorQEncoder());
    e->K = K;
    e->L = L;
    e->h_ = h;
    if (err) *err = Error{};
    return e;
}

class RaptorQDecoder {
  public:
    int K = 0, L = 0;
    ~RaptorQDecoder() { if (h_) rq_decoder_free(h_); }
    RaptorQDecoder(const RaptorQDecoder&) = delete;
    RaptorQDecoder& operator=(const RaptorQDecoder&) = delete;

    // AddSymbol: returns whether decoding can be attempted (K <= unique symbols held).
    bool AddSymbol(uint32_t id, const Bytes& data, Error* err) {
        int can = 0;
        const int rc = rq_decoder_add(h_, id, data.data(), data.size(), &can);
        if (err) *err = rc == RQ_OK ? Error{} : last_error(rc);
        return can != 0;
    }
    // Decode: (ok, bytes, err); ok=false with no error when the system is rank-deficient.
    bool Decode(Bytes* out, Error* err) {
        out->assign(size_, 0);
        int ok = 0;
        const int rc = rq_decoder_decode(h_, out->data(), &ok);
        if (rc != RQ_OK) { out->clear(); if (err) *err = last_error(rc); return false; }
        if (err) *err = Error{};
        if (!ok) out->clear();
        return ok != 0;
    }

  private:
    friend std::unique_ptr<RaptorQDecoder> NewRaptorQDecoder(int, int, Error*);
    RaptorQDecoder() = default;
    rq_dec* h_ = nullptr;
    size_t size_ = 0;
};

// raptorq_wrap.go:52-63
inline std::unique_ptr<RaptorQDecoder> NewRaptorQDecoder(int dataSize, int L, Error* err) {
    if (dataSize < 0 || L <= 0) { if (err) *err = Error{RQ_ERR_BAD_ARG, "bad dataSize or L"}; return nullptr; }
    int rc = RQ_OK;
    rq_dec* h = rq_decoder_create((uint64_t)dataSize, (uint32_t)L, &rc);
    if (!h) { if (err) *err = last_error(rc); return nullptr; }
    std::unique_ptr<RaptorQDecoder> d(new RaptorQDecoder());
    d->K = (int)rq_decoder_k(h);
    d->L = L;
    d->h_ = h;
    d->size_ = (size_t)dataSize;
    if (err) *err = Error{};
    return d;
}

// raptorq_wrap.go:81-99 (data clamped to K*L; symbols 0..N-1)
inline std::vector<Packet> RaptorQEncodeBlock(Bytes data, int N, int K, int L, Error* err) {
    std::vector<Packet> out;
    if (N <= 0 || K <= 0 || L <= 0 || K > N) { if (err) *err = Error{RQ_ERR_BAD_ARG, "bad N/K/L"}; return out; }
    if (data.size() > (size_t)K * L) data.resize((size_t)K * L);
    auto enc = NewRaptorQEncoder(data, K, L, err);
    if (!enc) return out;
    auto syms = enc->GenSymbols(0, (uint32_t)N, err);
    if (syms.size() != (size_t)N) return out;
    for (int i = 0; i < N; ++i) out.push_back(Packet{i, std::move(syms[i])});
    if (err) *err = Error{};
    return out;
}

// raptorq_wrap.go:103-124 (bad Index and AddSymbol errors ignored)
inline Bytes RaptorQDecodeBytes(const std::vector<Packet>& recv, int N, int K, int L, int dataSize, bool* ok) {
    *ok = false;
    if (K <= 0 || L <= 0 || dataSize < 0) return {};
    Error err;
    auto dec = NewRaptorQDecoder(dataSize, L, &err);
    if (!dec) return {};
    for (const Packet& p : recv) {
        if (p.Index < 0 || p.Index >= N) continue;
        Error e;
        dec->AddSymbol((uint32_t)p.Index, p.Data, &e);
    }
    Bytes out;
    const bool good = dec->Decode(&out, &err);
    if (err || !good) return {};
    *ok = true;
    return out;
}

}  // namespace fec
