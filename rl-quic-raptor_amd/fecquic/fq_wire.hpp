// fq_wire.hpp -- symbol and file headers of the fecquic transfer.
//
// Version 1 is go/internal/fecwire/header.go:15-59 byte for byte: 16 bytes, little endian,
// {Version u8, Scheme u8, BlockID u16, N u8, K u8, SymID u8, Flags u8, PayloadLen u32, SeedOrIdx u32}.
// Its uint8 N/K/SymID cap blocks at K <= 255, so the K=1024/2048 configs cannot
// travel in it.  Version 2 widens them and the block counter:
//   {Version u8 = 2, Scheme u8, Flags u16, BlockID u32, K u16, HdrLen u16 = 24, N u32, SymID u32,
//    PayloadLen u32}                                                              24 bytes, LE
// (K <= 56403, the largest RFC 6330 K', fits u16).  unmarshal() reads either version by the first
// byte, so a v2 receiver still takes every v1 datagram; a v1 receiver (the reference) rejects v2
// datagrams at its Scheme check only by accident, so senders emit v1 whenever the block fits it.
//
// FileHeader is go/fecquic/fileheader.go:10-57 ("QFEC", version 1, size, SHA-256, chunk L).
#pragma once
#include <cstdint>
#include <cstring>

namespace fq {

constexpr uint8_t SCHEME_RLC = 0, SCHEME_RS = 1, SCHEME_POLAR = 2, SCHEME_RAPTORQ = 3;  // header.go:9-14
constexpr uint32_t HEADER_V1_LEN = 16, HEADER_V2_LEN = 24, HEADER_MAX_LEN = 24;

struct FecHeader {
    uint8_t version = 1;
    uint8_t scheme = SCHEME_RAPTORQ;
    uint16_t flags = 0;
    uint32_t block_id = 0;
    uint32_t n = 0, k = 0, sym_id = 0;
    uint32_t payload_len = 0;
    uint32_t seed_or_idx = 0;  // v1 only
};

inline void put16(uint8_t* b, uint16_t v) { b[0] = (uint8_t)v; b[1] = (uint8_t)(v >> 8); }
inline void put32(uint8_t* b, uint32_t v) { for (int i = 0; i < 4; ++i) b[i] = (uint8_t)(v >> (8 * i)); }
inline uint16_t get16(const uint8_t* b) { return (uint16_t)(b[0] | (b[1] << 8)); }
inline uint32_t get32(const uint8_t* b) {
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

// True when the header's fields fit version 1.
inline bool fits_v1(const FecHeader& h) {
    return h.block_id <= 0xFFFF && h.n <= 0xFF && h.k <= 0xFF && h.sym_id <= 0xFF && h.flags <= 0xFF;
}

// Writes h as h.version (1 or 2) into b (>= HEADER_MAX_LEN bytes); returns the header length, 0 if
// the fields do not fit the requested version.
inline uint32_t marshal(const FecHeader& h, uint8_t* b) {
    if (h.version == 1) {  // header.go:29-43
        if (!fits_v1(h)) return 0;
        b[0] = 1;
        b[1] = h.scheme;
        put16(b + 2, (uint16_t)h.block_id);
        b[4] = (uint8_t)h.n;
        b[5] = (uint8_t)h.k;
        b[6] = (uint8_t)h.sym_id;
        b[7] = (uint8_t)h.flags;
        put32(b + 8, h.payload_len);
        put32(b + 12, h.seed_or_idx);
        return HEADER_V1_LEN;
    }
    if (h.version == 2) {
        if (h.k > 0xFFFF) return 0;
        b[0] = 2;
        b[1] = h.scheme;
        put16(b + 2, h.flags);
        put32(b + 4, h.block_id);
        put16(b + 8, (uint16_t)h.k);
        put16(b + 10, (uint16_t)HEADER_V2_LEN);
        put32(b + 12, h.n);
        put32(b + 16, h.sym_id);
        put32(b + 20, h.payload_len);
        return HEADER_V2_LEN;
    }
    return 0;
}

// The smallest version that carries h (v1 whenever the block fits it).
inline uint32_t marshal_auto(FecHeader h, uint8_t* b) {
    h.version = fits_v1(h) ? 1 : 2;
    return marshal(h, b);
}

// Parses a header of either version; returns its length (0: short or unknown version).  v1 keeps
// the reference's rule that any byte-0 value parses as v1 fields (header.go:45-59 checks only the
// length); here byte 0 == 2 selects v2 and everything else parses as v1.
inline uint32_t unmarshal(const uint8_t* b, uint32_t len, FecHeader* h) {
    if (len >= 1 && b[0] == 2) {
        if (len < HEADER_V2_LEN || get16(b + 10) != HEADER_V2_LEN) return 0;
        h->version = 2;
        h->scheme = b[1];
        h->flags = get16(b + 2);
        h->block_id = get32(b + 4);
        h->k = get16(b + 8);
        h->n = get32(b + 12);
        h->sym_id = get32(b + 16);
        h->payload_len = get32(b + 20);
        h->seed_or_idx = 0;
        return HEADER_V2_LEN;
    }
    if (len < HEADER_V1_LEN) return 0;
    h->version = b[0];
    h->scheme = b[1];
    h->block_id = get16(b + 2);
    h->n = b[4];
    h->k = b[5];
    h->sym_id = b[6];
    h->flags = b[7];
    h->payload_len = get32(b + 8);
    h->seed_or_idx = get32(b + 12);
    return HEADER_V1_LEN;
}

// go/fecquic/fileheader.go:10-57.
constexpr uint32_t FILE_HEADER_LEN = 4 + 2 + 8 + 32 + 4 + 8;
struct FileHeader {
    uint16_t version = 1;
    uint64_t file_size = 0;
    uint8_t sha256[32] = {};
    uint32_t chunk_l = 0;
};

inline void marshal_file(const FileHeader& h, uint8_t* b) {
    std::memset(b, 0, FILE_HEADER_LEN);
    std::memcpy(b, "QFEC", 4);
    put16(b + 4, h.version);
    for (int i = 0; i < 8; ++i) b[6 + i] = (uint8_t)(h.file_size >> (8 * i));
    std::memcpy(b + 14, h.sha256, 32);
    put32(b + 46, h.chunk_l);
}

// 0 ok; -1 short header; -2 bad magic; -3 unsupported version (fileheader.go:42-57).
inline int unmarshal_file(const uint8_t* b, uint32_t len, FileHeader* h) {
    if (len < FILE_HEADER_LEN) return -1;
    if (std::memcmp(b, "QFEC", 4) != 0) return -2;
    h->version = get16(b + 4);
    if (h->version != 1) return -3;
    h->file_size = 0;
    for (int i = 0; i < 8; ++i) h->file_size |= (uint64_t)b[6 + i] << (8 * i);
    std::memcpy(h->sha256, b + 14, 32);
    h->chunk_l = get32(b + 46);
    return 0;
}

}  // namespace fq
