// fq_tx.cpp -- fecquic sender on the GPU engine (see fq_tx.hpp).
#include "fq_tx.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../include/rqhip.h"
#include "fq_wire.hpp"

namespace fq {

namespace {

using Clock = std::chrono::steady_clock;

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Pinned {
    uint8_t* p = nullptr;
    explicit Pinned(size_t n) : p(static_cast<uint8_t*>(rq_host_alloc(n))) {}
    ~Pinned() { rq_host_free(p); }
};

size_t read_full(int fd, uint8_t* p, size_t n) {
    size_t got = 0;
    while (got < n) {
        const ssize_t r = ::read(fd, p + got, n - got);
        if (r <= 0) break;
        got += (size_t)r;
    }
    return got;
}

}  // namespace

int send_file(const std::string& path, const TxOptions& o, const std::function<void(const uint8_t*, size_t)>& send,
              TxStats* st) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return -1;
    const uint32_t K = o.K, N = o.N, L = o.L, R = N - K, W = std::max<uint32_t>(1, o.window);
    const size_t blk = (size_t)K * L;
    Pinned src(blk * W), rep((size_t)std::max<uint32_t>(R, 1) * L * W);
    if (!src.p || !rep.p) { ::close(fd); return RQ_ERR_DEVICE; }
    std::vector<uint32_t> esi(R);
    for (uint32_t i = 0; i < R; ++i) esi[i] = K + i;
    std::mt19937_64 rng(o.seed);
    std::uniform_real_distribution<double> uni(0.0, 1.0);
    std::vector<uint8_t> dg(HEADER_MAX_LEN + L);
    const auto t_start = Clock::now();
    uint32_t block_id = 0;
    int rc = 0;
    bool eof = false;
    // emits block b of the window: ESI 0..N-1, sources from s (kk rows), repairs from r
    auto emit = [&](const uint8_t* s, const uint8_t* r, uint32_t kk) -> int {
        for (uint32_t i = 0; i < N; ++i) {
            FecHeader h;
            h.scheme = SCHEME_RAPTORQ;
            h.block_id = block_id;
            h.n = N;
            h.k = K;  // the wire K (transfer.go:191); a short block's library K travels implicitly
            h.sym_id = i;
            h.payload_len = L;
            uint32_t hl;
            if (o.header_version) {
                h.version = (uint8_t)o.header_version;
                hl = marshal(h, dg.data());
            } else {
                hl = marshal_auto(h, dg.data());
            }
            if (!hl) return -2;
            std::memcpy(dg.data() + hl, i < kk ? s + (size_t)i * L : r + (size_t)(i - kk) * L, L);
            if (o.drop > 0 && uni(rng) < o.drop) {
                st->dropped++;
                continue;
            }
            const auto t0 = Clock::now();
            send(dg.data(), hl + L);
            st->send_s += secs(t0, Clock::now());
            st->dgrams++;
            st->bytes += hl + L;
        }
        st->blocks++;
        ++block_id;
        return 0;
    };
    while (!eof && rc == 0) {
        const size_t got = read_full(fd, src.p, blk * W);
        const uint32_t full = (uint32_t)(got / blk);
        const size_t tail = got - (size_t)full * blk;
        eof = got < blk * W;
        if (full) {
            const auto t0 = Clock::now();
            rq_encode_desc d{};
            d.T = L; d.K = K; d.n_blocks = full; d.src = src.p; d.src_stride = blk;
            d.n_esi = R; d.esi = esi.data(); d.out = rep.p; d.out_stride = (uint64_t)R * L;
            if (R && (rc = rq_encode_batch_host(&d, o.device_mask)) != 0) break;
            st->gpu_calls += R ? 1 : 0;
            st->enc_s += secs(t0, Clock::now());
            for (uint32_t b = 0; b < full && rc == 0; ++b)
                rc = emit(src.p + b * blk, rep.p + (size_t)b * R * L, K);
        }
        if (tail && rc == 0) {  // the final short block: library K = ceil(bytes / L), zero padded
            const uint32_t kk = (uint32_t)((tail + L - 1) / L);
            uint8_t* s = src.p + (size_t)full * blk;
            std::memset(s + tail, 0, (size_t)kk * L - tail);
            std::vector<uint32_t> e2;
            for (uint32_t i = kk; i < N; ++i) e2.push_back(i);
            const auto t0 = Clock::now();
            rq_encode_desc d{};
            d.T = L; d.K = kk; d.n_blocks = 1; d.src = s; d.src_stride = (uint64_t)kk * L;
            d.n_esi = (uint32_t)e2.size(); d.esi = e2.data(); d.out = rep.p; d.out_stride = (uint64_t)e2.size() * L;
            if (!e2.empty() && (rc = rq_encode_batch_host(&d, o.device_mask)) != 0) break;
            st->gpu_calls += e2.empty() ? 0 : 1;
            st->enc_s += secs(t0, Clock::now());
            rc = emit(s, rep.p, kk);
        }
        if (o.pace_us) std::this_thread::sleep_for(std::chrono::microseconds(o.pace_us));
    }
    ::close(fd);
    st->dur_s = secs(t_start, Clock::now());
    return rc;
}

}  // namespace fq
