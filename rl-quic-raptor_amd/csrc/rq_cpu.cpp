// rq_cpu.cpp -- librqcpu.so: the engine's algorithm on host cores, as the CPU baseline.
//
// NOT a product path: librqhip.so never calls it (its device entry points fail without a GPU), and
// only bench.py's cpu_baseline leg and the tests load this library.  It exists so that the GPU path is
// timed against the same algorithm family on the box's own cores ("time the
// build's C++ CPU restatement (same algorithm family) ... 1 thread plus all cores"), instead of the
// oracle's deliberately naive dense elimination.
//
//   encode  the same column program IR as the GPU (rq_colprog.cpp: per-K' elimination compiled to
//           XOR / alpha-multiply nodes), evaluated per block in 64-byte column strips over a
//           liveness-packed slot array that stays in L1/L2
//   decode  the syndrome design of the GPU path (rq_engine.cpp): erased rows zeroed, the union
//           program gives r0, the coefficient rows come from the program on the identity payload,
//           an incremental GF(256) basis picks e independent received repairs (first e + 8 first,
//           then all of them), and x_E = X * s with split-nibble table multiplies -- the
//           reference's own asmSSSE3MulAdd technique (RQ/discmath/optimizations.s:36-78), here as
//           AVX2 vpshufb when the host has it
// Blocks are spread over `threads` host threads (one block at a time per thread).
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rq_colprog.hpp"

namespace rq {
const GF& gf() {
    static const GF g;
    return g;
}
}  // namespace rq

using namespace rq;

namespace {

constexpr uint32_t SW = 64;  // strip width (bytes) evaluated per pass over the program

// IR with every value assigned a slot of a liveness-packed array (linear scan in program order).
struct CpuProg {
    Params p{};
    uint32_t n_out = 0, n_slots = 0;
    struct Op {
        uint8_t k;
        uint32_t d, a, b, c, imm;
    };
    std::vector<Op> ops;
    std::vector<uint8_t> mrep;  // decode: outputs on the identity payload, n_out x mrep_stride
    uint32_t mrep_stride = 0;
};

bool compile(const Params& p, const uint32_t* esi, uint32_t n, CpuProg* cp, std::string* err) {
    ColIR ir;
    if (!build_colprog(p, esi, n, &ir, err)) return false;
    const uint32_t nn = (uint32_t)ir.nodes.size();
    std::vector<uint32_t> last(nn, 0);
    for (uint32_t i = 0; i < nn; ++i)
        for (uint32_t x : {ir.nodes[i].a, ir.nodes[i].b, ir.nodes[i].c})
            if (x != NOVAL) last[x] = i;
    std::vector<uint32_t> slot(nn, NOVAL), freel;
    uint32_t ns = 0;
    cp->p = p;
    cp->n_out = ir.n_out;
    for (uint32_t i = 0; i < nn; ++i) {
        const IrNode& d = ir.nodes[i];
        CpuProg::Op o{d.k, 0, 0, 0, 0, d.imm};
        if (d.a != NOVAL) o.a = slot[d.a];
        if (d.b != NOVAL) o.b = slot[d.b];
        if (d.c != NOVAL) o.c = slot[d.c];
        // operands whose last use is this node free their slots first (the result may reuse one)
        for (uint32_t x : {d.a, d.b, d.c})
            if (x != NOVAL && last[x] == i && slot[x] != NOVAL) {
                freel.push_back(slot[x]);
                slot[x] = NOVAL;
            }
        if (d.k != IR_STORE) {
            uint32_t s;
            if (!freel.empty()) { s = freel.back(); freel.pop_back(); }
            else s = ns++;
            slot[i] = s;
            o.d = s;
            if (last[i] <= i) { freel.push_back(s); slot[i] = NOVAL; }  // dead value (never read)
        }
        cp->ops.push_back(o);
    }
    cp->n_slots = std::max<uint32_t>(ns, 1);
    return true;
}

__attribute__((target_clones("avx512f", "avx2", "default")))
void eval_strip(const CpuProg& cp, uint64_t* V, const uint8_t* src, uint32_t T, uint32_t off, uint8_t* out,
                uint64_t out_row_stride) {
    constexpr uint32_t W = SW / 8;
    const uint32_t w = std::min(SW, T - off);
    for (const CpuProg::Op& o : cp.ops) {
        uint64_t* d = V + (size_t)o.d * W;
        const uint64_t* a = V + (size_t)o.a * W;
        const uint64_t* b = V + (size_t)o.b * W;
        const uint64_t* c = V + (size_t)o.c * W;
        switch (o.k) {
            case IR_LOAD:
                if (w == SW) std::memcpy(d, src + (size_t)o.imm * T + off, SW);
                else { std::memset(d, 0, SW); std::memcpy(d, src + (size_t)o.imm * T + off, w); }
                break;
            case IR_ZERO: for (uint32_t i = 0; i < W; ++i) d[i] = 0; break;
            case IR_XOR2: for (uint32_t i = 0; i < W; ++i) d[i] = a[i] ^ b[i]; break;
            case IR_XOR3: for (uint32_t i = 0; i < W; ++i) d[i] = a[i] ^ b[i] ^ c[i]; break;
            case IR_XT:
                for (uint32_t i = 0; i < W; ++i) {
                    const uint64_t x = a[i], hi = (x >> 7) & 0x0101010101010101ull;
                    d[i] = ((x & 0x7F7F7F7F7F7F7F7Full) << 1) ^ (hi * 0x1D);
                }
                break;
            case IR_XTX:
                for (uint32_t i = 0; i < W; ++i) {
                    const uint64_t x = a[i], hi = (x >> 7) & 0x0101010101010101ull;
                    d[i] = ((x & 0x7F7F7F7F7F7F7F7Full) << 1) ^ (hi * 0x1D) ^ b[i];
                }
                break;
            case IR_STORE: std::memcpy(out + (size_t)o.imm * out_row_stride + off, a, w); break;
        }
    }
}

// Outputs of the program for one block (src: K rows of T bytes) -> out rows (row stride out_row).
void eval_block(const CpuProg& cp, std::vector<uint64_t>& V, const uint8_t* src, uint32_t T, uint8_t* out,
                uint64_t out_row) {
    V.resize((size_t)cp.n_slots * (SW / 8));
    for (uint32_t off = 0; off < T; off += SW) eval_strip(cp, V.data(), src, T, off, out, out_row);
}

// ---------------- GF(256): tables and split-nibble mul-add ----------------
struct MulTab {
    uint8_t lo[256][16], hi[256][16];  // c * i and c * (i << 4)
    MulTab() {
        const GF& g = gf();
        for (int c = 0; c < 256; ++c)
            for (int i = 0; i < 16; ++i) {
                lo[c][i] = g.mul((uint8_t)c, (uint8_t)i);
                hi[c][i] = g.mul((uint8_t)c, (uint8_t)(i << 4));
            }
    }
};
const MulTab& mt() {
    static const MulTab t;
    return t;
}

__attribute__((target("avx2"))) void muladd_avx2(uint8_t* dst, const uint8_t* src, uint8_t c, uint32_t n) {
    const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(mt().lo[c])));
    const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(mt().hi[c])));
    const __m256i m = _mm256_set1_epi8(0x0F);
    uint32_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i l = _mm256_shuffle_epi8(lo, _mm256_and_si256(x, m));
        const __m256i h = _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi16(x, 4), m));
        __m256i* dp = reinterpret_cast<__m256i*>(dst + i);
        _mm256_storeu_si256(dp, _mm256_xor_si256(_mm256_loadu_si256(dp), _mm256_xor_si256(l, h)));
    }
    for (; i < n; ++i) dst[i] ^= (uint8_t)(mt().lo[c][src[i] & 15] ^ mt().hi[c][src[i] >> 4]);
}

void muladd_scalar(uint8_t* dst, const uint8_t* src, uint8_t c, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) dst[i] ^= (uint8_t)(mt().lo[c][src[i] & 15] ^ mt().hi[c][src[i] >> 4]);
}

void muladd(uint8_t* dst, const uint8_t* src, uint8_t c, uint32_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (!c) return;
    if (avx2) muladd_avx2(dst, src, c, n);
    else muladd_scalar(dst, src, c, n);
}

// ---------------- programs, cached per (K, outputs) ----------------
std::mutex g_mu;
std::map<std::string, std::unique_ptr<CpuProg>> g_progs;
thread_local std::string g_err;

CpuProg* get_prog(const Params& p, const std::vector<uint32_t>& esi, bool want_mrep) {
    std::string key = std::to_string(p.K);
    for (uint32_t e : esi) key += "," + std::to_string(e);
    std::lock_guard<std::mutex> lk(g_mu);
    auto& slot = g_progs[key];
    if (!slot) {
        std::unique_ptr<CpuProg> cp(new CpuProg());
        if (!compile(p, esi.data(), (uint32_t)esi.size(), cp.get(), &g_err)) { g_progs.erase(key); return nullptr; }
        slot = std::move(cp);
    }
    CpuProg* cp = slot.get();
    if (want_mrep && !cp->mrep_stride) {  // coefficients: the program on the identity payload
        const uint32_t Ti = (p.K + 3) & ~3u;
        std::vector<uint8_t> id((size_t)p.K * Ti, 0);
        for (uint32_t i = 0; i < p.K; ++i) id[(size_t)i * Ti + i] = 1;
        cp->mrep.assign((size_t)cp->n_out * Ti, 0);
        std::vector<uint64_t> V;
        eval_block(*cp, V, id.data(), Ti, cp->mrep.data(), Ti);
        cp->mrep_stride = Ti;
    }
    return cp;
}

template <class F>
void parallel_blocks(uint32_t n_blocks, int threads, F f) {
    const uint32_t nt = (uint32_t)std::max(1, std::min<int>(threads, (int)n_blocks));
    if (nt <= 1) {
        for (uint32_t b = 0; b < n_blocks; ++b) f(b);
        return;
    }
    std::atomic<uint32_t> next{0};
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; ++t)
        th.emplace_back([&] {
            for (uint32_t b; (b = next.fetch_add(1)) < n_blocks;) f(b);
        });
    for (auto& t : th) t.join();
}

// Incremental basis over the candidate rows (the GPU general solver's algorithm, rq_kernels.hip
// k_solve): returns false if fewer than e independent rows; else X (e x e, X[k][m] at k*e + m) and
// the chosen rows.
bool solve_block(const CpuProg& cp, const uint32_t* E, uint32_t e, const uint32_t* U, uint32_t nr,
                 std::vector<uint8_t>& X, std::vector<uint32_t>& rows) {
    const GF& g = gf();
    const uint32_t W2 = 2 * e;
    std::vector<uint8_t> A((size_t)e * W2), v(W2);
    std::vector<uint32_t> pc(e);
    uint32_t np = 0;
    rows.assign(e, 0);
    for (uint32_t j = 0; j < nr && np < e; ++j) {
        const uint8_t* mr = &cp.mrep[(size_t)U[j] * cp.mrep_stride];
        for (uint32_t c = 0; c < e; ++c) v[c] = mr[E[c]];
        std::fill(v.begin() + e, v.end(), 0);
        v[e + np] = 1;
        for (uint32_t i = 0; i < np; ++i) {
            const uint8_t f = v[pc[i]];
            if (f) muladd(v.data(), &A[(size_t)i * W2], f, W2);
        }
        uint32_t p = e;
        for (uint32_t c = 0; c < e; ++c)
            if (v[c]) { p = c; break; }
        if (p == e) continue;
        const uint8_t inv = g.inv(v[p]);
        for (uint32_t c = 0; c < W2; ++c) v[c] = g.mul(v[c], inv);
        for (uint32_t i = 0; i < np; ++i) {
            uint8_t* r = &A[(size_t)i * W2];
            const uint8_t f = r[p];
            if (f) muladd(r, v.data(), f, W2);
        }
        std::memcpy(&A[(size_t)np * W2], v.data(), W2);
        pc[np] = p;
        rows[np] = j;
        ++np;
    }
    if (np < e) return false;
    X.assign((size_t)e * e, 0);
    for (uint32_t i = 0; i < e; ++i)
        for (uint32_t m = 0; m < e; ++m) X[(size_t)pc[i] * e + m] = A[(size_t)i * W2 + e + m];
    return true;
}

}  // namespace

extern "C" {

const char* rqc_last_error(void) { return g_err.c_str(); }

int rqc_encode(uint32_t K, uint32_t T, uint32_t n_blocks, const uint8_t* src, uint64_t src_stride, const uint32_t* esi,
               uint32_t n_esi, uint8_t* out, uint64_t out_stride, int threads) {
    Params p;
    if (T == 0 || params_for_K(K, &p)) return -5;
    CpuProg* cp = get_prog(p, std::vector<uint32_t>(esi, esi + n_esi), false);
    if (!cp) return -8;
    parallel_blocks(n_blocks, threads, [&](uint32_t b) {
        thread_local std::vector<uint64_t> V;
        eval_block(*cp, V, src + b * src_stride, T, out + b * out_stride, T);
    });
    return 0;
}

// Decode in place (the rq_decode_desc contract with host buffers): status 1 decoded, 0 rank-deficient,
// -3 not enough symbols.
int rqc_decode(uint32_t K, uint32_t T, uint32_t n_blocks, uint8_t* data, uint64_t data_stride, const uint32_t* n_erased,
               const uint32_t* erased, const uint32_t* n_repair, const uint32_t* repair_esi, const uint8_t* repair,
               int32_t* status, int threads) {
    Params p;
    if (T == 0 || params_for_K(K, &p)) return -5;
    std::vector<uint64_t> eoff(n_blocks + 1, 0), roff(n_blocks + 1, 0);
    for (uint32_t b = 0; b < n_blocks; ++b) {
        eoff[b + 1] = eoff[b] + n_erased[b];
        roff[b + 1] = roff[b] + n_repair[b];
    }
    auto run_pass = [&](const std::vector<uint32_t>& blocks, const std::vector<uint32_t>& cnt) -> int {
        std::vector<uint32_t> uni;
        for (uint32_t b : blocks) uni.insert(uni.end(), repair_esi + roff[b], repair_esi + roff[b] + cnt[b]);
        std::sort(uni.begin(), uni.end());
        uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
        CpuProg* cp = get_prog(p, uni, true);
        if (!cp) return -8;
        parallel_blocks((uint32_t)blocks.size(), threads, [&](uint32_t bi) {
            const uint32_t b = blocks[bi], e = n_erased[b], nr = cnt[b];
            uint8_t* blk = data + b * data_stride;
            const uint32_t* E = erased + eoff[b];
            for (uint32_t k = 0; k < e; ++k) std::memset(blk + (size_t)E[k] * T, 0, T);
            std::vector<uint32_t> U(nr);
            for (uint32_t j = 0; j < nr; ++j)
                U[j] = (uint32_t)(std::lower_bound(uni.begin(), uni.end(), repair_esi[roff[b] + j]) - uni.begin());
            std::vector<uint8_t> X;
            std::vector<uint32_t> rows;
            if (!solve_block(*cp, E, e, U.data(), nr, X, rows)) { status[b] = 0; return; }
            thread_local std::vector<uint64_t> V;
            thread_local std::vector<uint8_t> r0, s;
            r0.resize((size_t)uni.size() * T);
            eval_block(*cp, V, blk, T, r0.data(), T);
            s.resize((size_t)e * T);  // syndromes of the chosen rows
            for (uint32_t m = 0; m < e; ++m) {
                const uint8_t* r = repair + (roff[b] + rows[m]) * (uint64_t)T;
                const uint8_t* z = &r0[(size_t)U[rows[m]] * T];
                for (uint32_t c = 0; c < T; ++c) s[(size_t)m * T + c] = r[c] ^ z[c];
            }
            for (uint32_t k = 0; k < e; ++k) {
                uint8_t* dst = blk + (size_t)E[k] * T;
                for (uint32_t m = 0; m < e; ++m) muladd(dst, &s[(size_t)m * T], X[(size_t)k * e + m], T);
            }
            status[b] = 1;
        });
        return 0;
    };
    std::vector<uint32_t> blocks, cnt(n_blocks, 0);
    for (uint32_t b = 0; b < n_blocks; ++b) {
        const uint32_t e = n_erased[b], nr = n_repair[b];
        if (e > nr) { status[b] = -3; continue; }
        if (e == 0) { status[b] = 1; continue; }
        cnt[b] = std::min(nr, e + 8);
        blocks.push_back(b);
    }
    if (blocks.empty()) return 0;
    int rc = run_pass(blocks, cnt);
    if (rc) return rc;
    std::vector<uint32_t> again;
    for (uint32_t b : blocks)
        if (status[b] == 0 && cnt[b] < n_repair[b]) { cnt[b] = n_repair[b]; again.push_back(b); }
    return again.empty() ? 0 : run_pass(again, cnt);
}

}  // extern "C"
