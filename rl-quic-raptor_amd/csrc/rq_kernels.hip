// rq_kernels.hip -- HIP kernels for gfx950 (CDNA4): RaptorQ encode-schedule replay, LT repair
// generation, and syndrome decode (solve + apply).  No MFMA: GF(2)/GF(256) byte arithmetic.
//
// Reference hot routines replaced (native inventory):
//   asmSSE2XORBlocks  RQ/discmath/optimizations.s:9-28   -> dword XOR of LDS-resident strip rows
//   asmSSSE3MulAdd    RQ/discmath/optimizations.s:36-78  -> gfmul4 (packed 4-byte GF(256) mul)
//   Solve             RQ/solver.go:25-185                -> k_encode replaying the per-K' plan
//   encodeGen         RQ/params.go:162-182               -> k_encode output stage / k_gather
//   Decoder.Decode    RQ/decoder.go:64-134               -> k_encode (syndromes) + k_solve + k_apply
//
// Data layout: a source block is K rows of T bytes (row-major, as the wire carries symbols).
// One workgroup owns one (block, column strip); the strip of every intermediate-symbol slot
// (n_slots x sd dwords) lives in LDS for the whole program, so HBM is touched only to read the
// source strip once (plus L2-resident re-reads of rows named by SRC_GLOBAL terms) and to write
// the requested output rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "rfc6330_tables.h"
#include "rq_device.hpp"
#include "rq_wave_format.hpp"

namespace rq {

__constant__ uint32_t c_V[4][256];
__constant__ uint32_t c_DEG[31];

int upload_tables() {
    uint32_t v[4][256];
    for (int i = 0; i < 256; ++i) {
        v[0][i] = RQ_V0[i]; v[1][i] = RQ_V1[i]; v[2][i] = RQ_V2[i]; v[3][i] = RQ_V3[i];
    }
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_V), v, sizeof v);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_DEG), RQ_DEGREE_F, sizeof(uint32_t) * 31);
    return (int)e;
}

// ------------------------------ GF(256) on packed dwords ------------------------------------
__device__ __forceinline__ uint32_t xtime4(uint32_t x) {
    const uint32_t hi = (x >> 7) & 0x01010101u;
    const uint32_t mask = (hi << 8) - hi;  // 0x00 / 0xFF per byte (no multiply)
    return ((x & 0x7F7F7F7Fu) << 1) ^ (mask & 0x1D1D1D1Du);
}
// x * c in GF(256) for each of the 4 bytes of x (poly 0x11D): XOR over the bits b of x of
// (c * 2^b) -- eight independent terms (short dependency chain) instead of a doubling chain on x.
__device__ __forceinline__ uint32_t gfmul4(uint32_t x, uint32_t c) {
    uint32_t r = 0, kb = c & 0xFFu;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t m = (x >> b) & 0x01010101u;
        const uint32_t mask = (m << 8) - m;            // 0x00 / 0xFF per byte
        r ^= mask & (__umul24(kb, 0x010101u) | (kb << 24));  // kb replicated to 4 bytes
        kb = ((kb << 1) ^ ((kb & 0x80u) ? 0x11Du : 0u)) & 0xFFu;
    }
    return r;
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {  // one v_bitop3_b32
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// alpha * x per byte without a multiply: v_perm_b32 selectors 8..11 replicate the top bit of
// bytes 1, 3, 5, 7 of {S0:S1}; with S1 = x, S0 = x << 8 those are the top bits of x's bytes
// 1, 3, 0, 2, so selector 0x090B080A yields 0xFF in every byte whose top bit is set.
__device__ __forceinline__ uint32_t xtime4p(uint32_t x) {
    const uint32_t m = __builtin_amdgcn_perm(x << 8, x, 0x090B080Au);
    return ((x << 1) & 0xFEFEFEFEu) ^ (m & 0x1D1D1D1Du);
}
// c * x per byte from the host-built byte tables of c (rq_core.hpp gf_perm_tables): three
// v_perm_b32 lookups on the 3/3/2-bit groups of each byte.
__device__ __forceinline__ uint32_t gfmul4_tab(uint32_t x, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                               uint32_t t4) {
    const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
    return xor3(__builtin_amdgcn_perm(t1, t0, s0), __builtin_amdgcn_perm(t3, t2, s1), __builtin_amdgcn_perm(t4, t4, s2));
}

// ------------------------------ LT tuple on device (RQ/params.go:83-112) -------------------
__device__ __forceinline__ uint32_t d_rand(uint32_t y, uint32_t i, uint32_t m) {
    return (c_V[0][(y + i) & 255u] ^ c_V[1][((y >> 8) + i) & 255u] ^ c_V[2][((y >> 16) + i) & 255u] ^
            c_V[3][((y >> 24) + i) & 255u]) % m;
}
struct LtIter {
    uint32_t d, a, b, d1, a1, b1;
};
__device__ __forceinline__ LtIter d_tuple(const DevParams& p, uint32_t X) {
    uint32_t A = 53591u + 997u * p.J;
    if ((A & 1u) == 0) ++A;
    const uint32_t y = 10267u * (p.J + 1u) + X * A;
    const uint32_t v = d_rand(y, 0, 1u << 20);
    uint32_t d = 30;
    for (uint32_t i = 0; i < 31; ++i)
        if (v < c_DEG[i]) { d = i; break; }
    if (d > p.W - 2) d = p.W - 2;
    LtIter t;
    t.d = d;
    t.a = 1 + d_rand(y, 1, p.W - 1);
    t.b = d_rand(y, 2, p.W);
    t.d1 = d < 4 ? 2 + d_rand(X, 3, 2) : 2;
    t.a1 = 1 + d_rand(X, 4, p.P1 - 1);
    t.b1 = d_rand(X, 5, p.P1);
    return t;
}
// Calls f(col) for every column XORed into the symbol of ISI X (encodeGen order).
template <class F>
__device__ __forceinline__ void d_for_cols(const DevParams& p, uint32_t X, F&& f) {
    LtIter t = d_tuple(p, X);
    uint32_t b = t.b;
    f(b);
    for (uint32_t j = 1; j < t.d; ++j) { b = (b + t.a) % p.W; f(b); }
    uint32_t b1 = t.b1;
    while (b1 >= p.P) b1 = (b1 + t.a1) % p.P1;
    f(p.W + b1);
    for (uint32_t j = 1; j < t.d1; ++j) {
        b1 = (b1 + t.a1) % p.P1;
        while (b1 >= p.P) b1 = (b1 + t.a1) % p.P1;
        f(p.W + b1);
    }
}

// ------------------------------ encode: plan replay ------------------------------------------
constexpr uint32_t OUT_BATCH = 128;  // LT tuples staged in LDS per output batch

__device__ __forceinline__ uint32_t d_degree(uint32_t v, uint32_t W) {
    // first d with v < DEG[d] (DEG[0] = 0, DEG[30] = 2^20 > v): branch-free binary search
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 16; step; step >>= 1)
        if (lo + step <= 30 && c_DEG[lo + step - 1] <= v) lo += step;
    const uint32_t d = lo;  // c_DEG[d-1] <= v < c_DEG[d]
    return d > W - 2 ? W - 2 : d;
}

// grid = (n_strips, n_blocks), block = NW waves.  LDS: n_slots x sd dwords, the LT-tuple
// staging area (OUT_BATCH x 6 words) and the erasure bitmap.  Each wave executes its own
// instruction stream (WaveProgram): an op runs two statements side by side (lanes 0-31
// statement A, lanes 32-63 statement B, one strip dword per lane); a workgroup barrier closes
// each dependency level.  Descriptor words are wave-uniform and live in two VGPR pages (current
// and prefetched next), extracted with v_readlane: no memory latency inside a segment.
// ERASE: decode's syndrome pass (erased source rows read as zero); a separate instantiation so
// the encode path carries no erasure checks and profiles name the two passes apart.
template <int NW, bool ERASE>
__global__ void __launch_bounds__(NW * 64) k_encode(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t sd = a.sd, T = a.T, Td = T >> 2;
    const uint32_t strip = blockIdx.x;
    const uint32_t b = a.blk_map ? a.blk_map[blockIdx.y] : blockIdx.y;
    const uint32_t c0 = strip * sd;
    const uint32_t width = min(sd, Td - c0);
    const uint32_t tid = threadIdx.x, nthr = NW * 64;
    const uint32_t K = a.p.K;
    const uint32_t nebw = ERASE ? (K + 31) / 32 : 0;
    // LDS: slot image | R (stream ring during the program, LT-tuple staging after it) | bitmap
    const uint32_t img = (a.n_slots * sd + 3u) & ~3u;           // dwords, 16-byte aligned
    const uint32_t rsz = max(NW * 2u * WV_PAGE, OUT_BATCH * 6u);
    uint32_t* tup = lds + img;                                  // OUT_BATCH x 6 (after the program)
    uint32_t* ebits = lds + img + rsz;

    // per-wave stream ring: two 64-word pages (current, next) staged from global memory
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63u;
    const uint32_t* ws = a.wstream;
    uint32_t pg = __builtin_amdgcn_readfirstlane(a.wave_off[wave]);  // word offset of the current page
    uint32_t* ring = lds + img + wave * 2u * WV_PAGE;
    {
        const uint32_t p0 = ws[pg + lane], p1 = ws[pg + WV_PAGE + lane];
        ring[lane] = p0;
        ring[WV_PAGE + lane] = p1;
    }

    {   // zero the slot image (16-byte stores) and the bitmap
        const uint32_t nw4 = (a.n_slots * sd) >> 2;
        uint4* l4 = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = tid; i < nw4; i += nthr) l4[i] = make_uint4(0, 0, 0, 0);
        for (uint32_t i = (nw4 << 2) + tid; i < a.n_slots * sd; i += nthr) lds[i] = 0;
        for (uint32_t i = tid; i < nebw; i += nthr) ebits[i] = 0;
    }
    __syncthreads();
    if (nebw) {
        for (uint32_t i = a.erased_off[b] + tid; i < a.erased_off[b + 1]; i += nthr) {
            const uint32_t e = a.erased[i];
            if (e < K) atomicOr(&ebits[e >> 5], 1u << (e & 31));
        }
        __syncthreads();
    }
    const uint32_t half = lane >> 5, hl = lane & 31u;
    const uint32_t grp = tid >> 5, ngrp = nthr >> 5;
    const uint32_t hlc = min(hl, sd - 1);  // lanes past the strip read a valid column, never write
    const bool live = hl < sd;
    const bool inb = hl < width;
    const uint8_t* blk = a.src + (size_t)b * a.src_stride;
    const uint8_t* gcol = blk + (size_t)(c0 + hlc) * 4;
    auto erased_row = [&](uint32_t r) -> bool { return ERASE && ((ebits[r >> 5] >> (r & 31)) & 1u); };
    if (!(a.dbg & 1u)) {   // source strip -> slots: one 32-lane group per row, 4 rows in flight per group
        uint32_t r = grp;
        for (; r + 3 * ngrp < K; r += 4 * ngrp) {
            uint32_t v[4], s[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t row = r + u * ngrp;
                v[u] = inb ? *reinterpret_cast<const uint32_t*>(gcol + (size_t)row * T) : 0u;
                s[u] = a.load_slot[row];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (inb && !erased_row(r + u * ngrp)) lds[s[u] * sd + hl] = v[u];
        }
        for (; r < K; r += ngrp)
            if (inb && !erased_row(r)) lds[(uint32_t)a.load_slot[r] * sd + hl] = *reinterpret_cast<const uint32_t*>(gcol + (size_t)r * T);
    }
    __syncthreads();

    auto gload = [&](uint32_t isi) -> uint32_t {
        if (!inb || isi >= K || erased_row(isi)) return 0u;
        return *reinterpret_cast<const uint32_t*>(gcol + (size_t)isi * T);
    };

    // ---- the wave's instruction stream (rq_wave_format.hpp) ----
    // Each half of the wave reads its 4 words of a group with one ds_read_b128; slot fields are
    // LDS byte offsets, so a source costs one add (the lane's column) and one ds_read_b32.
    char* const ldsb = reinterpret_cast<char*>(lds);
    const uint32_t hl4 = hlc << 2;
    const uint32_t ring_b = (uint32_t)((char*)ring - ldsb);
    const uint32_t hv = ring_b + (half << 4);  // this half's words of a group
    auto grp_at = [&](uint32_t gpos) -> uint4 {  // gpos: byte offset of a group within the ring
        return *reinterpret_cast<const uint4*>(ldsb + hv + gpos);
    };
    auto rd = [&](uint32_t off) -> uint32_t { return *reinterpret_cast<const uint32_t*>(ldsb + off + hl4); };
    // lanes past the strip write the (last) trash slot
    const uint32_t trash_b = (a.n_slots - 1) * sd * 4 + hl4;
    auto wr_addr = [&](uint32_t off) -> uint32_t { return live ? off + hl4 : trash_b; };
    auto wr = [&](uint32_t addr, uint32_t v) { *reinterpret_cast<uint32_t*>(ldsb + addr) = v; };
    constexpr uint32_t GB = WV_GROUP * 4;  // group bytes

    const uint32_t n_levels = (a.dbg & 2u) ? 0u : a.n_levels;
    // diagnostics: per level and wave, [cycles working, cycles at the barrier] of workgroup (0,0)
    const bool stamping = a.stamp && blockIdx.x == 0 && blockIdx.y == 0 && lane == 0;
    unsigned long long t_lv = stamping ? __builtin_amdgcn_s_memtime() : 0ull;
    // Page refills are LDS-DMA (global_load_lds_dword: 64 lanes x 4 B = one page straight into
    // the freed ring slot, no VGPR).  The compiler does not see them; each is waited for with
    // vmcnt(0) at the next page switch, which orders the wave's own later ds_reads behind it.
    // The compiler's counted waits for its own loads stay correct (at worst they wait longer).
    // compiler-visible drain of the prologue's loads, so no VMEM wait lands inside the loop
    __builtin_amdgcn_s_waitcnt(0x0F70);

    uint32_t cslot = 0;   // ring page slot of the current page
    // page switch: the next page is staged in the other slot; refill this one with the page after
    auto advance = [&]() -> uint32_t {
        const uint32_t old_b = ring_b + cslot * (WV_PAGE * 4);  // wave-uniform LDS address of the freed slot
        cslot ^= 1u;
        pg += WV_PAGE;
        const uint32_t* src = ws + pg + WV_PAGE + lane;        // the page after the new current one
        uint32_t keep;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
                     "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(old_b) : "memory");
        return cslot * (WV_PAGE * 4);
    };
    // XOR of 4N sources (N payload groups), straight-line: all group reads, then all source reads
    auto xor_n = [&](auto NC, uint32_t pay) -> uint32_t {
        constexpr uint32_t N = decltype(NC)::value;
        uint4 s[N];
#pragma unroll
        for (uint32_t q = 0; q < N; ++q) s[q] = grp_at(pay + q * GB);
        uint32_t v = 0;
#pragma unroll
        for (uint32_t q = 0; q < N; ++q) v = xor3(xor3(v, rd(s[q].x), rd(s[q].y)), rd(s[q].z), rd(s[q].w));
        return v;
    };
    auto mul_n = [&](auto NC, uint32_t pay) -> uint32_t {
        constexpr uint32_t N = decltype(NC)::value;  // sources (2 groups each)
        uint4 g1[N], g2[N];
#pragma unroll
        for (uint32_t q = 0; q < N; ++q) { g1[q] = grp_at(pay + 2 * q * GB); g2[q] = grp_at(pay + (2 * q + 1) * GB); }
        uint32_t v = 0;
#pragma unroll
        for (uint32_t q = 0; q < N; ++q) v ^= gfmul4_tab(rd(g1[q].x), g1[q].y, g1[q].z, g1[q].w, g2[q].x, g2[q].y);
        return v;
    };
    using I1 = std::integral_constant<uint32_t, 1>; using I2 = std::integral_constant<uint32_t, 2>;
    using I3 = std::integral_constant<uint32_t, 3>; using I4 = std::integral_constant<uint32_t, 4>;
    using I5 = std::integral_constant<uint32_t, 5>; using I6 = std::integral_constant<uint32_t, 6>;
    static_assert(WV_MAX_PIECE - 1 == 6, "xor_n cases");

    uint32_t ht = 0;      // HDPC Horner running value (kept across the pieces of a chunk)
    uint32_t gp = 0;      // byte offset of the current group within the ring
    uint32_t lv = 0;
    uint4 g = grp_at(0);
    while (lv < n_levels) {
        const uint32_t hdr = __builtin_amdgcn_readfirstlane(g.x);
        const uint32_t ty = hdr & 7u, n = hdr >> 16;
        if (ty == OP_END) {
            gp = (hdr & FLAG_ADVANCE) ? advance() : gp + GB;
            g = grp_at(gp);
            if (hdr & FLAG_BARRIER) {
                unsigned long long t_w = 0;
                if (stamping) t_w = __builtin_amdgcn_s_memtime();
                // level barrier: LDS traffic complete (lgkmcnt); the page load stays in flight
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (stamping) {
                    const unsigned long long t_b = __builtin_amdgcn_s_memtime();
                    a.stamp[(lv * NW + wave) * 2] = t_w - t_lv;
                    a.stamp[(lv * NW + wave) * 2 + 1] = t_b - t_w;
                    t_lv = t_b;
                }
                ++lv;
            }
            continue;
        }
        if (ty == OP_HORNER) {
            // One HDPC chunk piece on the whole wave (row indices are scalars): t = alpha*t ^ y;
            // partial[a] ^= t; partial[b] ^= t.  Between pieces of a chunk the partials wait in
            // their destination rows and t in a register.
            uint32_t hp[16];
            const uint32_t H = a.p.H;
            const uint32_t base = wr_addr(g.y), pstride = live ? sd * 4 : 0u;
            if (hdr & FLAG_HSTART) {
                ht = 0;
#pragma unroll
                for (int h = 0; h < 16; ++h) hp[h] = 0;
            } else {
#pragma unroll
                for (uint32_t h = 0; h < 16; ++h) hp[h] = h < H ? rd(g.y + h * sd * 4) : 0u;
            }
            const uint32_t pay = gp + GB;
            for (uint32_t q = 0; q < n; ++q) {
                const uint4 gc = grp_at(pay + q * GB);
                uint32_t e[8], y[8];
                e[0] = __builtin_amdgcn_readfirstlane(gc.x); e[1] = __builtin_amdgcn_readfirstlane(gc.y);
                e[2] = __builtin_amdgcn_readfirstlane(gc.z); e[3] = __builtin_amdgcn_readfirstlane(gc.w);
                e[4] = __builtin_amdgcn_readlane(gc.x, 32); e[5] = __builtin_amdgcn_readlane(gc.y, 32);
                e[6] = __builtin_amdgcn_readlane(gc.z, 32); e[7] = __builtin_amdgcn_readlane(gc.w, 32);
#pragma unroll
                for (int j = 0; j < 8; ++j) y[j] = rd(e[j] & 0x3FFFFu);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    ht = xtime4p(ht) ^ y[j];
                    hp[(e[j] >> 18) & 15u] ^= ht;
                    hp[(e[j] >> 22) & 15u] ^= ht;
                }
            }
            const bool fin = (hdr & FLAG_HFINISH) != 0;
            uint32_t tw[4] = {0, 0, 0, 0};
            if (fin) {
                const uint4 gt = grp_at(pay + n * GB);
                tw[0] = __builtin_amdgcn_readfirstlane(gt.x); tw[1] = __builtin_amdgcn_readfirstlane(gt.y);
                tw[2] = __builtin_amdgcn_readfirstlane(gt.z); tw[3] = __builtin_amdgcn_readfirstlane(gt.w);
            }
#pragma unroll
            for (uint32_t h = 0; h < 16; ++h)
                if (h < H) wr(base + h * pstride, fin ? hp[h] ^ gfmul4(ht, (tw[h >> 2] >> (8 * (h & 3))) & 0xFFu) : hp[h]);
            gp = pay + (n + (fin ? 1u : 0u)) * GB;
            g = grp_at(gp);
            continue;
        }
        const uint32_t npos = gp + (n + 1u) * GB;
        const uint4 gn = grp_at(npos);  // next op's header group, in flight during this op
        const uint32_t pay = gp + GB;
        uint32_t v = 0;
        if (hdr & FLAG_G) v = gload(g.z);
        if (ty == OP_XOR) {
            switch (n) {
                case 1: v ^= xor_n(I1{}, pay); break;
                case 2: v ^= xor_n(I2{}, pay); break;
                case 3: v ^= xor_n(I3{}, pay); break;
                case 4: v ^= xor_n(I4{}, pay); break;
                case 5: v ^= xor_n(I5{}, pay); break;
                default: v ^= xor_n(I6{}, pay); break;
            }
        } else {  // OP_MUL
            switch (n) {
                case 2: v ^= mul_n(I1{}, pay); break;
                case 4: v ^= mul_n(I2{}, pay); break;
                default: v ^= mul_n(I3{}, pay); break;
            }
        }
        wr(wr_addr(g.y), v);
        gp = npos;
        g = gn;
    }
    // no ring refill outlives the program: the ring becomes the tuple staging area
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // ---- outputs: repair symbols (encodeGen, RQ/params.go:162-182) or syndromes (decode) ----
    if (a.out && !(a.dbg & 4u)) {
        uint32_t o0 = 0, o1 = a.n_out;
        if (a.out_off) { o0 = a.out_off[b]; o1 = a.out_off[b + 1]; }
        const DevParams p = a.p;
        for (uint32_t ob = o0; ob < o1; ob += OUT_BATCH) {
            const uint32_t on = min(OUT_BATCH, o1 - ob);
            if (tid < on) {  // one thread per output: the tuple of its ISI
                const uint32_t esi = a.out_esi[ob + tid];
                uint32_t* t6 = tup + tid * 6;
                if (esi < K) {
                    t6[0] = 0xFFFFFFFFu; t6[1] = esi;
                } else {
                    const uint32_t X = esi + p.Kp - K;
                    uint32_t A = 53591u + 997u * p.J;
                    if ((A & 1u) == 0) ++A;
                    const uint32_t y = 10267u * (p.J + 1u) + X * A;
                    t6[0] = d_degree(d_rand(y, 0, 1u << 20), p.W);
                    t6[1] = 1 + d_rand(y, 1, p.W - 1);
                    t6[2] = d_rand(y, 2, p.W);
                    t6[3] = t6[0] < 4 ? 2 + d_rand(X, 3, 2) : 2;
                    t6[4] = 1 + d_rand(X, 4, p.P1 - 1);
                    t6[5] = d_rand(X, 5, p.P1);
                }
            }
            __syncthreads();
            for (uint32_t o = grp; o < on; o += ngrp) {
                const uint32_t* t6 = tup + o * 6;
                uint32_t v = 0;
                if (t6[0] == 0xFFFFFFFFu) {
                    v = gload(t6[1]);
                } else {
                    const uint32_t d = t6[0], aa = t6[1], d1 = t6[3], a1 = t6[4];
                    uint32_t bb = t6[2], b1 = t6[5];
                    v = lds[__umul24((uint32_t)a.col_slot[bb], sd) + hlc];
                    for (uint32_t j = 1; j < d; ++j) {
                        bb += aa; if (bb >= p.W) bb -= p.W;
                        v ^= lds[__umul24((uint32_t)a.col_slot[bb], sd) + hlc];
                    }
                    while (b1 >= p.P) { b1 += a1; if (b1 >= p.P1) b1 -= p.P1; }
                    v ^= lds[__umul24((uint32_t)a.col_slot[p.W + b1], sd) + hlc];
                    for (uint32_t j = 1; j < d1; ++j) {
                        b1 += a1; if (b1 >= p.P1) b1 -= p.P1;
                        while (b1 >= p.P) { b1 += a1; if (b1 >= p.P1) b1 -= p.P1; }
                        v ^= lds[__umul24((uint32_t)a.col_slot[p.W + b1], sd) + hlc];
                    }
                }
                const uint32_t og = ob + o;
                const size_t off = a.out_off ? (size_t)og * T : (size_t)b * a.out_stride + (size_t)(og - o0) * T;
                if (inb) {
                    if (a.xor_in) v ^= *reinterpret_cast<const uint32_t*>(a.xor_in + off + (size_t)(c0 + hl) * 4);
                    *reinterpret_cast<uint32_t*>(a.out + off + (size_t)(c0 + hl) * 4) = v;
                }
            }
            __syncthreads();
        }
    }
    if (a.c_out) {
        for (uint32_t c = grp; c < a.p.L; c += ngrp)
            if (inb)
                *reinterpret_cast<uint32_t*>(a.c_out + (size_t)b * a.c_stride + (size_t)c * T + (size_t)(c0 + hl) * 4) =
                    lds[(uint32_t)a.col_slot[c] * sd + hlc];
    }
}

// ------------------------------ decode: per-block GF(256) solve ------------------------------
// M[j][k] = sum_{c in LT(isi_j)} Ainv[c][e_k] (received repair j, erased source e_k);
// Gauss-Jordan on [M | I]: rank e <=> the reference's system is full rank.
// Output: X (e x e) and the e received repairs it combines: x_k = sum_m X[k][m] sigma_{piv[m]}.
__device__ __forceinline__ uint8_t gmul_t(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[lg[a] + lg[b]] : (uint8_t)0;
}

// LT tuple of ISI X into t6[0..5] = {d, a, b, d1, a1, b1} (RQ/params.go:83-112).
__device__ __forceinline__ void d_tuple6(const DevParams& p, uint32_t X, uint32_t* t6) {
    uint32_t A = 53591u + 997u * p.J;
    if ((A & 1u) == 0) ++A;
    const uint32_t y = 10267u * (p.J + 1u) + X * A;
    t6[0] = d_degree(d_rand(y, 0, 1u << 20), p.W);
    t6[1] = 1 + d_rand(y, 1, p.W - 1);
    t6[2] = d_rand(y, 2, p.W);
    t6[3] = t6[0] < 4 ? 2 + d_rand(X, 3, 2) : 2;
    t6[4] = 1 + d_rand(X, 4, p.P1 - 1);
    t6[5] = d_rand(X, 5, p.P1);
}
// Calls f(col) for the columns of a staged tuple (modular steps by add/subtract).
template <class F>
__device__ __forceinline__ void d_cols6(const DevParams& p, const uint32_t* t6, F&& f) {
    const uint32_t d = t6[0], aa = t6[1], d1 = t6[3], a1 = t6[4];
    uint32_t bb = t6[2], b1 = t6[5];
    f(bb);
    for (uint32_t j = 1; j < d; ++j) { bb += aa; if (bb >= p.W) bb -= p.W; f(bb); }
    while (b1 >= p.P) { b1 += a1; if (b1 >= p.P1) b1 -= p.P1; }
    f(p.W + b1);
    for (uint32_t j = 1; j < d1; ++j) {
        b1 += a1; if (b1 >= p.P1) b1 -= p.P1;
        while (b1 >= p.P) { b1 += a1; if (b1 >= p.P1) b1 -= p.P1; }
        f(p.W + b1);
    }
}

__global__ void __launch_bounds__(256) k_solve(SolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    __shared__ uint8_t ex[512], lg[256];
    __shared__ uint8_t fac[256];
    __shared__ uint16_t rowid[256];
    __shared__ int piv;
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_off[b + 1] - a.rep_off[b];
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* R = a.rep_esi + a.rep_off[b];
    const uint32_t ws = e + nr;
    uint32_t* tup = reinterpret_cast<uint32_t*>(sm + ((nr * ws + 15) & ~15u));  // nr x 6 words
    if (tid == 0) {
        uint32_t x = 1;
        for (int i = 0; i < 255; ++i) {
            ex[i] = (uint8_t)x; ex[i + 255] = (uint8_t)x; lg[x] = (uint8_t)i;
            x <<= 1; if (x & 0x100) x ^= 0x11D;
        }
        ex[510] = ex[0]; ex[511] = ex[1]; lg[0] = 0;
    }
    for (uint32_t r = tid; r < nr; r += nthr) {
        rowid[r] = (uint16_t)r;
        d_tuple6(a.p, R[r] + a.p.Kp - a.p.K, tup + r * 6);
    }
    for (uint32_t idx = tid; idx < nr * ws; idx += nthr) sm[idx] = 0;
    __syncthreads();
    for (uint32_t idx = tid; idx < nr * e; idx += nthr) {
        const uint32_t j = idx / e, k = idx - j * e;
        const uint32_t col = E[k];
        uint8_t v = 0;
        d_cols6(a.p, tup + j * 6, [&](uint32_t c) { v ^= a.cid[(size_t)c * a.cid_stride + col]; });
        sm[j * ws + k] = v;
    }
    for (uint32_t j = tid; j < nr; j += nthr) sm[j * ws + e + j] = 1;
    __syncthreads();
    for (uint32_t k = 0; k < e; ++k) {
        if (tid == 0) piv = (int)nr;
        __syncthreads();
        for (uint32_t r = k + tid; r < nr; r += nthr)
            if (sm[r * ws + k]) atomicMin(&piv, (int)r);
        __syncthreads();
        const uint32_t p = (uint32_t)piv;
        if (p >= nr) {
            if (tid == 0) a.status[b] = 0;
            return;
        }
        if (p != k) {
            for (uint32_t c = tid; c < ws; c += nthr) {
                const uint8_t t = sm[p * ws + c]; sm[p * ws + c] = sm[k * ws + c]; sm[k * ws + c] = t;
            }
            if (tid == 0) { const uint16_t t = rowid[p]; rowid[p] = rowid[k]; rowid[k] = t; }
            __syncthreads();
        }
        const uint8_t pv = sm[k * ws + k];
        const uint8_t inv = ex[255 - lg[pv]];
        __syncthreads();
        for (uint32_t c = k + tid; c < ws; c += nthr) sm[k * ws + c] = gmul_t(lg, ex, sm[k * ws + c], inv);
        for (uint32_t r = tid; r < nr; r += nthr) fac[r] = (r == k) ? 0 : sm[r * ws + k];
        __syncthreads();
        for (uint32_t idx = tid; idx < nr * (ws - k); idx += nthr) {
            const uint32_t r = idx / (ws - k), c = k + (idx - r * (ws - k));
            const uint8_t f = fac[r];
            if (f) sm[r * ws + c] ^= gmul_t(lg, ex, f, sm[k * ws + c]);
        }
        __syncthreads();
    }
    uint8_t* X = a.xmat + (size_t)blockIdx.x * a.max_e * a.max_e;
    uint16_t* XP = a.xpiv + (size_t)blockIdx.x * a.max_e;
    for (uint32_t m = tid; m < e; m += nthr) XP[m] = rowid[m];
    for (uint32_t idx = tid; idx < e * e; idx += nthr) {
        const uint32_t k = idx / e, m = idx - k * e;
        X[k * e + m] = sm[k * ws + e + rowid[m]];
    }
    if (tid == 0) a.status[b] = 1;
}

// ------------------------------ decode: x_E = X * sigma --------------------------------------
// grid = (strips of 64 dwords, blocks); one wave per erased row at a time, one dword per lane.
__global__ void __launch_bounds__(256) k_apply(ApplyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sg[];
    const uint32_t b = a.blk_map[blockIdx.y];
    if (a.status[b] != 1) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t Td = a.T >> 2, c0 = blockIdx.x * 64, width = min(64u, Td - c0);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint8_t* X = a.xmat + (size_t)blockIdx.y * a.max_e * a.max_e;
    const uint16_t* XP = a.xpiv + (size_t)blockIdx.y * a.max_e;
    uint8_t* xs = reinterpret_cast<uint8_t*>(sg + e * 64);
    for (uint32_t i = tid; i < e * 64; i += blockDim.x) {
        const uint32_t m = i >> 6, c = i & 63;
        sg[i] = (c < width) ? *reinterpret_cast<const uint32_t*>(a.sigma + (size_t)(a.rep_off[b] + XP[m]) * a.T +
                                                                  (size_t)(c0 + c) * 4)
                            : 0u;
    }
    for (uint32_t i = tid; i < e * e; i += blockDim.x) xs[i] = X[i];
    __syncthreads();
    uint8_t* blk = a.data + (size_t)b * a.data_stride;
    for (uint32_t k = wave; k < e; k += nw) {
        uint32_t acc = 0;
        for (uint32_t m = 0; m < e; ++m) {
            const uint32_t c = xs[k * e + m];
            if (c) acc ^= gfmul4(sg[m * 64 + lane], c);
        }
        if (lane < width) *reinterpret_cast<uint32_t*>(blk + (size_t)E[k] * a.T + (size_t)(c0 + lane) * 4) = acc;
    }
}

int launch_solve(const SolveArgs& a, uint32_t n_blocks, uint32_t lds_bytes, void* stream) {
    hipLaunchKernelGGL(k_solve, dim3(n_blocks), dim3(256), lds_bytes, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int launch_apply(const ApplyArgs& a, uint32_t n_strips, uint32_t n_blocks, uint32_t lds_bytes, void* stream) {
    hipLaunchKernelGGL(k_apply, dim3(n_strips, n_blocks), dim3(256), lds_bytes, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

// ------------------------------ gather repairs from a device-resident C ----------------------
// Per-call API: out[r] = XOR of C rows of LT(isi_r) (encodeGen, RQ/params.go:162-182).
__global__ void __launch_bounds__(256) k_gather(DevParams p, const uint8_t* C, uint32_t T, const uint32_t* esi,
                                                uint32_t n, uint8_t* out) {
    const uint32_t r = blockIdx.x;
    if (r >= n) return;
    const uint32_t Td = T >> 2;
    const uint32_t isi = esi[r] + p.Kp - p.K;
    for (uint32_t c = threadIdx.x; c < Td; c += blockDim.x) {
        uint32_t v = 0;
        d_for_cols(p, isi, [&](uint32_t col) { v ^= reinterpret_cast<const uint32_t*>(C + (size_t)col * T)[c]; });
        reinterpret_cast<uint32_t*>(out + (size_t)r * T)[c] = v;
    }
}

// Self-test of the packed GF(256) primitives against host tables (rq_debug_gf_selftest):
// out[i] = xtime4p(x[i]); out[n + c*n + i] = gfmul4_tab(x[i], tables of c).
__global__ void __launch_bounds__(256) k_gf_selftest(const uint32_t* x, uint32_t n, const uint32_t* tabs, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y;
    if (i >= n) return;
    const uint32_t* t = tabs + c * 5;
    if (c == 0) out[i] = xtime4p(x[i]);
    out[n + c * n + i] = gfmul4_tab(x[i], t[0], t[1], t[2], t[3], t[4]);
}
int launch_gf_selftest(const uint32_t* x, uint32_t n, const uint32_t* tabs, uint32_t* out) {
    hipLaunchKernelGGL(k_gf_selftest, dim3((n + 255) / 256, 256), dim3(256), 0, nullptr, x, n, tabs, out);
    return (int)hipGetLastError();
}

int launch_gather(const DevParams& p, const uint8_t* C, uint32_t T, const uint32_t* esi, uint32_t n, uint8_t* out,
                  void* stream) {
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, (hipStream_t)stream, p, C, T, esi, n, out);
    return (int)hipGetLastError();
}

int launch_encode(const EncArgs& a, uint32_t n_strips, uint32_t n_blocks, uint32_t /*group*/, void* stream) {
    const uint32_t nebw = a.erased_off ? (a.p.K + 31) / 32 : 0;
    const size_t img = ((size_t)a.n_slots * a.sd + 3) & ~(size_t)3;
    const size_t rsz = std::max<size_t>((size_t)a.n_waves * 2 * WV_PAGE, OUT_BATCH * 6);
    const size_t lds = (img + rsz + nebw) * 4;
    if ((a.n_waves != 8 && a.n_waves != 16) || a.sd > 32 || lds > 160 * 1024) return (int)hipErrorInvalidValue;
    static bool attr_set = false;  // allow the full 160 KiB of LDS
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_encode<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, 158 * 1024);
        (void)hipFuncSetAttribute((const void*)k_apply, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    const dim3 grid(n_strips, n_blocks);
    const bool erase = a.erased_off != nullptr;
    if (a.n_waves == 16) {
        if (erase) hipLaunchKernelGGL((k_encode<16, true>), grid, dim3(16 * 64), lds, (hipStream_t)stream, a);
        else hipLaunchKernelGGL((k_encode<16, false>), grid, dim3(16 * 64), lds, (hipStream_t)stream, a);
    } else {
        if (erase) hipLaunchKernelGGL((k_encode<8, true>), grid, dim3(8 * 64), lds, (hipStream_t)stream, a);
        else hipLaunchKernelGGL((k_encode<8, false>), grid, dim3(8 * 64), lds, (hipStream_t)stream, a);
    }
    return (int)hipGetLastError();
}

}  // namespace rq
