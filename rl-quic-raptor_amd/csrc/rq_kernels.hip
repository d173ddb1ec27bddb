// rq_kernels.hip -- HIP kernels for gfx950 (CDNA4) around the generated encode code objects:
// the per-block decode solve and apply of the syndrome decoder, and the per-object GenSymbol
// gather.  No MFMA: GF(2)/GF(256) byte arithmetic.
//
// Reference routines replaced (native inventory):
//   Decoder.Decode   RQ/decoder.go:64-134 -> column program (syndromes) + k_solve + k_apply
//   encodeGen        RQ/params.go:162-182 -> k_gather (per-object GenSymbol from device-resident C)
//   asmSSSE3MulAdd   RQ/discmath/optimizations.s:36-78 -> k_apply's bit-sliced GF(256) mul-add
//
// Syndrome decode: with the erased source rows E zeroed, the column program
// yields r0_j = (G_j A^-1 D)(E := 0) for every candidate repair j, so s_j = r_j ^ r0_j =
// sum_k M[j][k] x_k with M[j][k] = mrep[j][E_k] (the same program run once on the identity
// payload).  Rank(M) = |E| <=> the reference's system is full rank, and x_E is unique.
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "rfc6330_tables.h"
#include "rq_device.hpp"

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
// alpha * x per byte: v_perm's sign-replicating selectors turn the four top bits into 0x00/0xFF
// byte masks (selector bytes 0x0a,0x08,0x0b,0x09 read bits 7,15,23,31 of {x<<8 : x}), no multiply.
__device__ __forceinline__ uint32_t xtime4(uint32_t x) {
    const uint32_t mask = __builtin_amdgcn_perm(x << 8, x, 0x090b080au);
    return ((x << 1) & 0xFEFEFEFEu) ^ (mask & 0x1D1D1D1Du);
}

// a ^ (b & m) in one v_bitop3 (src0 a 0xF0, src1 b 0xCC, src2 m 0xAA -> 0x78)
__device__ __forceinline__ uint32_t bitop_xand(uint32_t a, uint32_t b, uint32_t m) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(d) : "v"(a), "v"(b), "v"(m));
    return d;
}

// a ^ b ^ c in one v_bitop3 (hipcc does not form it from three XORs)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// ------------------------------ LT tuple on device (RQ/params.go:83-112) -------------------
__device__ __forceinline__ uint32_t d_rand(uint32_t y, uint32_t i, uint32_t m) {
    return (c_V[0][(y + i) & 255u] ^ c_V[1][((y >> 8) + i) & 255u] ^ c_V[2][((y >> 16) + i) & 255u] ^
            c_V[3][((y >> 24) + i) & 255u]) % m;
}
// Calls f(col) for every column XORed into the symbol of ISI X (encodeGen order).
template <class F>
__device__ __forceinline__ void d_for_cols(const DevParams& p, uint32_t X, F&& f) {
    uint32_t A = 53591u + 997u * p.J;
    if ((A & 1u) == 0) ++A;
    const uint32_t y = 10267u * (p.J + 1u) + X * A;
    const uint32_t v = d_rand(y, 0, 1u << 20);
    uint32_t d = 30;
    for (uint32_t i = 0; i < 31; ++i)
        if (v < c_DEG[i]) { d = i; break; }
    if (d > p.W - 2) d = p.W - 2;
    const uint32_t a = 1 + d_rand(y, 1, p.W - 1);
    uint32_t b = d_rand(y, 2, p.W);
    const uint32_t d1 = d < 4 ? 2 + d_rand(X, 3, 2) : 2;
    const uint32_t a1 = 1 + d_rand(X, 4, p.P1 - 1);
    uint32_t b1 = d_rand(X, 5, p.P1);
    f(b);
    for (uint32_t j = 1; j < d; ++j) { b = (b + a) % p.W; f(b); }
    while (b1 >= p.P) b1 = (b1 + a1) % p.P1;
    f(p.W + b1);
    for (uint32_t j = 1; j < d1; ++j) {
        b1 = (b1 + a1) % p.P1;
        while (b1 >= p.P) b1 = (b1 + a1) % p.P1;
        f(p.W + b1);
    }
}

// ------------------------------ decode: pack the recovered rows ---------------------------
// Recovered row i of the same list -> pack + i*T (dense D2H staging), one wave per row.
__global__ void __launch_bounds__(256) k_pack_rows(PackArgs a) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= a.n) return;
    const uint32_t* r4 = reinterpret_cast<const uint32_t*>(a.data + (size_t)a.blk[i] * a.data_stride + (size_t)a.row[i] * a.T);
    uint32_t* p4 = reinterpret_cast<uint32_t*>(a.pack + (size_t)i * a.T);
    for (uint32_t c = lane; c < a.T / 4; c += 64) p4[c] = r4[c];
}

int launch_pack_rows(const PackArgs& a, void* stream) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_pack_rows, dim3((a.n + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

// ------------------------------ decode: per-block GF(256) solve ------------------------------
// M[j][k] = mrep[uidx_j][e_k] (received repair j, erased source e_k); Gauss-Jordan on [M | I]
// (replaces GaussianElimination, RQ/discmath/gauss.go:7-45, on the e erased columns only):
// rank e <=> the reference's system is full rank.
// Output: X (e x e) and the e received repairs it combines: x_k = sum_m X[k][m] s_{piv[m]}, stored
// as xcoef[m * xc_stride + k] (one uniform 64-byte row per m for k_apply's scalar loads).
__device__ __forceinline__ uint8_t gmul_t(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[lg[a] + lg[b]] : (uint8_t)0;
}

// GF(256) exp/log tables (poly 0x11D, alpha = 2), constant-initialised in device memory and copied
// into LDS by the blocks that need them.
struct alignas(16) GfTabs {
    uint8_t ex[512];
    uint8_t lg[256];
};
constexpr GfTabs make_gf_tabs() {
    GfTabs t{};
    uint32_t x = 1;
    for (int i = 0; i < 255; ++i) {
        t.ex[i] = (uint8_t)x; t.ex[i + 255] = (uint8_t)x; t.lg[x] = (uint8_t)i;
        x <<= 1; if (x & 0x100) x ^= 0x11D;
    }
    t.ex[510] = t.ex[0]; t.ex[511] = t.ex[1];
    return t;
}
__device__ const GfTabs kGf = make_gf_tabs();

__device__ __forceinline__ void gf_tables_copy(uint8_t* ex, uint8_t* lg) {
    // as 192 dwords, one load per thread (no serialised byte-load loop)
    const uint32_t* se = reinterpret_cast<const uint32_t*>(kGf.ex);
    const uint32_t* sl = reinterpret_cast<const uint32_t*>(kGf.lg);
    for (uint32_t i = threadIdx.x; i < 192; i += blockDim.x) {
        if (i < 128) reinterpret_cast<uint32_t*>(ex)[i] = se[i];
        else reinterpret_cast<uint32_t*>(lg)[i - 128] = sl[i - 128];
    }
}

// Row gather of the solvers: wave g copies coefficient bytes k = g, g + NW, ... of one received
// repair (mr[Es[k]], a byte gather from the program's identity-payload outputs) into its LDS row,
// sixteen loads in flight per lane instead of one load-then-store round trip per byte.
template <int NW>
__device__ __forceinline__ void gather_row(uint8_t* myb, const uint8_t* mr, const uint32_t* Es, uint32_t e, uint32_t g) {
    for (uint32_t k0 = g; k0 < e; k0 += 16 * NW) {
        uint8_t v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t k = k0 + NW * u;
            v[u] = k < e ? mr[Es[k]] : (uint8_t)0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t k = k0 + NW * u;
            if (k < e) myb[k] = v[u];
        }
    }
}

// Four waves per block, RPL rows per lane: lane j of every wave holds received repairs j + 64q
// (q < RPL) as LDS rows of 128*RPL bytes: e coefficient bytes, then the identity part (byte e + row);
// wave g updates the 16-byte quads g, g+4, ... of every row.  RPL = 1 takes blocks with e <= 64 on
// their first 64 received repairs; RPL = 2 takes the blocks it deferred (e <= 128, first 128
// repairs).  Each step picks the lowest unused row with a nonzero coefficient (ballot: every wave
// sees all rows and picks the same one), scales it by the inverse and stores its eight alpha^b
// multiples (one byte per thread, exp/log tables), and every other row XORs in the multiples its own
// coefficient's bits select (one v_bitop3 per bit and dword).
template <int RPL, int NW>
__global__ void __launch_bounds__(64 * NW) k_solve_fast(SolveArgs a) {
    constexpr uint32_t NT = 64 * NW;
    constexpr uint32_t NROWS = 64 * RPL, WQ = 8 * RPL, SW = 32 * RPL + 4;  // quads per row, row stride
    __shared__ __attribute__((aligned(16))) uint32_t rows[NROWS * SW];
    __shared__ __attribute__((aligned(16))) uint4 mult[8][WQ];  // alpha^b * scaled pivot row
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[NROWS];
    __shared__ uint32_t Es[NROWS];
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    if (RPL > 1 && a.status[b] != ST_FALLBACK) return;  // the wide pass takes deferred blocks only
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > NROWS) {
        if (tid == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = min(nr, NROWS);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    for (uint32_t i = tid; i < e; i += NT) Es[i] = E[i];
    gf_tables_copy(ex, lg);
    for (uint32_t i = tid; i < NROWS * SW; i += NT) rows[i] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const uint32_t row = lane + 64 * q;
        if (row < nrow) {  // row gather: wave g takes columns g, g+4, ...
            uint8_t* myb = reinterpret_cast<uint8_t*>(rows + row * SW);
            const uint8_t* mr = a.mrep + (size_t)U[row] * a.mrep_stride;
            gather_row<NW>(myb, mr, Es, e, g);
            if (g == 0) myb[e + row] = 1;
        }
    }
    __syncthreads();
    const uint32_t q1 = (e + nrow + 15) >> 4;  // quads holding live columns
    bool used[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) used[q] = lane + 64 * q >= nrow;
    uint8_t* mb = reinterpret_cast<uint8_t*>(mult);
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    for (uint32_t k = 0; k < e; ++k) {
        uint32_t f[RPL];
        uint32_t p = 0xFFFFFFFFu;
#pragma unroll
        for (int q = RPL - 1; q >= 0; --q) {
            f[q] = (rows[(lane + 64 * q) * SW + (k >> 2)] >> ((k & 3) * 8)) & 0xFFu;
            const uint64_t bal = __ballot(f[q] != 0 && !used[q]);
            if (bal) p = 64 * q + (uint32_t)__ffsll((unsigned long long)bal) - 1;
        }
        if (p == 0xFFFFFFFFu) {  // uniform over the block: every wave saw the same rows
            if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + 64 * q == p) used[q] = true;
        if (tid == 0) pivl[k] = (uint8_t)p;
        // scaled pivot row and its alpha multiples: alpha^bt * x / x_k = exp(log x - log x_k + bt)
        const uint32_t lginv = 255u - lg[rb[p * SW * 4 + k]];
        for (uint32_t pos = tid; pos < 128 * RPL; pos += NT) {
            const uint32_t x = rb[p * SW * 4 + pos];
            uint32_t t = lg[x] + lginv;
            t = t >= 255u ? t - 255u : t;
#pragma unroll
            for (int bt = 0; bt < 8; ++bt) mb[bt * WQ * 16 + pos] = x ? ex[t + bt] : (uint8_t)0;
        }
        __syncthreads();
        // columns < k are zero in the pivot row (all are earlier pivot columns): start at quad k/16
        const uint32_t q0 = k >> 4;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            uint4* my4 = reinterpret_cast<uint4*>(rows + (lane + 64 * q) * SW);
            if (lane + 64 * q == p) {
                for (uint32_t w = q0 + g; w < q1; w += NW) my4[w] = mult[0][w];
            } else if (f[q]) {
                uint32_t msk[8];
#pragma unroll
                for (int bt = 0; bt < 8; ++bt) msk[bt] = 0u - ((f[q] >> bt) & 1u);
                for (uint32_t w = q0 + g; w < q1; w += NW) {
                    uint4 r = my4[w];
#pragma unroll
                    for (int bt = 0; bt < 8; ++bt) {
                        const uint4 m = mult[bt][w];
                        r.x = bitop_xand(r.x, m.x, msk[bt]);
                        r.y = bitop_xand(r.y, m.y, msk[bt]);
                        r.z = bitop_xand(r.z, m.z, msk[bt]);
                        r.w = bitop_xand(r.w, m.w, msk[bt]);
                    }
                    my4[w] = r;
                }
            }
        }
        __syncthreads();
    }
    // X[k][m] = identity byte (e + piv_m) of pivot row piv_k
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    for (uint32_t idx = tid; idx < e * e; idx += NT) {
        const uint32_t m = idx / e, k = idx - m * e;
        xc[m * xs + k] = rb[pivl[k] * SW * 4 + e + pivl[m]];
    }
    if (tid == 0) a.status[b] = 1;
}

// The five v_perm tables of a coefficient c (byte lanes): c*{0..3}, c*{4..7}, c*{0,8,16,24},
// c*{32,40,48,56}, c*{0,64,128,192}, from the eight alpha^i multiples of c.
__device__ __forceinline__ uint8_t xtime1(uint32_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80u) ? 0x1Du : 0u)); }

__device__ __forceinline__ void perm_tables(uint32_t c, uint4* A, uint32_t* B) {
    uint32_t m[8];
    m[0] = c;
#pragma unroll
    for (int i = 1; i < 8; ++i) m[i] = xtime1(m[i - 1]);
    auto lo = [&](uint32_t x) { return ((x & 1u) ? m[0] : 0u) ^ ((x & 2u) ? m[1] : 0u) ^ ((x & 4u) ? m[2] : 0u); };
    auto pack = [](uint32_t a, uint32_t b, uint32_t c2, uint32_t d) { return a | (b << 8) | (c2 << 16) | (d << 24); };
    A->x = pack(0, lo(1), lo(2), lo(3));
    A->y = pack(lo(4), lo(5), lo(6), lo(7));
    A->z = pack(0, m[3], m[4], m[3] ^ m[4]);
    A->w = pack(m[5], m[5] ^ m[3], m[5] ^ m[4], m[5] ^ m[4] ^ m[3]);
    *B = pack(0, m[6], m[7], m[6] ^ m[7]);
}

// perm_tables of every nonzero coefficient alpha^l (l < 255), constant-initialised in device memory:
// the solvers copy them into LDS (five dword loads per entry) instead of building 255 table sets per
// block (~70 VALU each).
struct alignas(16) PermTabs {
    uint32_t A[255][4];
    uint32_t B[255];
};
constexpr PermTabs make_perm_tabs() {
    PermTabs t{};
    const GfTabs g = make_gf_tabs();
    for (int l = 0; l < 255; ++l) {
        uint32_t m[8] = {g.ex[l], 0, 0, 0, 0, 0, 0, 0};
        for (int i = 1; i < 8; ++i) m[i] = ((m[i - 1] << 1) ^ ((m[i - 1] & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
        auto lo = [&](uint32_t x) { return ((x & 1u) ? m[0] : 0u) ^ ((x & 2u) ? m[1] : 0u) ^ ((x & 4u) ? m[2] : 0u); };
        auto pack = [](uint32_t a, uint32_t b, uint32_t c2, uint32_t d) { return a | (b << 8) | (c2 << 16) | (d << 24); };
        t.A[l][0] = pack(0, lo(1), lo(2), lo(3));
        t.A[l][1] = pack(lo(4), lo(5), lo(6), lo(7));
        t.A[l][2] = pack(0, m[3], m[4], m[3] ^ m[4]);
        t.A[l][3] = pack(m[5], m[5] ^ m[3], m[5] ^ m[4], m[5] ^ m[4] ^ m[3]);
        t.B[l] = pack(0, m[6], m[7], m[6] ^ m[7]);
    }
    return t;
}
__device__ const PermTabs kPerm = make_perm_tabs();

// c * x on four bytes with c's perm_tables: three v_perm lookups (3 + 3 + 2 bits of each byte).
__device__ __forceinline__ uint32_t perm_mul(const uint4& A, uint32_t B, uint32_t x) {
    const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
    return xor3(__builtin_amdgcn_perm(A.y, A.x, s0), __builtin_amdgcn_perm(A.w, A.z, s1),
                __builtin_amdgcn_perm(B, B, s2));
}

// k_solve_fast's layout (four waves, RPL rows per lane as LDS rows, wave g on the quads g, g+4, ...)
// with the elimination done by GF(256) multiplication instead of alpha-multiple tables: each lane
// turns its coefficient c_j = f_j / f_p into v_perm tables (perm_tables) and folds c_j times the
// pivot row into its row, the pivot row's dwords read once per quad (one broadcast b128) and made
// scalar, so the lookups' selectors are SGPRs.  The pivot lane uses c = 1 ^ 1/f_p, which leaves
// row_p / f_p (each wave reads the pivot quad before its pivot lane rewrites it).  One barrier per
// step (the alpha-multiple tables, their byte stores and the second barrier are gone) and an eighth
// of the LDS reads.
template <int RPL, int NW, bool LUT>
__global__ void __launch_bounds__(64 * NW) k_solve_pm(SolveArgs a) {
    constexpr uint32_t NT = 64 * NW;
    constexpr uint32_t NROWS = 64 * RPL, SW = 32 * RPL + 4;  // rows, row stride (dwords)
    __shared__ __attribute__((aligned(16))) uint32_t rows[NROWS * SW];
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[NROWS];
    __shared__ uint32_t Es[NROWS];
    // LUT: the v_perm tables of every nonzero coefficient, indexed by its log (built once per block)
    __shared__ __attribute__((aligned(16))) uint4 tlA[LUT ? 255 : 1];
    __shared__ uint32_t tlB[LUT ? 255 : 1];
    // LUT: per pivot value f (!= 0), log f | log(1 ^ 1/f) << 8 | (1 ^ 1/f != 0) << 16: one lookup per
    // step instead of three dependent ones (lg[f_p], ex[255 - lg f_p], lg[c_p])
    __shared__ uint32_t pinfo[LUT ? 256 : 1];
    __shared__ uint8_t fcol[2][NROWS];  // column k of every row by step parity (see k_solve_pq)
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    if (a.status_init)  // the host-decided statuses (disjoint from the solver's blocks, ST_PENDING)
        for (uint32_t i = blockIdx.x * NT + tid; i < a.n_all; i += gridDim.x * NT)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
    if (RPL > 1 && a.status[b] != ST_FALLBACK) return;  // the wide pass takes deferred blocks only
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > NROWS) {
        if (tid == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = (RPL == 1 && a.row_margin) ? min(min(nr, NROWS), e + a.row_margin) : min(nr, NROWS);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    for (uint32_t i = tid; i < e; i += NT) Es[i] = E[i];
    gf_tables_copy(ex, lg);
    if (LUT)
        for (uint32_t l = tid; l < 255; l += NT) perm_tables(kGf.ex[l], &tlA[l], &tlB[l]);
    for (uint32_t i = tid; i < NROWS * SW; i += NT) rows[i] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const uint32_t row = lane + 64 * q;
        if (row < nrow) {  // row gather: wave g takes columns g, g+4, ...
            uint8_t* myb = reinterpret_cast<uint8_t*>(rows + row * SW);
            const uint8_t* mr = a.mrep + (size_t)U[row] * a.mrep_stride;
            gather_row<NW>(myb, mr, Es, e, g);
            if (g == 0) myb[e + row] = 1;
        }
    }
    if (LUT)
        for (uint32_t x = 1 + tid; x < 256; x += NT) {
            const uint32_t lx = lg[x], cp = 1u ^ ex[255u - lx];
            pinfo[x] = lx | (cp ? (uint32_t)lg[cp] << 8 | 1u << 16 : 0u);
        }
    __syncthreads();
    for (uint32_t r = tid; r < NROWS; r += NT) fcol[0][r] = (uint8_t)(rows[r * SW] & 0xFFu);
    __syncthreads();
    const uint32_t q1 = (e + nrow + 15) >> 4;  // quads holding live columns
    bool used[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) used[q] = lane + 64 * q >= nrow;
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    for (uint32_t k = 0; k < e; ++k) {
        uint32_t f[RPL];
        uint32_t p = 0xFFFFFFFFu;
#pragma unroll
        for (int q = RPL - 1; q >= 0; --q) {
            f[q] = fcol[k & 1][lane + 64 * q];
            const uint64_t bal = __ballot(f[q] != 0 && !used[q]);
            if (bal) p = 64 * q + (uint32_t)__ffsll((unsigned long long)bal) - 1;
        }
        if (p == 0xFFFFFFFFu) {  // uniform over the block: every wave saw the same rows
            if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + 64 * q == p) used[q] = true;
        if (tid == 0) pivl[k] = (uint8_t)p;
        // f_p from the pivot lane's register (no LDS round trip); lg[f] issued beside lg[f_p]
        uint32_t fp = 0;
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if ((p >> 6) == (uint32_t)q) fp = __builtin_amdgcn_readlane(f[q], p & 63);
        uint4 A[RPL];
        uint32_t B[RPL];
        bool act[RPL];
        if (LUT) {
            const uint32_t pi = pinfo[fp];
            const uint32_t lgp = pi & 0xFFu, lcp = (pi >> 8) & 0xFFu;  // the pivot lane's coefficient 1 ^ 1/f_p
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                uint32_t l = 0;
                if (lane + 64 * q == p) {
                    act[q] = (pi >> 16) != 0;
                    l = lcp;
                } else {
                    act[q] = f[q] != 0;
                    l = lg[f[q]] + 255u - lgp;
                    l = l >= 255u ? l - 255u : l;
                }
                A[q] = tlA[act[q] ? l : 0];
                B[q] = tlB[act[q] ? l : 0];
            }
        } else {
            const uint32_t lgp = lg[fp];
            const uint32_t inv = ex[255u - lgp];
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                uint32_t c = 0;
                if (lane + 64 * q == p) {
                    c = 1u ^ inv;
                } else if (f[q]) {
                    uint32_t t = lg[f[q]] + 255u - lgp;
                    t = t >= 255u ? t - 255u : t;
                    c = ex[t];
                }
                act[q] = c != 0;
                perm_tables(c, &A[q], &B[q]);
            }
        }
        // columns < k are zero in the pivot row (all are earlier pivot columns): start at quad k/16
        const uint4* prow = reinterpret_cast<const uint4*>(rows + p * SW);
        const uint32_t kn = k + 1;
        for (uint32_t w = (k >> 4) + g; w < q1; w += NW) {
            const uint4 P = prow[w];
            const uint32_t px = __builtin_amdgcn_readfirstlane(P.x), py = __builtin_amdgcn_readfirstlane(P.y);
            const uint32_t pz = __builtin_amdgcn_readfirstlane(P.z), pw = __builtin_amdgcn_readfirstlane(P.w);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                uint4* my4 = reinterpret_cast<uint4*>(rows + (lane + 64 * q) * SW);
                uint4 r = my4[w];
                if (act[q]) {
                    r.x ^= perm_mul(A[q], B[q], px);
                    r.y ^= perm_mul(A[q], B[q], py);
                    r.z ^= perm_mul(A[q], B[q], pz);
                    r.w ^= perm_mul(A[q], B[q], pw);
                    my4[w] = r;
                }
                if (kn < e && w == (kn >> 4)) {  // wave-uniform: this wave owns column k + 1
                    const uint32_t d = (kn >> 2) & 3u;
                    const uint32_t dw = d == 0 ? r.x : d == 1 ? r.y : d == 2 ? r.z : r.w;
                    fcol[kn & 1][lane + 64 * q] = (uint8_t)(dw >> ((kn & 3u) * 8));
                }
            }
        }
        __syncthreads();
    }
    // X[k][m] = identity byte (e + piv_m) of pivot row piv_k
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    for (uint32_t idx = tid; idx < e * e; idx += NT) {
        const uint32_t m = idx / e, k = idx - m * e;
        xc[m * xs + k] = rb[pivl[k] * SW * 4 + e + pivl[m]];
    }
    if (tid == 0) a.status[b] = 1;
}

// k_solve_pm (LUT) with a shorter dependent chain per pivot step: each wave issues the loads of its
// row quads for the step (at most QW per row) at the step's start, reads pinfo[f] of its own
// coefficient (log f, and the pivot-lane coefficient's log) instead of lg[f] after pinfo[f_p] (f_p's
// log is then a v_readlane of the pivot lane's entry), and loads all its pivot-row quads at once: a
// step is three dependent LDS round trips (f, pinfo[f], the tables) plus the barrier, where the
// quad-at-a-time loop had two more per quad.
// PF (experiments, RQHIP_SOLVE_PF=1): the column buffer carries each row's pinfo word instead of its
// coefficient byte, looked up by the wave that writes it while it updates its other quads, so a step
// starts one dependent LDS round trip later in its chain.
template <int RPL, int NW, bool PF = false>
__global__ void __launch_bounds__(64 * NW) k_solve_pq(SolveArgs a) {
    constexpr uint32_t NT = 64 * NW;
    constexpr uint32_t NROWS = 64 * RPL, SW = 32 * RPL + 4;  // rows, row stride (dwords)
    constexpr uint32_t QW = (8 * RPL + NW - 1) / NW;          // quads per row a wave may update
    __shared__ __attribute__((aligned(16))) uint32_t rows[NROWS * SW];
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[NROWS];
    __shared__ uint32_t Es[NROWS];
    // tables by log, twice over (entry l + 255 = entry l), so that log f - log f_p + 255 needs no mod
    __shared__ __attribute__((aligned(16))) uint4 tlA[510];
    __shared__ uint32_t tlB[510];
    __shared__ uint32_t pinfo[256];
    // column k of every row, double-buffered by step parity: step k reads fcol[k & 1]; the wave that
    // updates the quad holding column k + 1 writes fcol[(k + 1) & 1] from its registers.  Reading
    // column k from `rows` instead would race with wave 0, which rewrites quad k / 16 in the same step
    // (a late wave then sees column k already eliminated: a wrong X with status 1).
    using FC = typename std::conditional<PF, uint32_t, uint8_t>::type;
    __shared__ FC fcol[2][NROWS];
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    if (a.status_init)
        for (uint32_t i = blockIdx.x * NT + tid; i < a.n_all; i += gridDim.x * NT)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
    if (RPL > 1 && a.status[b] != ST_FALLBACK) return;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > NROWS) {
        if (tid == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = (RPL == 1 && a.row_margin) ? min(min(nr, NROWS), e + a.row_margin) : min(nr, NROWS);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    for (uint32_t i = tid; i < e; i += NT) Es[i] = E[i];
    gf_tables_copy(ex, lg);
    for (uint32_t l = tid; l < 510; l += NT) {
        const uint32_t lm = l < 255 ? l : l - 255;
        tlA[l] = make_uint4(kPerm.A[lm][0], kPerm.A[lm][1], kPerm.A[lm][2], kPerm.A[lm][3]);
        tlB[l] = kPerm.B[lm];
    }
    for (uint32_t i = tid; i < NROWS * SW; i += NT) rows[i] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const uint32_t row = lane + 64 * q;
        if (row < nrow) {
            uint8_t* myb = reinterpret_cast<uint8_t*>(rows + row * SW);
            const uint8_t* mr = a.mrep + (size_t)U[row] * a.mrep_stride;
            gather_row<NW>(myb, mr, Es, e, g);
            if (g == 0) myb[e + row] = 1;
        }
    }
    // pinfo[f] = log f | log(1 ^ 1/f) << 8 | (1 ^ 1/f != 0) << 16 [| (f != 0) << 17 with PF]; pinfo[0] = 0
    for (uint32_t x = tid; x < 256; x += NT) {
        uint32_t v = 0;
        if (x) {
            const uint32_t lx = lg[x], cp = 1u ^ ex[255u - lx];
            v = lx | (cp ? (uint32_t)lg[cp] << 8 | 1u << 16 : 0u) | (PF ? 1u << 17 : 0u);
        }
        pinfo[x] = v;
    }
    __syncthreads();
    for (uint32_t r = tid; r < NROWS; r += NT) {
        const uint32_t f0 = rows[r * SW] & 0xFFu;
        fcol[0][r] = PF ? (FC)pinfo[f0] : (FC)f0;
    }
    __syncthreads();
    const uint32_t q1 = (e + nrow + 15) >> 4;  // quads holding live columns
    bool used[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) used[q] = lane + 64 * q >= nrow;
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    const uint32_t ksteps = a.diag_steps ? min(e, a.diag_steps) : e;
    for (uint32_t k = 0; k < ksteps; ++k) {
        // (1) this wave's row quads for the step and every row's coefficient in column k
        const uint32_t w0 = (k >> 4) + g;
        // quads past q1 are loaded from a clamped (valid, unused) position: unconditional loads keep
        // the compiler from carrying the arrays across iterations in register copies
        uint4 R[RPL][QW];
#pragma unroll
        for (int j = 0; j < (int)QW; ++j)
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                R[q][j] = reinterpret_cast<const uint4*>(rows + (lane + 64 * q) * SW)[min(w0 + NW * j, 8u * RPL)];
        uint32_t f[RPL], pif[RPL];
        if constexpr (PF) {  // nonzero-ness from the pinfo word (bit 17)
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                pif[q] = fcol[k & 1][lane + 64 * q];
                f[q] = (pif[q] >> 17) & 1u;
            }
        } else {
#pragma unroll
            for (int q = 0; q < RPL; ++q) f[q] = fcol[k & 1][lane + 64 * q];
            // (2) pinfo of every row's coefficient, beside the ballot
#pragma unroll
            for (int q = 0; q < RPL; ++q) pif[q] = pinfo[f[q]];
        }
        uint32_t p = 0xFFFFFFFFu;
#pragma unroll
        for (int q = RPL - 1; q >= 0; --q) {
            const uint64_t bal = __ballot(f[q] != 0 && !used[q]);
            if (bal) p = 64 * q + (uint32_t)__ffsll((unsigned long long)bal) - 1;
        }
        if (p == 0xFFFFFFFFu) {  // uniform over the block: every wave saw the same rows
            if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (lane + 64 * q == p) used[q] = true;
        if (tid == 0) pivl[k] = (uint8_t)p;
        uint4 P[QW];
        const uint4* prow = reinterpret_cast<const uint4*>(rows + p * SW);
#pragma unroll
        for (int j = 0; j < (int)QW; ++j) P[j] = prow[min(w0 + NW * j, 8u * RPL)];
        uint32_t pip = 0;
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if ((p >> 6) == (uint32_t)q) pip = __builtin_amdgcn_readlane(pif[q], p & 63);
        const uint32_t ilgp = 255u - (pip & 0xFFu);  // log(1 / f_p) + 255 - 255, uniform
        // (3) the tables of c = f / f_p (the pivot lane: 1 ^ 1/f_p, which leaves row_p / f_p)
        uint4 A[RPL];
        uint32_t B[RPL];
        bool act[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const bool piv = lane + 64 * q == p;
            act[q] = piv ? ((pif[q] >> 16) & 1u) != 0 : f[q] != 0;
            const uint32_t l = piv ? (pif[q] >> 8) & 0xFFu : (pif[q] & 0xFFu) + ilgp;  // < 510
            A[q] = tlA[l];
            B[q] = tlB[l];
        }
        // columns < k are zero in the pivot row (all are earlier pivot columns): quads from k/16
        const uint32_t kn = k + 1;  // the column the next step reads
#pragma unroll
        for (int j = 0; j < (int)QW; ++j) {
            const uint32_t w = w0 + NW * j;
            if (w >= q1) break;
            const uint32_t px = __builtin_amdgcn_readfirstlane(P[j].x), py = __builtin_amdgcn_readfirstlane(P[j].y);
            const uint32_t pz = __builtin_amdgcn_readfirstlane(P[j].z), pw = __builtin_amdgcn_readfirstlane(P[j].w);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                uint4 r = R[q][j];
                r.x ^= perm_mul(A[q], B[q], px);
                r.y ^= perm_mul(A[q], B[q], py);
                r.z ^= perm_mul(A[q], B[q], pz);
                r.w ^= perm_mul(A[q], B[q], pw);
                if (act[q]) reinterpret_cast<uint4*>(rows + (lane + 64 * q) * SW)[w] = r;
                if (kn < ksteps && w == (kn >> 4)) {  // wave-uniform: this wave owns column k + 1
                    const uint4 v = act[q] ? r : R[q][j];
                    const uint32_t d = (kn >> 2) & 3u;
                    const uint32_t dw = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
                    const uint32_t fb = (dw >> ((kn & 3u) * 8)) & 0xFFu;
                    fcol[kn & 1][lane + 64 * q] = PF ? (FC)pinfo[fb] : (FC)fb;
                }
            }
        }
        __syncthreads();
    }
    if (ksteps < e) {  // diagnostic step limit (timing only): valid pivot rows, meaningless X
        __syncthreads();
        for (uint32_t m = ksteps + tid; m < e; m += NT) pivl[m] = (uint8_t)m;
        __syncthreads();
    }
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    for (uint32_t m = g; m < e; m += NW) {  // wave g writes rows m = g, g + NW, ... (no index division)
        const uint32_t pm = pivl[m];
        for (uint32_t k = lane; k < e; k += 64) xc[m * xs + k] = rb[pivl[k] * SW * 4 + e + pm];
    }
    if (tid == 0) a.status[b] = 1;
}

// One wave per block for e <= 64 on the first <= 64 received repairs, the rows held in registers:
// lane j owns received repair j as 32 dwords (e coefficient bytes, then the identity part at byte
// e + j).  Each step k takes the lowest unused row with a nonzero coefficient in column k (ballot),
// and every lane folds the pivot row (read dword by dword with v_readlane: uniform, so the v_perm
// selectors are scalar) scaled by its own coefficient c_j = f_j / f_p into its row -- one GF(256)
// multiply per dword as three v_perm lookups against per-lane tables of c_j (perm_tables).  The
// pivot lane uses c = 1 ^ 1/f_p, which leaves row_p / f_p.  No barrier inside the elimination.
__global__ void __launch_bounds__(64) k_solve_reg(SolveArgs a) {
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[64];
    __shared__ uint32_t rows[64 * 33];  // final rows, stride 33 dwords (no bank conflicts)
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t lane = threadIdx.x;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > 64) {
        if (lane == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = min(nr, 64u);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    gf_tables_copy(ex, lg);
    uint32_t row[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) row[w] = 0;
    if (lane < nrow) {
        const uint8_t* mr = a.mrep + (size_t)U[lane] * a.mrep_stride;
#pragma unroll
        for (int w = 0; w < 16; ++w)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if ((uint32_t)(4 * w + i) < e) row[w] |= (uint32_t)mr[E[4 * w + i]] << (8 * i);
        const uint32_t pos = e + lane;
#pragma unroll
        for (int w = 0; w < 32; ++w)
            if ((pos >> 2) == (uint32_t)w) row[w] |= 1u << (8 * (pos & 3));
    }
    bool used = lane >= nrow;
    const uint32_t q1 = (e + nrow + 3) >> 2;  // live dwords
    __syncthreads();                          // GF tables
    for (uint32_t k = 0; k < e; ++k) {
        const uint32_t W = k >> 2;
        uint32_t rw = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w)
            if ((uint32_t)w == W) rw = row[w];
        const uint32_t f = (rw >> (8 * (k & 3))) & 0xFFu;
        const uint64_t bal = __ballot(f != 0 && !used);
        if (bal == 0) {  // rank-deficient on these rows (uniform)
            if (lane == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
        const uint32_t p = (uint32_t)__ffsll((unsigned long long)bal) - 1;
        const bool me = lane == p;
        used |= me;
        const uint32_t fp = (uint32_t)__builtin_amdgcn_readlane((int)f, (int)p);
        const uint32_t lginv = 255u - lg[fp];
        uint32_t c = f ? ex[lg[f] + lginv] : 0u;
        if (me) c = ex[lginv] ^ 1u;
        uint4 A;
        uint32_t B;
        perm_tables(c, &A, &B);
#pragma unroll
        for (int w = 0; w < 32; ++w) {
            if ((uint32_t)w >= W && (uint32_t)w < q1) {
                const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)row[w], (int)p);
                row[w] ^= perm_mul(A, B, x);
            }
        }
        if (lane == 0) pivl[k] = (uint8_t)p;
    }
#pragma unroll
    for (int w = 0; w < 32; ++w) rows[lane * 33 + w] = row[w];
    __syncthreads();
    // X[k][m] = identity byte (e + piv_m) of pivot row piv_k
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = lane; m < e; m += 64) XP[m] = pivl[m];
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    for (uint32_t idx = lane; idx < e * e; idx += 64) {
        const uint32_t m = idx / e, k = idx - m * e;
        xc[m * xs + k] = rb[pivl[k] * 132 + e + pivl[m]];
    }
    if (lane == 0) a.status[b] = 1;
}

// One wave per block, rows in registers, for e <= 64 on the first e + margin (<= 64) received
// repairs: a lean first-pass solver (RQHIP_SOLVE_LEAN=1 in experiments builds).  Lane j owns received
// repair j as 32 dwords (e coefficient bytes, then the identity part at byte e + j).  Each step k takes
// the lowest unused row with a nonzero coefficient in column k (ballot); the pivot lane posts its live
// dwords to LDS, every lane reads them back (one broadcast address per b128) and folds c_j times the
// pivot row into its own (c_j = f_j / f_p, the pivot lane 1 ^ 1/f_p, which leaves row_p / f_p), with
// c_j's v_perm tables read from an LDS copy of kPerm by log c_j and the pivot dwords made scalar, so
// the selectors are SALU work.  Against k_solve_reg: no per-step table build (~70 VALU), no v_readlane
// per pivot dword; against k_solve_pq: one wave and ~9 KB of LDS per block and no barrier, so blocks
// also fit beside the syndrome program's waves.
__global__ void __launch_bounds__(64) k_solve_lean(SolveArgs a) {
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[64];
    __shared__ __attribute__((aligned(16))) uint4 prow_s[8];  // the pivot row's live dwords, by quad
    // the coefficient tables and pivot infos during the elimination; the final rows after it
    constexpr uint32_t RS = 33;  // final row stride (dwords; no bank conflicts)
    __shared__ __attribute__((aligned(16))) uint32_t un[64 * RS];
    uint4* tlA = reinterpret_cast<uint4*>(un);    // [255]
    uint32_t* tlB = un + 4 * 255;                 // [255]
    uint32_t* pinfo = tlB + 255;                  // [256]: log f | log(1 ^ 1/f) << 8 | (1 ^ 1/f != 0) << 16
    const uint32_t lane = threadIdx.x;
    if (a.status_init)  // the host-decided statuses (disjoint from the solver's blocks, ST_PENDING)
        for (uint32_t i = blockIdx.x * 64 + lane; i < a.n_all; i += gridDim.x * 64)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > 64) {
        if (lane == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = a.row_margin ? min(min(nr, 64u), e + a.row_margin) : min(nr, 64u);
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    gf_tables_copy(ex, lg);
    for (uint32_t l = lane; l < 255; l += 64) {
        tlA[l] = make_uint4(kPerm.A[l][0], kPerm.A[l][1], kPerm.A[l][2], kPerm.A[l][3]);
        tlB[l] = kPerm.B[l];
    }
    uint32_t row[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) row[w] = 0;
    if (lane < nrow) {  // every byte load of the row in flight at once
        const uint8_t* mr = a.mrep + (size_t)U[lane] * a.mrep_stride;
#pragma unroll
        for (int w = 0; w < 16; ++w)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if ((uint32_t)(4 * w + i) < e) row[w] |= (uint32_t)mr[E[4 * w + i]] << (8 * i);
        const uint32_t pos = e + lane;
#pragma unroll
        for (int w = 0; w < 32; ++w)
            if ((pos >> 2) == (uint32_t)w) row[w] |= 1u << (8 * (pos & 3));
    }
    __syncthreads();  // ex / lg
    for (uint32_t x = lane; x < 256; x += 64) {
        uint32_t v = 0;
        if (x) {
            const uint32_t lx = lg[x], cp = 1u ^ ex[255u - lx];
            v = lx | (cp ? (uint32_t)lg[cp] << 8 | 1u << 16 : 0u);
        }
        pinfo[x] = v;
    }
    __syncthreads();  // tables and pinfo
    bool used = lane >= nrow;
    const uint32_t q1 = (e + nrow + 3) >> 2;  // live dwords
    for (uint32_t k = 0; k < e; ++k) {
        const uint32_t W = k >> 2;
        uint32_t rw = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w)
            if ((uint32_t)w == W) rw = row[w];
        const uint32_t f = (rw >> (8 * (k & 3))) & 0xFFu;
        const uint64_t bal = __ballot(f != 0 && !used);
        if (bal == 0) {  // rank-deficient on these rows (uniform)
            if (lane == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
        const uint32_t p = (uint32_t)__ffsll((unsigned long long)bal) - 1;
        const bool me = lane == p;
        used |= me;
        const uint32_t pif = pinfo[f];
        // the pivot lane posts its live dwords (quads from W / 4; columns < k are zero there)
        const uint32_t w4 = W >> 2, q4 = (q1 + 3) >> 2;
        if (me) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if ((uint32_t)j >= w4 && (uint32_t)j < q4)
                    prow_s[j] = make_uint4(row[4 * j], row[4 * j + 1], row[4 * j + 2], row[4 * j + 3]);
        }
        const uint32_t pip = (uint32_t)__builtin_amdgcn_readlane((int)pif, (int)p);
        const uint32_t ilgp = 255u - (pip & 0xFFu);
        uint32_t l = me ? (pif >> 8) & 0xFFu : (pif & 0xFFu) + ilgp;
        l = l >= 255u ? l - 255u : l;
        const bool act = me ? (pif >> 16) != 0 : f != 0;
        const uint4 A = tlA[act ? l : 0];
        const uint32_t B = tlB[act ? l : 0];
        __builtin_amdgcn_wave_barrier();  // (LDS operations of one wave complete in order)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((uint32_t)j < w4 || (uint32_t)j >= q4) continue;  // uniform
            const uint4 P = prow_s[j];
            const uint32_t px[4] = {(uint32_t)__builtin_amdgcn_readfirstlane(P.x), (uint32_t)__builtin_amdgcn_readfirstlane(P.y),
                                    (uint32_t)__builtin_amdgcn_readfirstlane(P.z), (uint32_t)__builtin_amdgcn_readfirstlane(P.w)};
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const uint32_t m = act ? perm_mul(A, B, px[d]) : 0u;
                row[4 * j + d] ^= m;
            }
        }
        if (lane == 0) pivl[k] = (uint8_t)p;
        __builtin_amdgcn_wave_barrier();
    }
    // the final rows into LDS (over the tables), X[k][m] = identity byte (e + piv_m) of pivot row piv_k
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 32; ++w) un[lane * RS + w] = row[w];
    __syncthreads();
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = lane; m < e; m += 64) XP[m] = pivl[m];
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(un);
    for (uint32_t m = 0; m < e; ++m) {  // row m of X: one byte per lane, no index division
        const uint32_t pm = pivl[m];
        for (uint32_t k = lane; k < e; k += 64) xc[m * xs + k] = rb[pivl[k] * (RS * 4) + e + pm];
    }
    if (lane == 0) a.status[b] = 1;
}

// General solver for the blocks the fast solvers deferred: any e, every received repair.  The
// received rows are taken in order and reduced against a Gauss-Jordan basis of the rows kept so far
// (basis row i: pivot column pc[i], coefficients zero on every other pivot column, then the
// combination of selected received rows it stands for); a row that reduces to zero is dependent and
// skipped, the others extend the basis, until e rows are kept (rank e: the block decodes, and X is
// the combination part) or the rows run out (rank-deficient: Decode returns (false, nil, nil),
// RQ/decoder.go:120-121).  The working set is e x 2e bytes whatever the number of received repairs:
// in LDS for e <= lds_e, else in a global workspace.  Replaces GaussianElimination
// (RQ/discmath/gauss.go:7-45) on the e erased columns.
__global__ void __launch_bounds__(256) k_solve(SolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ int piv;
    __shared__ uint32_t todo[256], ntodo;
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    bool tables = false;  // the exp/log tables are copied before the first block this workgroup solves
    // A persistent grid of at most one workgroup per CU: each pass, every thread checks one block's
    // status (all of a workgroup's checks in flight at once) and the workgroup solves the deferred
    // ones.  Almost every decode defers none, and the launch then costs one status read per thread.
    for (uint32_t base = blockIdx.x; base < a.n_map; base += gridDim.x * 256) {
    if (tid == 0) ntodo = 0;
    __syncthreads();
    {
        const uint32_t bi = base + tid * gridDim.x;
        if (tid < 256 && bi < a.n_map && a.status[a.blk_map[bi]] == ST_FALLBACK) todo[atomicAdd(&ntodo, 1u)] = bi;
    }
    __syncthreads();
    const uint32_t nt = ntodo;
    for (uint32_t ti = 0; ti < nt; ++ti) {
    const uint32_t bi = todo[ti], b = a.blk_map[bi];
    if (!tables) {
        gf_tables_copy(ex, lg);
        tables = true;
    }
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    const uint32_t W2 = basis_width(e);
    // v (W2) | coefficient of v on each basis row (e) | pc (e x u16) | rowid (e x u16) | basis (e x W2):
    // in LDS for e <= lds_e, else in this block's global workspace (solve_ws_bytes(e))
    uint8_t* v = (e <= a.lds_e) ? sm : a.gws + 64ull * a.goff[bi];
    uint8_t* cf = v + W2;
    uint16_t* pc = reinterpret_cast<uint16_t*>(cf + ((e + 15) & ~15u));
    uint16_t* rowid = pc + ((e + 7) & ~7u);
    uint8_t* A = reinterpret_cast<uint8_t*>(rowid + ((e + 7) & ~7u));
    __syncthreads();
    auto gm = [&](uint8_t x, uint8_t y) -> uint8_t { return (x && y) ? ex[lg[x] + lg[y]] : (uint8_t)0; };
    uint32_t np = 0;
    for (uint32_t j = 0; j < nr && np < e; ++j) {
        const uint8_t* mr = a.mrep + (size_t)U[j] * a.mrep_stride;
        for (uint32_t c = tid; c < W2; c += nthr) v[c] = (c < e) ? mr[E[c]] : (uint8_t)(c == e + np);
        __syncthreads();
        for (uint32_t i = tid; i < np; i += nthr) cf[i] = v[pc[i]];
        if (tid == 0) piv = (int)e;
        __syncthreads();
        // v ^= sum_i cf[i] * basis_i (basis rows vanish on each other's pivot columns)
        for (uint32_t c = tid; c < W2; c += nthr) {
            uint8_t x = v[c];
            for (uint32_t i = 0; i < np; ++i) {
                const uint8_t f = cf[i];
                if (f) x ^= gm(f, A[(size_t)i * W2 + c]);
            }
            v[c] = x;
            if (c < e && x) atomicMin(&piv, (int)c);
        }
        __syncthreads();
        const uint32_t p = (uint32_t)piv;
        if (p >= e) {  // dependent on the rows kept so far
            __syncthreads();
            continue;
        }
        const uint8_t inv = ex[255 - lg[v[p]]];
        __syncthreads();
        for (uint32_t c = tid; c < W2; c += nthr) v[c] = gm(v[c], inv);
        __syncthreads();
        // clear column p from the basis, then append v
        for (size_t idx = tid; idx < (size_t)np * W2; idx += nthr) {
            const uint32_t i = (uint32_t)(idx / W2), c = (uint32_t)(idx - (size_t)i * W2);
            const uint8_t f = A[(size_t)i * W2 + p];
            if (f && c != p) A[idx] ^= gm(f, v[c]);
        }
        __syncthreads();
        for (uint32_t i = tid; i < np; i += nthr) A[(size_t)i * W2 + p] = 0;
        for (uint32_t c = tid; c < W2; c += nthr) A[(size_t)np * W2 + c] = v[c];
        if (tid == 0) { pc[np] = (uint16_t)p; rowid[np] = (uint16_t)j; }
        ++np;
        __syncthreads();
    }
    if (np < e) {
        if (tid == 0) a.status[b] = 0;
        __syncthreads();
        continue;
    }
    // basis row i solves erased column pc[i]: x_pc[i] = sum_m A[i][e + m] s_rowid[m]
    uint8_t* xc = a.xcoef + 64ull * a.xoff[bi];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += nthr) XP[m] = rowid[m];
    for (size_t idx = tid; idx < (size_t)e * e; idx += nthr) {
        const uint32_t i = (uint32_t)(idx / e), m = (uint32_t)(idx - (size_t)i * e);
        xc[(size_t)m * xs + pc[i]] = A[(size_t)i * W2 + e + m];
    }
    if (tid == 0) a.status[b] = 1;
    __syncthreads();  // the next block reuses the LDS
    }
    __syncthreads();  // todo / ntodo are rewritten by the next pass
    }
}

// k_solve's working set for e erased rows (LDS when e <= lds_e, else global workspace).
size_t solve_ws_bytes(uint32_t e) {
    const uint32_t W2 = basis_width(e);
    return W2 + ((e + 15) & ~15u) + 4 * ((e + 7) & ~7u) + (size_t)e * W2;
}

// The e <= 64 solver: k_solve_fast<1> with four waves per block; experiments builds select one wave
// (RQHIP_SOLVE_NW=1) or the register-resident k_solve_reg (RQHIP_SOLVE_NW=0; measured 111 us against
// 94 us for the four-wave solver at 1 024 blocks, e = 55: profiles/r02r).
// Elimination by GF(256) multiplication (k_solve_pm, the default) or by alpha-multiple tables
// (k_solve_fast: RQHIP_SOLVE_PM=0 in experiments builds).  Measured at 1 024 blocks K=1024, e ~ 52:
// decode 0.810 against 0.820 ms per step; the e ~ 113 wide pass at K=2048: 192 against 237 us
// (profiles/r02ag).
static bool solve_pm() {
#ifdef RQHIP_EXPERIMENTS
    static const bool on = [] { const char* e = std::getenv("RQHIP_SOLVE_PM"); return !(e && e[0] == '0'); }();
    return on;
#else
    return true;
#endif
}

// k_solve_pm's coefficient tables from a per-block log-indexed LUT (the default; RQHIP_SOLVE_LUT=0 in
// experiments builds builds them per step): the solve is VALU-bound at four blocks per CU, and the
// per-step perm_tables were ~40 VALU per lane.  Decode 0.806 -> 0.790 ms, wide pass 194 -> 182 us
// (profiles/r02ag/lut).
static bool solve_lut() {
#ifdef RQHIP_EXPERIMENTS
    static const bool on = [] { const char* e = std::getenv("RQHIP_SOLVE_LUT"); return !(e && e[0] == '0'); }();
    return on;
#else
    return true;
#endif
}

// k_solve_pq (the default) against k_solve_pm (RQHIP_SOLVE_PQ=0 in experiments builds)
static bool solve_pq() {
#ifdef RQHIP_EXPERIMENTS
    static const bool on = [] { const char* e = std::getenv("RQHIP_SOLVE_PQ"); return !(e && e[0] == '0'); }();
    return on;
#else
    return true;
#endif
}

// k_solve_pq's column buffer with pinfo words (RQHIP_SOLVE_PF=1 in experiments builds)
static bool solve_pf() {
#ifdef RQHIP_EXPERIMENTS
    static const bool on = [] { const char* e = std::getenv("RQHIP_SOLVE_PF"); return e && e[0] == '1'; }();
    return on;
#else
    return false;
#endif
}

// the lean one-wave first-pass solver (k_solve_lean; RQHIP_SOLVE_LEAN=1 in experiments builds)
static bool solve_lean() {
#ifdef RQHIP_EXPERIMENTS
    static const bool on = [] { const char* e = std::getenv("RQHIP_SOLVE_LEAN"); return e && e[0] == '1'; }();
    return on;
#else
    return false;
#endif
}

static int solve_nw() {
#ifdef RQHIP_EXPERIMENTS
    static const int nw = [] {
        const char* e = std::getenv("RQHIP_SOLVE_NW");
        return e ? std::atoi(e) : 4;
    }();
    return nw;
#else
    return 4;
#endif
}

int launch_solve(const SolveArgs& a_in, uint32_t n_blocks, bool need_general, bool wide, uint32_t max_lds_e,
                 void* stream) {
    // the first k_solve_pm launch copies the host-decided statuses (a_in.status_init); the other
    // solvers get them uploaded first, and later launches never copy
    SolveArgs first = a_in;  // the first pass copies the host-decided statuses
    first.diag_steps = 0;
#ifdef RQHIP_EXPERIMENTS
    static const uint32_t dsteps = [] { const char* e = std::getenv("RQHIP_SOLVE_STEPS"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    first.diag_steps = dsteps;
#endif
    SolveArgs a = first;
    a.status_init = nullptr;
    const bool pm_first = solve_lean() || solve_nw() == 8 ||
                          (solve_pm() && (solve_nw() == 1 || solve_nw() == 2 || solve_nw() == 4));
    if (a_in.status_init && !pm_first &&
        hipMemcpyAsync(a.status, a_in.status_init, (size_t)a_in.n_all * 4, hipMemcpyHostToDevice,
                       (hipStream_t)stream) != hipSuccess)
        return (int)hipGetLastError();
    if (solve_lean()) hipLaunchKernelGGL(k_solve_lean, dim3(n_blocks), dim3(64), 0, (hipStream_t)stream, first);
    else switch (solve_nw()) {
        case 1:
            if (solve_pm() && solve_pq()) hipLaunchKernelGGL((k_solve_pq<1, 1>), dim3(n_blocks), dim3(64), 0, (hipStream_t)stream, first);
            else if (solve_pm()) hipLaunchKernelGGL((k_solve_pm<1, 1, true>), dim3(n_blocks), dim3(64), 0, (hipStream_t)stream, first);
            else hipLaunchKernelGGL((k_solve_fast<1, 1>), dim3(n_blocks), dim3(64), 0, (hipStream_t)stream, a);
            break;
        case 8:  // experiments: eight waves per block
            hipLaunchKernelGGL((k_solve_pq<1, 8>), dim3(n_blocks), dim3(512), 0, (hipStream_t)stream, first);
            break;
        case 2:
            if (solve_pq()) hipLaunchKernelGGL((k_solve_pq<1, 2>), dim3(n_blocks), dim3(128), 0, (hipStream_t)stream, first);
            else hipLaunchKernelGGL((k_solve_pm<1, 2, true>), dim3(n_blocks), dim3(128), 0, (hipStream_t)stream, first);
            break;
        case 4:
            if (solve_pm() && solve_lut() && solve_pq() && solve_pf())
                hipLaunchKernelGGL((k_solve_pq<1, 4, true>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, first);
            else if (solve_pm() && solve_lut() && solve_pq())
                hipLaunchKernelGGL((k_solve_pq<1, 4>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, first);
            else if (solve_pm() && solve_lut())
                hipLaunchKernelGGL((k_solve_pm<1, 4, true>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, first);
            else if (solve_pm())
                hipLaunchKernelGGL((k_solve_pm<1, 4, false>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, first);
            else hipLaunchKernelGGL((k_solve_fast<1, 4>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a);
            break;
        default: hipLaunchKernelGGL(k_solve_reg, dim3(n_blocks), dim3(64), 0, (hipStream_t)stream, a); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !need_general) return (int)e;
    if (wide) {  // blocks with 64 < e <= 128; the rare rank-deficient-on-64-rows block goes to k_solve
        if (solve_pm() && solve_lut() && solve_pq())
            hipLaunchKernelGGL((k_solve_pq<2, 4>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a);
        else if (solve_pm() && solve_lut())
            hipLaunchKernelGGL((k_solve_pm<2, 4, true>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a);
        else if (solve_pm())
            hipLaunchKernelGGL((k_solve_pm<2, 4, false>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a);
        else hipLaunchKernelGGL((k_solve_fast<2, 4>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    // k_solve's dynamic-LDS limit is a per-device attribute, and the host-memory API drives one host thread
    // per device (run_sharded): set it once per device, race-free, on the device this thread launches on
    static std::once_flag attr_once[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    std::call_once(attr_once[dev], [] {
        (void)hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    });
    const size_t lds = solve_ws_bytes(std::min<uint32_t>(max_lds_e, a.lds_e));
    a.n_map = n_blocks;
    uint32_t grid = std::min<uint32_t>(n_blocks, 256);
#ifdef RQHIP_EXPERIMENTS
    if (const char* g = std::getenv("RQHIP_GSOLVE_GRID")) grid = std::max(1, std::min(256, std::atoi(g)));
#endif
    hipLaunchKernelGGL(k_solve, dim3(grid), dim3(256), lds, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

uint32_t solve_lds_e_max() {
    uint32_t e = 1;
    while (solve_ws_bytes(e + 1) <= 140 * 1024) ++e;
    return e;
}

// ------------------------------ decode: x_E = X * s ------------------------------------------
// GF(256) multiply by a uniform constant c with v_perm_b32 as an 8-entry byte lookup on four bytes
// at once: x = x0 + 8*x1 + 64*x2 (3 + 3 + 2 bits), c*x = c*x0 ^ c*(8*x1) ^ c*(64*x2), so three
// v_perm (selectors x & 7, (x >> 3) & 7, x >> 6 per byte) against per-coefficient tables and two
// XORs per dword: 5 VALU per mul-add instead of 8 bit-selects (replaces asmSSSE3MulAdd's nibble
// pshufb, RQ/discmath/optimizations.s:36-78, with CDNA4's byte permute).

// One wave per (unit = solved block x strip, output slice of KC).  Workgroup w maps to slice
// (w / 8) % np of unit (w / 8np) * 8 + w % 8: the slices of one unit share an XCD (workgroups are
// dealt to the 8 XCDs round-robin) and are dispatched together, so their common syndrome rows are
// read from HBM once and hit L2 after.  Each lane owns CPL dword columns (64 apart: every
// load/store instruction is one contiguous 256-B segment).  The slice's tables are built from X
// straight into LDS (perm_tables: A = the four 8-entry halves (b128), B = the 2-bit table), for
// MC syndromes m at a time (one chunk whenever e <= MC).
template <int KC, int CPL, int PD, int OCC, bool PAIR = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OCC)))
k_apply(ApplyArgs a, uint32_t n_units, uint32_t np, uint32_t MC) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xsh[];
    const uint32_t strips = ((a.T >> 2) + 64 * CPL - 1) / (64 * CPL);
    const uint32_t w = blockIdx.x, slice = (w / 8) % np, unit = (w / (8 * np)) * 8 + (w & 7);
    if (unit >= n_units) return;
    const uint32_t bi = unit / strips, strip = unit - bi * strips;
    const uint32_t b = a.blk_map[bi];
    if (a.status[b] != 1) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t k0 = slice * KC;
    if (k0 >= e) return;
    const uint32_t Td = a.T >> 2;
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint16_t* XP = a.xpiv + a.erased_off[b];
    const uint32_t r0b = a.rep_off[b];
    // the block's received repair rows and its r0 rows as buffer resources: a syndrome row's offset
    // is one SGPR (soffset) and a lane's column one VGPR, so the loads carry no address arithmetic.
    // Offsets are 32-bit within one block (its received repairs and r0 rows span < 4 GiB, as every
    // launch's buffers do, rq_engine.cpp launch_col); the record count is unlimited.
    const __amdgpu_buffer_rsrc_t rsR =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.recv + (size_t)r0b * a.T), (short)0, -1, 0x20000);
    const __amdgpu_buffer_rsrc_t rs0 =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.r0 + (size_t)b * a.n_union * a.T), (short)0, -1, 0x20000);
    // the block's rows likewise (g_E in, x_E out): a row's byte offset E_k * T < 4 GiB (K' * T)
    const __amdgpu_buffer_rsrc_t rsD =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.data + (size_t)b * a.data_stride), (short)0, -1, 0x20000);
    // a chunk's syndromes are processed in whole groups of PD: the padding m's get zero tables and
    // a valid row offset, so the ring needs no branch (and the compiler no register copies)
    const uint32_t mc_max = (min(MC, e) + PD - 1) / PD * PD;
    uint4* tA = reinterpret_cast<uint4*>(xsh);                  // [m - c0][KC]
    uint32_t* tB = xsh + (size_t)mc_max * KC * 4;                // [m - c0][KC]
    uint32_t* offr = tB + (size_t)mc_max * KC;                   // [m - c0], m < mcp + PD
    uint32_t* off0 = offr + mc_max + PD;
    const uint8_t* xc = a.xcoef + 64ull * a.xoff[bi];
    const uint32_t xs = x_stride(e);
    // a lane's byte offset in a row per column (dead columns past T/4 read column 0, store nothing)
    uint32_t vo[CPL];
    bool live[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const uint32_t c = strip * 64 * CPL + j * 64 + lane;
        live[j] = c < Td;
        vo[j] = live[j] ? c * 4 : 0u;
    }
    // The erased rows were not cleared before the syndrome program, so s = M (x_E ^ g_E) with g_E their
    // current bytes: start every output from g_E and X s completes it to x_E.
    const uint32_t kn = min((uint32_t)KC, e - k0);
    uint32_t acc[KC][CPL];
    // lane k holds output k's row offset (one load for the slice, KC <= 64; made scalar per k, so the
    // row loads and stores need no waterfall over a per-lane offset)
    const uint32_t erow = E[k0 + min(lane, kn - 1)] * a.T;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        const int go = __builtin_amdgcn_readlane((int)erow, k);
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const uint32_t g = __builtin_amdgcn_raw_buffer_load_b32(rsD, (int)vo[j], go, 0);
            acc[k][j] = (uint32_t)k < kn ? g : 0u;
        }
    }
    // syndromes are loaded PD m ahead into a ring (received row and r0 row, XORed on use); MC is a
    // multiple of PD, so ring slot d always holds syndrome m = d (mod PD) across chunks
    uint32_t ra[PD][CPL], rb[PD][CPL];
    for (uint32_t c0 = 0; c0 < e; c0 += MC) {
        const uint32_t mc = min(MC, e - c0), mcp = (mc + PD - 1) / PD * PD;
        __syncthreads();  // the previous chunk's tables are consumed
        // coefficient bytes loaded eight per lane at a time before their tables are built (one
        // dependent load round trip per eight instead of per coefficient)
        for (uint32_t i0 = lane; i0 < mcp * KC; i0 += 64 * 8) {
            uint32_t cv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t idx = i0 + 64 * u, m = idx / KC, k = idx - m * KC;
                cv[u] = (idx < mc * KC && k0 + k < e) ? xc[(size_t)(c0 + m) * xs + k0 + k] : 0u;
            }
            // the coefficient's tables from the constant set by its log (five loads) instead of built
            // from its alpha-multiples (~70 VALU each); c = 0 gives all-zero tables
            uint32_t lc[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) lc[u] = kGf.lg[cv[u]];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t idx = i0 + 64 * u;
                if (idx >= mcp * KC) break;
                const bool nz = cv[u] != 0;
                const uint32_t* pa = kPerm.A[lc[u]];
                tA[idx] = nz ? make_uint4(pa[0], pa[1], pa[2], pa[3]) : make_uint4(0, 0, 0, 0);
                tB[idx] = nz ? kPerm.B[lc[u]] : 0u;
            }
        }
        for (uint32_t m = lane; m < mcp + PD; m += 64) {  // byte offsets in the block (row 0 past e)
            const uint32_t j = c0 + m < e ? XP[c0 + m] : 0u;
            offr[m] = j * a.T;
            off0[m] = c0 + m < e ? a.rep_uidx[r0b + j] * a.T : 0u;
        }
        __syncthreads();
        if (c0 == 0) {
#pragma unroll
            for (int d = 0; d < PD; ++d) {
                const int sr = (int)__builtin_amdgcn_readfirstlane(offr[d]);
                const int s0o = (int)__builtin_amdgcn_readfirstlane(off0[d]);
#pragma unroll
                for (int j = 0; j < CPL; ++j) {
                    ra[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rsR, (int)vo[j], sr, 0);
                    rb[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rs0, (int)vo[j], s0o, 0);
                }
            }
        }
        // (round 2 measured the syndromes in pairs 3 % slower, profiles/r02w; the round-3 pair loop
        // above is 4 % faster; skipping a last slice's padding outputs by a uniform branch per k, 188
        // -> 203 us: profiles/r03_dense/r03e)
        // Software pipeline: the tables of the next (m, k) and the next ring offsets are read from LDS
        // one step ahead, and sched_barrier keeps the scheduler from sinking those reads next to their
        // use (it did: one exposed LDS round trip per 25 VALU).  The last step's look-ahead reads one
        // entry past the chunk (inside the allocation, launch_apply) and is discarded.
        if constexpr (PAIR) {
            static_assert(PD == 2, "paired syndromes take the ring two at a time");
            // Syndromes m, m + 1 folded into each accumulator together: six lookups by three XOR3 (4.5
            // VALU per mul-add instead of 5); both syndromes' fields and both tables live at once (11
            // VGPRs spill at KC 8, CPL 5 under the four-waves-per-SIMD bound, and it is still faster).
            uint4 An0 = tA[0], An1 = tA[KC];
            uint32_t Bn0 = tB[0], Bn1 = tB[KC];
            for (uint32_t mb = 0; mb < mcp; mb += 2) {
                uint32_t f0[2][CPL], f1[2][CPL], f2[2][CPL];
#pragma unroll
                for (int d = 0; d < 2; ++d)
#pragma unroll
                    for (int j = 0; j < CPL; ++j) {
                        const uint32_t x = ra[d][j] ^ rb[d][j];
                        f0[d][j] = x & 0x07070707u;
                        f1[d][j] = (x >> 3) & 0x07070707u;
                        f2[d][j] = (x >> 6) & 0x03030303u;
                    }
#pragma unroll
                for (int d = 0; d < 2; ++d) {  // the next pair's rows (row 0 past e)
                    const int sr = (int)__builtin_amdgcn_readfirstlane(offr[mb + 2 + d]);
                    const int s0o = (int)__builtin_amdgcn_readfirstlane(off0[mb + 2 + d]);
#pragma unroll
                    for (int j = 0; j < CPL; ++j) {
                        ra[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rsR, (int)vo[j], sr, 0);
                        rb[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rs0, (int)vo[j], s0o, 0);
                    }
                }
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    const uint4 A0 = An0, A1 = An1;
                    const uint32_t B0 = Bn0, B1 = Bn1;
                    const uint32_t n0 = (k + 1 < KC) ? mb * KC + k + 1 : (mb + 2) * KC;
                    An0 = tA[n0];
                    Bn0 = tB[n0];
                    An1 = tA[n0 + KC];
                    Bn1 = tB[n0 + KC];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < CPL; ++j) {
                        const uint32_t p0 = __builtin_amdgcn_perm(A0.y, A0.x, f0[0][j]);
                        const uint32_t p1 = __builtin_amdgcn_perm(A0.w, A0.z, f1[0][j]);
                        const uint32_t p2 = __builtin_amdgcn_perm(B0, B0, f2[0][j]);
                        const uint32_t q0 = __builtin_amdgcn_perm(A1.y, A1.x, f0[1][j]);
                        const uint32_t q1 = __builtin_amdgcn_perm(A1.w, A1.z, f1[1][j]);
                        const uint32_t q2 = __builtin_amdgcn_perm(B1, B1, f2[1][j]);
                        acc[k][j] = xor3(xor3(xor3(acc[k][j], p0, p1), p2, q0), q1, q2);
                    }
                }
            }
            continue;
        }
        uint4 An = tA[0];
        uint32_t Bn = tB[0];
        uint32_t nsr = offr[PD], ns0o = off0[PD];  // read one step ahead, made scalar at use
        for (uint32_t mb = 0; mb < mcp; mb += PD) {
#pragma unroll
            for (int d = 0; d < PD; ++d) {
                const uint32_t m = mb + d;
                uint32_t s0[CPL], s1[CPL], s2[CPL];
#pragma unroll
                for (int j = 0; j < CPL; ++j) {
                    const uint32_t x = ra[d][j] ^ rb[d][j];
                    s0[j] = x & 0x07070707u;
                    s1[j] = (x >> 3) & 0x07070707u;
                    s2[j] = (x >> 6) & 0x03030303u;
                }
                {  // past e the ring reads row 0 (zero tables consume it)
                    const int sr = (int)__builtin_amdgcn_readfirstlane(nsr);
                    const int s0o = (int)__builtin_amdgcn_readfirstlane(ns0o);
#pragma unroll
                    for (int j = 0; j < CPL; ++j) {
                        ra[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rsR, (int)vo[j], sr, 0);
                        rb[d][j] = __builtin_amdgcn_raw_buffer_load_b32(rs0, (int)vo[j], s0o, 0);
                    }
                    nsr = offr[m + PD + 1];
                    ns0o = off0[m + PD + 1];
                }
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    const uint4 A = An;
                    const uint32_t B = Bn;
                    An = tA[m * KC + k + 1];
                    Bn = tB[m * KC + k + 1];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < CPL; ++j) {
                        const uint32_t p0 = __builtin_amdgcn_perm(A.y, A.x, s0[j]);
                        const uint32_t p1 = __builtin_amdgcn_perm(A.w, A.z, s1[j]);
                        const uint32_t p2 = __builtin_amdgcn_perm(B, B, s2[j]);
                        acc[k][j] = xor3(acc[k][j], p0, p1) ^ p2;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        if ((uint32_t)k < kn) {
            const int go = __builtin_amdgcn_readlane((int)erow, k);
#pragma unroll
            for (int j = 0; j < CPL; ++j)
                if (live[j]) {
                    if (a.out_sc1) __builtin_amdgcn_raw_buffer_store_b32(acc[k][j], rsD, (int)vo[j], go, 16);
                    else __builtin_amdgcn_raw_buffer_store_b32(acc[k][j], rsD, (int)vo[j], go, 0);
                }
        }
    }
}

// KC is at most 8 in the shipped library (launch_apply's cap); experiments builds (RQHIP_APPLY_KC)
// reach the wider slices.
template <int CPL, int PD, int OCC, int KCMAX>
static void launch_apply_cpl(const ApplyArgs& a, uint32_t kc, dim3 g, uint32_t ec, size_t lds_min, hipStream_t st,
                             uint32_t nu, uint32_t np, uint32_t mc) {
    // the kernel's LDS: tables (20 or 24 B per coefficient) for a chunk of up to ec syndromes padded to
    // whole groups of PD, the two row-offset arrays (PD past the chunk) and 16 B for the pipelined
    // look-ahead past the last offset -- sized exactly, so four 64-lane waves per SIMD also fit the
    // LDS (e ~ 58, KC 8: 9.8 KB per wave)
    const size_t mcx = (ec + PD - 1) / PD * PD;
    const size_t lds = std::max(lds_min, mcx * kc * 20 + (mcx + PD) * 8 + 16);
    // Syndromes in pairs (the default at PD = 2; RQHIP_APPLY_PAIR=0 in experiments builds restores the
    // one-at-a-time loop): 185 -> 178 us at 1 024 blocks K=1024, two interleaved rounds on one box
    // (profiles/r03_apply2).  The look-ahead of a chunk's last pair reads up to 2 KC table entries past
    // it, hence the slack.
#ifdef RQHIP_EXPERIMENTS
    static const bool pair = [] { const char* e = std::getenv("RQHIP_APPLY_PAIR"); return !(e && e[0] == '0'); }();
#else
    constexpr bool pair = true;
#endif
    if constexpr (PD == 2 && KCMAX == 8) {
        if (pair && kc <= 4) {
            hipLaunchKernelGGL((k_apply<4, CPL, 2, OCC, true>), g, dim3(64), lds + 40 * 4, st, a, nu, np, mc);
            return;
        }
        if (pair && kc == 8) {
            // the KC = 8 pair loop at three waves per SIMD: under four's 128 VGPRs it spills 11 (CPL 5);
            // 170.9 against 177.1 us, three interleaved rounds (profiles/r03_apply2/occ);
            // RQHIP_APPLY_PAIROCC=4 in experiments builds restores four
#ifdef RQHIP_EXPERIMENTS
            static const bool occ4p = [] { const char* e = std::getenv("RQHIP_APPLY_PAIROCC"); return e && e[0] == '4'; }();
            if (occ4p) {
                hipLaunchKernelGGL((k_apply<8, CPL, 2, OCC, true>), g, dim3(64), lds + 40 * 8, st, a, nu, np, mc);
                return;
            }
#endif
            hipLaunchKernelGGL((k_apply<8, CPL, 2, 3, true>), g, dim3(64), lds + 40 * 8, st, a, nu, np, mc);
            return;
        }
    }
    if (kc <= 4) { hipLaunchKernelGGL((k_apply<4, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc); return; }
    if constexpr (KCMAX > 8) {
        switch (kc) {
            case 12: { hipLaunchKernelGGL((k_apply<12, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc); return; }
            case 16: { hipLaunchKernelGGL((k_apply<16, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc); return; }
            case 20: { hipLaunchKernelGGL((k_apply<20, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc); return; }
            case 24: { hipLaunchKernelGGL((k_apply<24, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc); return; }
            default: break;
        }
    }
    hipLaunchKernelGGL((k_apply<8, CPL, PD, OCC>), g, dim3(64), lds, st, a, nu, np, mc);
}

#ifdef RQHIP_EXPERIMENTS
// Syndrome prefetch depth of k_apply (RQHIP_APPLY_PD = 4 / 8 in experiments builds; else 2 at four
// waves per SIMD).
static int apply_pd() {
    static const int pd = [] {
        const char* e = std::getenv("RQHIP_APPLY_PD");
        return e ? std::atoi(e) : 2;
    }();
    return pd;
}
#endif

template <int CPL>
static void launch_apply_pd(const ApplyArgs& a, uint32_t kc, dim3 g, uint32_t ec, size_t lds_min, hipStream_t st,
                            uint32_t nu, uint32_t np, uint32_t mc) {
#ifdef RQHIP_EXPERIMENTS
    // RQHIP_APPLY_OCC=3: the round-2 shape (PD 4, no occupancy bound, ~3 waves per SIMD at CPL 5)
    static const bool occ3 = [] { const char* e = std::getenv("RQHIP_APPLY_OCC"); return e && e[0] == '3'; }();
    if (apply_pd() == 8) return launch_apply_cpl<CPL, 8, 1, 24>(a, kc, g, ec, lds_min, st, nu, np, mc);
    if (occ3 || apply_pd() == 4 || kc > 8) return launch_apply_cpl<CPL, 4, 1, 24>(a, kc, g, ec, lds_min, st, nu, np, mc);
#endif
    // four waves per SIMD (<= 128 VGPRs, spill-free for KC <= 8 with a two-deep ring): 200 -> 192 us
    // at 1 024 blocks K=1024 (profiles/r03q)
    launch_apply_cpl<CPL, 2, 4, 8>(a, kc, g, ec, lds_min, st, nu, np, mc);
}

int launch_apply(const ApplyArgs& a, uint32_t /*n_strips*/, uint32_t n_blocks, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    const uint32_t Td = a.T / 4;
    uint32_t cpl = 1, best = 0xFFFFFFFFu;  // fewest padded columns, then the widest lanes
    for (uint32_t c : {1u, 2u, 4u, 5u}) {
        const uint32_t w = 64 * c, pad = (Td + w - 1) / w * w - Td;
        if (pad <= best) { best = pad; cpl = c; }
    }
    // balanced slices of KC <= 8 outputs (measured at e ~ 58, K=1024 T=1200: KC 4/8/12/16/20/28 ->
    // 244/210/238/254/282/324 us; small slices keep the accumulators few, so more waves fit per SIMD),
    // the slice's tables (20 B per coefficient) for MC syndromes within ~20 KB of LDS
    constexpr uint32_t MC = 256;
    const uint32_t e = std::max<uint32_t>(a.max_e, 1), ec = std::min(e, MC);
    uint32_t cap = std::max<uint32_t>(4, std::min<uint32_t>(8, (21504 / (20 * ec)) & ~3u));
#ifdef RQHIP_EXPERIMENTS
    if (const char* v = std::getenv("RQHIP_APPLY_KC")) cap = std::max(4, std::min(24, std::atoi(v))) & ~3u;
#endif
    const uint32_t np = (e + cap - 1) / cap, kc = (((e + np - 1) / np) + 3) & ~3u;
    size_t lds = 0;
#ifdef RQHIP_EXPERIMENTS
    if (const char* v = std::getenv("RQHIP_APPLY_LDS")) lds = (size_t)std::atoi(v);  // occupancy cap
#endif
    const uint32_t nu = (Td + 64 * cpl - 1) / (64 * cpl) * n_blocks;
    const dim3 g((nu + 7) / 8 * 8 * np);
    switch (cpl) {
        case 1: launch_apply_pd<1>(a, kc, g, ec, lds, st, nu, np, MC); break;
        case 2: launch_apply_pd<2>(a, kc, g, ec, lds, st, nu, np, MC); break;
        case 4: launch_apply_pd<4>(a, kc, g, ec, lds, st, nu, np, MC); break;
        default: launch_apply_pd<5>(a, kc, g, ec, lds, st, nu, np, MC); break;
    }
    return (int)hipGetLastError();
}

// ------------------------------ gather repairs from a device-resident C ----------------------
// Per-object API: out[r] = XOR of C rows of LT(isi_r) (encodeGen, RQ/params.go:162-182).
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

int launch_gather(const DevParams& p, const uint8_t* C, uint32_t T, const uint32_t* esi, uint32_t n, uint8_t* out,
                  void* stream) {
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, (hipStream_t)stream, p, C, T, esi, n, out);
    return (int)hipGetLastError();
}

}  // namespace rq
