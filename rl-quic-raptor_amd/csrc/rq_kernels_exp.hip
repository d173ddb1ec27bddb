// rq_kernels_exp.hip -- decode solvers measured and not shipped, compiled into the experiments library
// only (make EXPERIMENTS=1; knobs RQHIP_SOLVE_PM / _LUT / _NW / _LEAN, rq_kernels.hip launch_solve):
//   k_solve_fast  the round-1 solver (alpha-multiple tables, two barriers per pivot step)
//   k_solve_pm    GF(256) multiplication by per-lane v_perm tables (round 2; k_solve_pq's predecessor)
//   k_solve_reg   one wave, rows in registers (round 2: 111 vs 94 us, profiles/r02r)
//   k_solve_lean  one wave, LDS-broadcast pivot row (round 4: 122 us alone, 483 beside, profiles/r04j)
// The shipped solvers (k_solve_pq<1,4>, k_solve_pq<2,4>, k_solve) stay in rq_kernels.hip.
#ifndef RQHIP_EXPERIMENTS
#error "rq_kernels_exp.hip belongs to the experiments build only"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "rq_kernels_common.hpp"

namespace rq {

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

// The knob-selected first-pass solver (RQHIP_SOLVE_*): returns -1 when the knobs select a shipped
// k_solve_pq, else the launch's hipError_t.  first: the arguments of the launch that copies the
// host-decided statuses; a: the others (their statuses were uploaded).
int launch_solve_exp_first(const SolveArgs& first, const SolveArgs& a, uint32_t n_blocks, bool pm, bool lut, bool pq,
                           bool lean, int nw, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (lean) {
        hipLaunchKernelGGL(k_solve_lean, dim3(n_blocks), dim3(64), 0, st, first);
        return (int)hipGetLastError();
    }
    switch (nw) {
        case 1:
            if (pm && pq) return -1;
            if (pm) hipLaunchKernelGGL((k_solve_pm<1, 1, true>), dim3(n_blocks), dim3(64), 0, st, first);
            else hipLaunchKernelGGL((k_solve_fast<1, 1>), dim3(n_blocks), dim3(64), 0, st, a);
            break;
        case 2:
            if (pq) return -1;
            hipLaunchKernelGGL((k_solve_pm<1, 2, true>), dim3(n_blocks), dim3(128), 0, st, first);
            break;
        case 4:
            if (pm && lut && pq) return -1;
            if (pm && lut) hipLaunchKernelGGL((k_solve_pm<1, 4, true>), dim3(n_blocks), dim3(256), 0, st, first);
            else if (pm) hipLaunchKernelGGL((k_solve_pm<1, 4, false>), dim3(n_blocks), dim3(256), 0, st, first);
            else hipLaunchKernelGGL((k_solve_fast<1, 4>), dim3(n_blocks), dim3(256), 0, st, a);
            break;
        case 8:
            return -1;
        default:
            hipLaunchKernelGGL(k_solve_reg, dim3(n_blocks), dim3(64), 0, st, a);
            break;
    }
    return (int)hipGetLastError();
}

// The wide (64 < e <= 128) pass when the knobs select a non-shipped solver; -1 for k_solve_pq<2, 4>.
int launch_solve_exp_wide(const SolveArgs& a, uint32_t n_blocks, bool pm, bool lut, bool pq, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (pm && lut && pq) return -1;
    if (pm && lut) hipLaunchKernelGGL((k_solve_pm<2, 4, true>), dim3(n_blocks), dim3(256), 0, st, a);
    else if (pm) hipLaunchKernelGGL((k_solve_pm<2, 4, false>), dim3(n_blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_solve_fast<2, 4>), dim3(n_blocks), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

}  // namespace rq
