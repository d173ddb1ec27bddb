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
#include "rq_kernels_common.hpp"
#include "rq_gistream.hpp"

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

// ------------------------------ decode: X -> the register-table apply's stream ---------------
// gi_stream (rq_gistream.hpp) writes one block's part; k_xbits runs it for every block of the solve
// list, and the solvers run it for the blocks they finish (xb_on).
template <int KC, int G, int PDG, int PK = 0>
__device__ void xbits_block(const XbitsArgs& a, uint32_t bi, uint32_t tid) {
    const uint32_t b = a.blk_map[bi];
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint8_t* xc = a.xcoef + 64ull * a.xoff[bi];
    const uint32_t xs = x_stride(e);
    const uint16_t* xp = a.xpiv + a.erased_off[b];
    auto X = [&](uint32_t k, uint32_t m) { return xc[(size_t)m * xs + k]; };
    auto P = [&](uint32_t m) { return (uint32_t)xp[m]; };
    gi_stream<KC, G, PDG, decltype(X), decltype(P), PK>(a, bi, b, e, a.status[b] == 1, tid, 256, X, P);
}

template <int KC, int G, int PDG, int PK = 0>
__global__ void __launch_bounds__(256) k_xbits(XbitsArgs a) {
    xbits_block<KC, G, PDG, PK>(a, blockIdx.x, threadIdx.x);
}

int launch_xbits(const XbitsArgs& a, uint32_t n_blocks, const GiShape& s, void* stream) {
    if (!n_blocks) return 0;
    const hipStream_t st = (hipStream_t)stream;
#define RQ_XB(kc, g, p)                                                                                   \
    if (s.KC == kc && s.G == g && s.PDG == p && !s.PACK) {                                                \
        hipLaunchKernelGGL((k_xbits<kc, g, p>), dim3(n_blocks), dim3(256), 0, st, a);                     \
        return (int)hipGetLastError();                                                                    \
    }
#define RQ_XBP(kc, g, p)                                                                                  \
    if (s.KC == kc && s.G == g && s.PDG == p && s.PACK) {                                                 \
        hipLaunchKernelGGL((k_xbits<kc, g, p, 1>), dim3(n_blocks), dim3(256), 0, st, a);                  \
        return (int)hipGetLastError();                                                                    \
    }
    RQ_XB(8, 5, 2)
#ifdef RQHIP_EXPERIMENTS
    RQ_XB(16, 6, 1) RQ_XB(16, 6, 2) RQ_XB(16, 5, 2) RQ_XB(8, 6, 2) RQ_XB(8, 5, 1) RQ_XB(8, 4, 1) RQ_XB(16, 4, 2)
    RQ_XB(8, 4, 2) RQ_XB(8, 6, 1) RQ_XB(12, 5, 1) RQ_XB(12, 5, 2) RQ_XB(4, 5, 1) RQ_XB(4, 4, 1) RQ_XB(4, 5, 2)
    RQ_XB(12, 4, 2) RQ_XB(16, 5, 1) RQ_XBP(8, 5, 2) RQ_XBP(8, 5, 1) RQ_XBP(16, 5, 2) RQ_XBP(8, 6, 2)
#endif
#undef RQ_XB
#undef RQ_XBP
    return (int)hipErrorInvalidValue;
}

// ------------------------------ decode: per-block GF(256) solve ------------------------------
// M[j][k] = mrep[uidx_j][e_k] (received repair j, erased source e_k); Gauss-Jordan on [M | I]
// (replaces GaussianElimination, RQ/discmath/gauss.go:7-45, on the e erased columns only):
// rank e <=> the reference's system is full rank.
// Output: X (e x e) and the e received repairs it combines: x_k = sum_m X[k][m] s_{piv[m]}, stored
// as xcoef[m * xc_stride + k] (one uniform 64-byte row per m for k_apply's scalar loads).
// The general algorithm on one block (k_solve's per-block body; the first solver runs it in place of a
// deferral when inline_general is set): `ws` is an LDS working set of solve_ws_bytes(e) bytes, used when
// e <= lds_e (else the block's global workspace); ex / lg the GF(256) tables in LDS; piv one LDS int.
// Every thread of the workgroup calls it (barriers inside).
__device__ __forceinline__ void general_block(const SolveArgs& a, uint32_t bi, uint32_t b, uint8_t* ws, const uint8_t* ex,
                              const uint8_t* lg, int* piv, uint32_t tid, uint32_t nthr) {
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    const uint32_t W2 = basis_width(e);
    // v (W2) | coefficient of v on each basis row (e) | pc (e x u16) | rowid (e x u16) | basis (e x W2):
    // in LDS for e <= lds_e, else in this block's global workspace (solve_ws_bytes(e))
    uint8_t* v = (e <= a.lds_e) ? ws : a.gws + 64ull * a.goff[bi];
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
        if (tid == 0) *piv = (int)e;
        __syncthreads();
        // v ^= sum_i cf[i] * basis_i (basis rows vanish on each other's pivot columns)
        for (uint32_t c = tid; c < W2; c += nthr) {
            uint8_t x = v[c];
            for (uint32_t i = 0; i < np; ++i) {
                const uint8_t f = cf[i];
                if (f) x ^= gm(f, A[(size_t)i * W2 + c]);
            }
            v[c] = x;
            if (c < e && x) atomicMin(piv, (int)c);
        }
        __syncthreads();
        const uint32_t p = (uint32_t)*piv;
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
        if (a.xb_on)
            gi_stream<8, 5, 2>(a.xb, bi, b, e, false, tid, nthr, [](uint32_t, uint32_t) { return 0u; },
                               [](uint32_t) { return 0u; });
        return;
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
#ifdef RQHIP_EXPERIMENTS
    if (a.sx_wgs && a.inline_general && a.row_margin && !(a.sx_pol & 16)) {
        // the first solver launch's syndrome workgroups XOR the first e + margin received rows (sx_rows);
        // a pivot row past them is XORed here (rows disjoint from theirs, so no race)
        typedef uint32_t V4 __attribute__((ext_vector_type(4)));
        const uint32_t xc = min(nr, e + a.row_margin), T = a.xb.T, cpr = T >> 4;
        const uint8_t* rv = a.xb.recv + (size_t)a.rep_off[b] * T;
        uint8_t* rz = const_cast<uint8_t*>(a.xb.r0) + (size_t)b * a.xb.n_union * T;
        for (uint32_t m = 0; m < e; ++m) {
            const uint32_t j = rowid[m];
            if (j < xc) continue;
            const V4* pv = reinterpret_cast<const V4*>(rv + (size_t)j * T);
            V4* pz = reinterpret_cast<V4*>(rz + (size_t)U[j] * T);
            for (uint32_t c = tid; c < cpr; c += nthr) pz[c] = pv[c] ^ pz[c];
        }
    }
#endif
    if (a.xb_on) {  // the apply's stream from the X just written (visible to the workgroup after the barrier)
        __syncthreads();
        gi_stream<8, 5, 2>(a.xb, bi, b, e, true, tid, nthr, [&](uint32_t k, uint32_t m) { return (uint32_t)xc[(size_t)m * xs + k]; },
                           [&](uint32_t m) { return (uint32_t)XP[m]; });
    }
}

#ifdef RQHIP_EXPERIMENTS
// Experiments library only (RQHIP_APPLY_SX=1; measured not to pay).
// The syndromes for the register-table apply (SolveArgs::sx_wgs): workgroup w of nwk XORs every received
// repair row of blocks bi = w, w + nwk, ... of the solve list into its r0 row, in place (a block's rows are
// distinct r0 rows), so that the r0 rows hold s = received ^ r0.  A block's rows are one flat range of
// 16-byte pieces (row j, piece c), dealt to the threads 256 at a time, U steps in flight per thread (the
// loads of all U before any store); the rows' r0 positions are staged in LDS (ru, cap entries).  T is a
// multiple of 16 and the received rows 16-byte aligned (the host checks both).  No solver reads the
// syndrome rows, so this runs beside them in the same launch, on the wave slots they leave free.
template <uint32_t NT, uint32_t U>
__device__ __forceinline__ void sx_rows(const SolveArgs& a, uint32_t w, uint32_t nwk, uint32_t tid, uint32_t* ru,
                                        uint32_t cap) {
    typedef uint32_t V4 __attribute__((ext_vector_type(4)));
    const XbitsArgs& x = a.xb;
    const uint32_t T = x.T, cpr = T >> 4, dq = NT / cpr, dr = NT % cpr;
    const uint32_t pol = a.sx_pol;  // experiments: 1 non-temporal stores, 2 non-temporal received-row loads
    // (timing only, wrong bytes: 4 no work at all, 8 the loads without the stores)
    if (pol & 4) return;
    for (uint32_t bi = w; bi < a.n_map; bi += nwk) {
        const uint32_t b = a.blk_map[bi];
        // the rows a solver may pivot on: with inline_general the first solver finishes every block, on its
        // first e + margin rows (general_block XORs any later pivot row itself); else every received row
        const uint32_t nr = a.inline_general && a.row_margin && !(pol & 16)
                                ? min(a.rep_cnt[b], a.erased_off[b + 1] - a.erased_off[b] + a.row_margin)
                                : a.rep_cnt[b];
        const uint8_t* rv = x.recv + (size_t)a.rep_off[b] * T;
        uint8_t* rz = const_cast<uint8_t*>(x.r0) + (size_t)b * x.n_union * T;
        const uint32_t* RU = a.rep_uidx + a.rep_off[b];
        const bool staged = nr <= cap;
        __syncthreads();  // the previous block's readers of ru are done
        if (staged)
            for (uint32_t i = tid; i < nr; i += NT) ru[i] = RU[i];
        __syncthreads();
        const uint32_t n = nr * cpr;
        uint32_t j = tid / cpr, c = tid - j * cpr;  // piece tid: row j, piece c
        for (uint32_t i0 = tid; i0 < n; i0 += U * NT) {
            V4 v[U], u[U];
            uint32_t off[U];
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) {
                const bool on = i0 + k * NT < n;
                off[k] = on ? (staged ? ru[j] : RU[j]) * T + 16 * c : 0u;
                if (on) {
                    const V4* pv = reinterpret_cast<const V4*>(rv + (size_t)j * T + 16 * c);
                    v[k] = (pol & 2) ? __builtin_nontemporal_load(pv) : *pv;
                    u[k] = *reinterpret_cast<const V4*>(rz + off[k]);
                }
                c += dr;
                j += dq;
                if (c >= cpr) { c -= cpr; ++j; }
            }
#pragma unroll
            for (uint32_t k = 0; k < U; ++k)
                if (i0 + k * NT < n) {
                    V4* q = reinterpret_cast<V4*>(rz + off[k]);
                    if (pol & 8) {
                        if ((v[k] ^ u[k]).x == 0x5eed5eedu && (v[k] ^ u[k]).y == 0x5eed5eedu) *q = v[k];
                    } else if (pol & 1) __builtin_nontemporal_store(v[k] ^ u[k], q);
                    else *q = v[k] ^ u[k];
                }
        }
    }
}
#endif

// The shipped solvers are k_solve_pq<1, 4> (e <= 64), k_solve_pq<2, 4> (e <= 128) and k_solve (any e);
// the variants measured slower live in rq_kernels_exp.hip (experiments builds only).
//
// Four waves per block, RPL rows per lane (lane j of every wave holds received repairs j + 64q as LDS
// rows: e coefficient bytes, then the identity part at byte e + row); each step picks the lowest unused
// row with a nonzero coefficient (ballot) and every other row folds c_j = f_j / f_p times the pivot
// row in (GF(256) multiplication by three v_perm lookups against c_j's tables, the pivot row's dwords
// made scalar so the selectors are SGPRs).  Round-2 k_solve_pm with a shorter dependent chain per pivot step: each wave issues the loads of its
// row quads for the step (at most QW per row) at the step's start, reads pinfo[f] of its own
// coefficient (log f, and the pivot-lane coefficient's log) instead of lg[f] after pinfo[f_p] (f_p's
// log is then a v_readlane of the pivot lane's entry), and loads all its pivot-row quads at once: a
// step is three dependent LDS round trips (f, pinfo[f], the tables) plus the barrier, where the
// quad-at-a-time loop had two more per quad.
// PF (experiments, RQHIP_SOLVE_PF=1): the column buffer carries each row's pinfo word instead of its
// coefficient byte, looked up by the wave that writes it while it updates its other quads, so a step
// starts one dependent LDS round trip later in its chain.
// RR (RPL = 1): the rows stay in registers across the steps -- wave g owns quads g, g + NW, ... of every
// row for the whole solve (quads below the step's column are final and skipped, as the shifting
// assignment skips them) -- and the pivot row's dwords are v_readlane'd from lane p: no row quad
// goes through LDS per step (RR's rows are written back once, after the last step, for X).
// SV (shipped, round 6): the pivot row's dwords stay in VGPRs and the v_perm selectors are formed by the
// VALU (five per dword) instead of by the CU's one scalar unit after a v_readfirstlane: a step's scalar
// instructions are shared by the CU's sixteen waves, its vector ones by a SIMD's four.  68.0 -> 66.1 us
// (profiles/r06_solve/sv); SV = false is the experiments library's RQHIP_SOLVE_SV=0.
template <int RPL, int NW, bool PF = false, bool RR = false, bool SV = true>
__global__ void __launch_bounds__(64 * NW) k_solve_pq(SolveArgs a) {
    static_assert(!RR || (RPL == 1 && !PF), "RR: one row per lane, coefficient-byte column buffer");
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
    __shared__ int gpiv;  // general_block's pivot (inline_general)
    static_assert(NROWS * SW * 4 >= 128 + 64 + 4 * 64 + 64 * 128, "general_block's working set for e <= 64 fits the rows");
    // g made scalar: the per-step quad choice and its branches are then wave-uniform SALU, not exec-masked
    // VALU (the compiler cannot prove tid >> 6 uniform)
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef RQHIP_SOLVE_STAMPS
    // built with -DRQHIP_SOLVE_STAMPS (experiments only: device printf slows every solver launch ~2x even
    // when it prints nothing), RQHIP_SOLVE_DIAG bit 16: phase stamps (100 MHz clock) of every 256th
    // block's first thread
    const bool stamp = (a.diag & 16) && blockIdx.x % 256 == 0 && tid == 0;
    uint64_t t_0 = stamp ? __builtin_amdgcn_s_memrealtime() : 0, t_1 = 0, t_2 = 0;
#endif
    if (a.status_init)
        for (uint32_t i = blockIdx.x * NT + tid; i < a.n_all; i += gridDim.x * NT)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
#ifdef RQHIP_EXPERIMENTS
    if constexpr (RPL == 1 && !PF && !RR) {
        if (a.sx_wgs && blockIdx.x >= gridDim.x - a.sx_wgs) {  // the syndrome workgroups
            sx_rows<NT, 4>(a, blockIdx.x - (gridDim.x - a.sx_wgs), a.sx_wgs, tid, rows, NROWS * SW);
            return;
        }
    }
#endif
    const uint32_t b = a.blk_map[blockIdx.x];
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
#ifdef RQHIP_SOLVE_STAMPS
    if (stamp) t_1 = __builtin_amdgcn_s_memrealtime();
#endif
    bool used[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) used[q] = lane + 64 * q >= nrow;
    uint64_t usedm[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) usedm[q] = __ballot(used[q]);
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    const uint32_t ksteps = a.diag_steps ? min(e, a.diag_steps) : e;
    const bool inl = RPL == 1 && a.inline_general != 0;
    // No pivot left (uniform over the block): rank-deficient on these rows.  With more received repairs
    // the block is deferred to the later solvers, or (inline_general) finished here with all of them;
    // otherwise final (status 0: the apply skips it).
    auto no_pivot = [&]() {
        if (nr > nrow && inl) {
            __syncthreads();  // every wave is done with the rows (general_block's working set)
            general_block(a, blockIdx.x, b, reinterpret_cast<uint8_t*>(rows), ex, lg, &gpiv, tid, NT);
            if (tid == 0 && a.host_status) a.host_status[b] = a.status[b];
            return;
        }
        if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
        if (tid == 0 && inl && a.host_status) a.host_status[b] = 0;
        if (a.xb_on && nr <= nrow)  // final: the apply skips it (a deferred block's solver writes its part)
            gi_stream<8, 5, 2>(a.xb, blockIdx.x, b, e, false, tid, NT, [](uint32_t, uint32_t) { return 0u; },
                               [](uint32_t) { return 0u; });
    };
    if constexpr (RR) {
        constexpr uint32_t QR = (8 + NW - 1) / NW;  // quads per row this wave owns
        uint4* myrow = reinterpret_cast<uint4*>(rows + lane * SW);
        uint4 R[QR];
#pragma unroll
        for (int j = 0; j < (int)QR; ++j) R[j] = myrow[min(g + NW * j, 8u)];
        bool used0 = used[0];
        for (uint32_t k = 0; k < ksteps; ++k) {
            const uint32_t f = fcol[k & 1][lane];
            const uint32_t pif = pinfo[f];
            const uint64_t bal = __ballot(f != 0 && !used0);
            if (!bal) {  // uniform over the block: every wave saw the same rows
                no_pivot();
                return;
            }
            const uint32_t p = (uint32_t)__ffsll((unsigned long long)bal) - 1;
            const bool piv = lane == p;
            used0 = used0 || piv;
            if (tid == 0) pivl[k] = (uint8_t)p;
            const uint32_t pip = __builtin_amdgcn_readlane(pif, p);
            const uint32_t ilgp = 255u - (pip & 0xFFu);
            const bool act = piv ? ((pif >> 16) & 1u) != 0 : f != 0;
            const uint32_t l = piv ? (pif >> 8) & 0xFFu : (pif & 0xFFu) + ilgp;  // < 510
            const uint4 A = tlA[l];
            const uint32_t B = tlB[l];
            const uint32_t kq = k >> 4, kn = k + 1;
#pragma unroll
            for (int j = 0; j < (int)QR; ++j) {
                const uint32_t w = g + NW * j;
                if (w >= q1 || w < kq) continue;  // wave-uniform
                const uint32_t px = __builtin_amdgcn_readlane(R[j].x, p), py = __builtin_amdgcn_readlane(R[j].y, p);
                const uint32_t pz = __builtin_amdgcn_readlane(R[j].z, p), pw = __builtin_amdgcn_readlane(R[j].w, p);
                uint4 r = R[j];
                r.x ^= perm_mul(A, B, px);
                r.y ^= perm_mul(A, B, py);
                r.z ^= perm_mul(A, B, pz);
                r.w ^= perm_mul(A, B, pw);
                if (act) R[j] = r;
                if (kn < ksteps && w == (kn >> 4)) {  // wave-uniform: this wave owns column k + 1
                    const uint32_t d = (kn >> 2) & 3u;
                    const uint32_t dw = d == 0 ? R[j].x : d == 1 ? R[j].y : d == 2 ? R[j].z : R[j].w;
                    fcol[kn & 1][lane] = (FC)((dw >> ((kn & 3u) * 8)) & 0xFFu);
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < (int)QR; ++j)
            if (g + NW * j <= 8u) myrow[g + NW * j] = R[j];
        __syncthreads();
    } else
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
#ifdef RQHIP_EXPERIMENTS
            if (a.diag & 1)
                for (int q = 0; q < RPL; ++q) pif[q] = f[q] | 0x10100u;
#endif
        }
        uint32_t p = 0xFFFFFFFFu;
#pragma unroll
        for (int q = RPL - 1; q >= 0; --q) {  // (the used rows as a scalar mask: no per-lane flag to test)
            const uint64_t bal = __ballot(f[q] != 0) & ~usedm[q];
            if (bal) p = 64 * q + (uint32_t)__ffsll((unsigned long long)bal) - 1;
        }
        if (p == 0xFFFFFFFFu) {  // uniform over the block: every wave saw the same rows
            no_pivot();
            return;
        }
        usedm[p >> 6] |= 1ull << (p & 63u);
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
            uint32_t l = piv ? (pif[q] >> 8) & 0xFFu : (pif[q] & 0xFFu) + ilgp;  // < 510
#ifdef RQHIP_EXPERIMENTS
            if (a.diag & 4) l = lane;
#endif
            A[q] = tlA[l];
            B[q] = tlB[l];
        }
        // columns < k are zero in the pivot row (all are earlier pivot columns): quads from k/16
        const uint32_t kn = k + 1;  // the column the next step reads
#pragma unroll
        for (int j = 0; j < (int)QW; ++j) {
            const uint32_t w = w0 + NW * j;
            if (w >= q1) break;
            uint32_t px, py, pz, pw;
            bool pzero;
            if constexpr (SV) {
                // the quad as VGPRs the compiler may not move to SGPRs (an empty asm makes them divergent)
                px = P[j].x; py = P[j].y; pz = P[j].z; pw = P[j].w;
                asm volatile("" : "+v"(px), "+v"(py), "+v"(pz), "+v"(pw));
                pzero = __builtin_amdgcn_readfirstlane(px | py | pz | pw) == 0u;
            } else {
                px = __builtin_amdgcn_readfirstlane(P[j].x); py = __builtin_amdgcn_readfirstlane(P[j].y);
                pz = __builtin_amdgcn_readfirstlane(P[j].z); pw = __builtin_amdgcn_readfirstlane(P[j].w);
                // a pivot-row quad of zeros leaves every row's quad as it is (the identity part of the pivot
                // row is zero beyond the rows folded into it so far): a scalar branch skips its updates
                pzero = (px | py | pz | pw) == 0u;
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                uint4 r = R[q][j];
                if (!pzero) {
#ifdef RQHIP_EXPERIMENTS
                if (a.diag & 8) {
                    r.x ^= px; r.y ^= py; r.z ^= pz; r.w ^= pw;
                } else
#endif
                {
                r.x ^= perm_mul(A[q], B[q], px);
                r.y ^= perm_mul(A[q], B[q], py);
                r.z ^= perm_mul(A[q], B[q], pz);
                r.w ^= perm_mul(A[q], B[q], pw);
                }
                if (act[q]) reinterpret_cast<uint4*>(rows + (lane + 64 * q) * SW)[w] = r;
                }
                if (kn < ksteps && w == (kn >> 4)) {  // wave-uniform: this wave owns column k + 1
                    // the dword first (d is uniform: a scalar branch), then the updated or old value
                    const uint32_t d = (kn >> 2) & 3u;
                    uint32_t dn, dold;
                    if (d == 0) { dn = r.x; dold = R[q][j].x; }
                    else if (d == 1) { dn = r.y; dold = R[q][j].y; }
                    else if (d == 2) { dn = r.z; dold = R[q][j].z; }
                    else { dn = r.w; dold = R[q][j].w; }
                    const uint32_t fb = ((act[q] ? dn : dold) >> ((kn & 3u) * 8)) & 0xFFu;
                    fcol[kn & 1][lane + 64 * q] = PF ? (FC)pinfo[fb] : (FC)fb;
                }
            }
        }
#ifdef RQHIP_EXPERIMENTS
        // issue-bound probe (bits 32 / 64): 32 dependent SALU / VALU instructions more per step, results
        // unused (what they cost says which issue unit binds the step)
        if (a.diag & 32) {
            uint32_t z = k;
#pragma unroll
            for (int t = 0; t < 32; ++t) asm volatile("s_add_u32 %0, %0, 1" : "+s"(z));
        }
        if (a.diag & 64) {
            uint32_t z = lane;
#pragma unroll
            for (int t = 0; t < 32; ++t) asm volatile("v_add_u32_e32 %0, 1, %0" : "+v"(z));
        }
#endif
        __syncthreads();
    }
    if (ksteps < e) {  // diagnostic step limit (timing only): valid pivot rows, meaningless X
        __syncthreads();
        for (uint32_t m = ksteps + tid; m < e; m += NT) pivl[m] = (uint8_t)m;
        __syncthreads();
    }
#ifdef RQHIP_SOLVE_STAMPS
    if (stamp) t_2 = __builtin_amdgcn_s_memrealtime();
#endif
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    if (a.xb_on) {  // the register-table apply's stream straight from the rows: X[k][m] = row pivl[k], column e + pivl[m]
        gi_stream<8, 5, 2>(a.xb, blockIdx.x, b, e, true, tid, NT,
                           [&](uint32_t k, uint32_t m) { return (uint32_t)rb[pivl[k] * SW * 4 + e + pivl[m]]; },
                           [&](uint32_t m) { return (uint32_t)pivl[m]; });
    } else {
        for (uint32_t m = g; m < e; m += NW) {  // wave g writes rows m = g, g + NW, ... (no index division)
            const uint32_t pm = pivl[m];
            for (uint32_t k = lane; k < e; k += 64) xc[m * xs + k] = rb[pivl[k] * SW * 4 + e + pm];
        }
    }
    if (tid == 0) a.status[b] = 1;
    if (tid == 0 && inl && a.host_status) a.host_status[b] = 1;
#ifdef RQHIP_SOLVE_STAMPS
    if (stamp) {
        const uint64_t t_3 = __builtin_amdgcn_s_memrealtime();
        printf("[solve-stamp] block %u e %u setup %llu loop %llu out %llu (10 ns ticks)\n", blockIdx.x, e,
               (unsigned long long)(t_1 - t_0), (unsigned long long)(t_2 - t_1), (unsigned long long)(t_3 - t_2));
    }
#endif
}



#ifdef RQHIP_EXPERIMENTS
// Experiments library only (rq_debug_solve_mode(1)): measured no faster than k_solve_pq<1, 4>.
// The same solve in place (e <= 64 on the first e + margin received repairs): a row holds only its e
// coefficient bytes, and the column eliminated at step k is reused for the identity column of that step's
// pivot row (the classic in-place Gauss-Jordan inverse).  After step k, byte k of row j holds c_j =
// f_j / f_p (the multiple of pivot row p it took) and byte k of the pivot row 1 / f_p, so at the end row
// pivl[k] byte m = X[k][m].  Every step updates all of a row's live quads (the identity columns keep
// changing), but rows are e bytes wide instead of e + e + margin: ceil(e / 16) quads, one per wave.
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_solve_ip(SolveArgs a) {
    constexpr uint32_t NT = 64 * NW, NROWS = 64, SW = 20;  // rows, row stride (dwords: 16 + 4 against bank conflicts)
    static_assert(NW == 4, "one 16-byte quad of each row per wave");
    __shared__ __attribute__((aligned(16))) uint32_t rows[NROWS * SW];
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[NROWS];
    __shared__ uint32_t Es[NROWS];
    __shared__ __attribute__((aligned(16))) uint4 tlA[510];
    __shared__ uint32_t tlB[510];
    __shared__ uint32_t pinfo[256];
    __shared__ uint8_t fcol[2][NROWS];
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    if (a.status_init)
        for (uint32_t i = blockIdx.x * NT + tid; i < a.n_all; i += gridDim.x * NT)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > NROWS) {
        if (tid == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = a.row_margin ? min(min(nr, NROWS), e + a.row_margin) : min(nr, NROWS);
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
    if (lane < nrow) gather_row<NW>(reinterpret_cast<uint8_t*>(rows + lane * SW), a.mrep + (size_t)U[lane] * a.mrep_stride, Es, e, g);
    for (uint32_t x = tid; x < 256; x += NT) {  // as k_solve_pq: log f | log(1 ^ 1/f) << 8 | (1 ^ 1/f != 0) << 16
        uint32_t v = 0;
        if (x) {
            const uint32_t lx = lg[x], cp = 1u ^ ex[255u - lx];
            v = lx | (cp ? (uint32_t)lg[cp] << 8 | 1u << 16 : 0u);
        }
        pinfo[x] = v;
    }
    __syncthreads();
    for (uint32_t r = tid; r < NROWS; r += NT) fcol[0][r] = (uint8_t)(rows[r * SW] & 0xFFu);
    __syncthreads();
    const uint32_t q1 = (e + 15) >> 4;  // quads holding the e columns
    bool used = lane >= nrow;
    uint4* myq = reinterpret_cast<uint4*>(rows + lane * SW) + g;
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    for (uint32_t k = 0; k < e; ++k) {
        const uint4 R = *myq;  // this wave's quad of the lane's row (quads past q1 stay zero)
        const uint32_t f = fcol[k & 1][lane];
        const uint32_t pif = pinfo[f];
        const uint64_t bal = __ballot(f != 0 && !used);
        if (!bal) {  // uniform over the block
            if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            return;
        }
        const uint32_t p = (uint32_t)__ffsll((unsigned long long)bal) - 1;
        const bool piv = lane == p;
        used |= piv;
        if (tid == 0) pivl[k] = (uint8_t)p;
        const uint4 P = reinterpret_cast<const uint4*>(rows + p * SW)[g];
        const uint32_t pip = __builtin_amdgcn_readlane(pif, p);
        const uint32_t ilgp = 255u - (pip & 0xFFu);
        // c_j = f_j / f_p; the pivot lane 1 ^ 1 / f_p, which leaves row_p / f_p
        const bool act = piv ? ((pif >> 16) & 1u) != 0 : f != 0;
        const uint32_t l = piv ? (pif >> 8) & 0xFFu : (pif & 0xFFu) + ilgp;
        const uint4 A = tlA[l];
        const uint32_t B = tlB[l];
        const uint32_t kn = k + 1;
        if (g < q1) {
            const uint32_t px = __builtin_amdgcn_readfirstlane(P.x), py = __builtin_amdgcn_readfirstlane(P.y);
            const uint32_t pz = __builtin_amdgcn_readfirstlane(P.z), pw = __builtin_amdgcn_readfirstlane(P.w);
            uint4 r = R;
            r.x ^= perm_mul(A, B, px);
            r.y ^= perm_mul(A, B, py);
            r.z ^= perm_mul(A, B, pz);
            r.w ^= perm_mul(A, B, pw);
            if (g == (k >> 4)) {  // byte k: c_j (its identity entry for pivot p), or 1 / f_p on the pivot row
                const uint32_t cb = ((A.x >> 8) & 0xFFu) ^ (piv ? 1u : 0u), sh = (k & 3u) * 8, d = (k >> 2) & 3u;
                uint32_t& dw = d == 0 ? r.x : d == 1 ? r.y : d == 2 ? r.z : r.w;
                dw = (dw & ~(0xFFu << sh)) | (cb << sh);
            }
            if (act) *myq = r;
            if (kn < e && g == (kn >> 4)) {  // the next step's column, from this wave's registers
                const uint4 v = act ? r : R;
                const uint32_t d = (kn >> 2) & 3u;
                const uint32_t dw = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
                fcol[kn & 1][lane] = (uint8_t)((dw >> ((kn & 3u) * 8)) & 0xFFu);
            }
        }
        __syncthreads();
    }
    uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
    const uint32_t xs = x_stride(e);
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    for (uint32_t m = g; m < e; m += NW)
        for (uint32_t k = lane; k < e; k += 64) xc[m * xs + k] = rb[pivl[k] * SW * 4 + m];
    if (tid == 0) a.status[b] = 1;
}

// Experiments (RQHIP_SOLVE_IPX=1): k_solve_ip with round 6's first-solver changes -- scalar wave index,
// used rows as a scalar mask, v_perm selectors on the VALU, the apply's index stream written from the
// rows, and the general algorithm inline for a block rank-deficient on its first rows.  One quad of every
// row per wave (rows are e bytes wide), against two for k_solve_pq<1, 4>.
__global__ void __launch_bounds__(256) k_solve_ipx(SolveArgs a) {
    constexpr uint32_t NW = 4, NT = 64 * NW, NROWS = 64, SW = 20;
    // rows: 64 x 20 dwords, sized up to general_block's working set for e <= 64 (inline general)
    __shared__ __attribute__((aligned(16))) uint32_t rows[2176];
    static_assert(NROWS * SW <= 2176 && 2176 * 4 >= 128 + 64 + 4 * 64 + 64 * 128, "rows and general_block fit");
    __shared__ __attribute__((aligned(4))) uint8_t ex[512], lg[256];
    __shared__ uint8_t pivl[NROWS];
    __shared__ uint32_t Es[NROWS];
    __shared__ __attribute__((aligned(16))) uint4 tlA[510];
    __shared__ uint32_t tlB[510];
    __shared__ uint32_t pinfo[256];
    __shared__ uint8_t fcol[2][NROWS];
    __shared__ int gpiv;
    const uint32_t tid = threadIdx.x, lane = tid & 63, g = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (a.status_init)
        for (uint32_t i = blockIdx.x * NT + tid; i < a.n_all; i += gridDim.x * NT)
            if (a.status_init[i] != ST_PENDING) a.status[i] = a.status_init[i];
    const uint32_t b = a.blk_map[blockIdx.x];
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t nr = a.rep_cnt[b];
    if (e > NROWS) {
        if (tid == 0) a.status[b] = ST_FALLBACK;
        return;
    }
    const uint32_t nrow = a.row_margin ? min(min(nr, NROWS), e + a.row_margin) : min(nr, NROWS);
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
    if (lane < nrow) gather_row<NW>(reinterpret_cast<uint8_t*>(rows + lane * SW), a.mrep + (size_t)U[lane] * a.mrep_stride, Es, e, g);
    for (uint32_t x = tid; x < 256; x += NT) {
        uint32_t v = 0;
        if (x) {
            const uint32_t lx = lg[x], cp = 1u ^ ex[255u - lx];
            v = lx | (cp ? (uint32_t)lg[cp] << 8 | 1u << 16 : 0u);
        }
        pinfo[x] = v;
    }
    __syncthreads();
    for (uint32_t r = tid; r < NROWS; r += NT) fcol[0][r] = (uint8_t)(rows[r * SW] & 0xFFu);
    __syncthreads();
    const uint32_t q1 = (e + 15) >> 4;
    uint64_t usedm = __ballot(lane >= nrow);
    uint4* myq = reinterpret_cast<uint4*>(rows + lane * SW) + g;
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
    const bool inl = a.inline_general != 0;
    for (uint32_t k = 0; k < e; ++k) {
        const uint4 R = *myq;
        const uint32_t f = fcol[k & 1][lane];
        const uint32_t pif = pinfo[f];
        const uint64_t bal = __ballot(f != 0) & ~usedm;
        if (!bal) {  // uniform over the block: rank-deficient on these rows
            if (nr > nrow && inl) {
                __syncthreads();
                general_block(a, blockIdx.x, b, reinterpret_cast<uint8_t*>(rows), ex, lg, &gpiv, tid, NT);
                if (tid == 0 && a.host_status) a.host_status[b] = a.status[b];
                return;
            }
            if (tid == 0) a.status[b] = (nr > nrow) ? ST_FALLBACK : 0;
            if (tid == 0 && inl && a.host_status) a.host_status[b] = 0;
            if (a.xb_on && nr <= nrow)
                gi_stream<8, 5, 2>(a.xb, blockIdx.x, b, e, false, tid, NT, [](uint32_t, uint32_t) { return 0u; },
                                   [](uint32_t) { return 0u; });
            return;
        }
        const uint32_t p = (uint32_t)__ffsll((unsigned long long)bal) - 1;
        const bool piv = lane == p;
        usedm |= 1ull << p;
        if (tid == 0) pivl[k] = (uint8_t)p;
        uint4 P = reinterpret_cast<const uint4*>(rows + p * SW)[g];
        const uint32_t pip = __builtin_amdgcn_readlane(pif, p);
        const uint32_t ilgp = 255u - (pip & 0xFFu);
        const bool act = piv ? ((pif >> 16) & 1u) != 0 : f != 0;
        const uint32_t l = piv ? (pif >> 8) & 0xFFu : (pif & 0xFFu) + ilgp;
        const uint4 A = tlA[l];
        const uint32_t B = tlB[l];
        const uint32_t kn = k + 1;
        if (g < q1) {
            asm volatile("" : "+v"(P.x), "+v"(P.y), "+v"(P.z), "+v"(P.w));
            uint4 r = R;
            r.x ^= perm_mul(A, B, P.x);
            r.y ^= perm_mul(A, B, P.y);
            r.z ^= perm_mul(A, B, P.z);
            r.w ^= perm_mul(A, B, P.w);
            if (g == (k >> 4)) {  // byte k: c_j, or 1 / f_p on the pivot row
                const uint32_t cb = ((A.x >> 8) & 0xFFu) ^ (piv ? 1u : 0u), sh = (k & 3u) * 8, d = (k >> 2) & 3u;
                uint32_t& dw = d == 0 ? r.x : d == 1 ? r.y : d == 2 ? r.z : r.w;
                dw = (dw & ~(0xFFu << sh)) | (cb << sh);
            }
            if (act) *myq = r;
            if (kn < e && g == (kn >> 4)) {
                const uint4 v = act ? r : R;
                const uint32_t d = (kn >> 2) & 3u;
                const uint32_t dw = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
                fcol[kn & 1][lane] = (uint8_t)((dw >> ((kn & 3u) * 8)) & 0xFFu);
            }
        }
        __syncthreads();
    }
    uint16_t* XP = a.xpiv + a.erased_off[b];
    for (uint32_t m = tid; m < e; m += NT) XP[m] = pivl[m];
    if (a.xb_on) {
        gi_stream<8, 5, 2>(a.xb, blockIdx.x, b, e, true, tid, NT,
                           [&](uint32_t k, uint32_t m) { return (uint32_t)rb[pivl[k] * SW * 4 + m]; },
                           [&](uint32_t m) { return (uint32_t)pivl[m]; });
    } else {
        uint8_t* xc = a.xcoef + 64ull * a.xoff[blockIdx.x];
        const uint32_t xs = x_stride(e);
        for (uint32_t m = g; m < e; m += NW)
            for (uint32_t k = lane; k < e; k += 64) xc[m * xs + k] = rb[pivl[k] * SW * 4 + m];
    }
    if (tid == 0) a.status[b] = 1;
    if (tid == 0 && inl && a.host_status) a.host_status[b] = 1;
}
#endif

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
    general_block(a, bi, b, sm, ex, lg, &piv, tid, nthr);
    __syncthreads();  // the next block reuses the LDS
    }
    if (a.host_status) {  // this pass's blocks are final now (solved above, or by an earlier solver)
        const uint32_t bi = base + tid * gridDim.x;
        if (tid < 256 && bi < a.n_map) {
            const uint32_t b = a.blk_map[bi];
            a.host_status[b] = a.status[b];
        }
    }
    __syncthreads();  // todo / ntodo are rewritten by the next pass
    }
}

// k_solve's working set for e erased rows (LDS when e <= lds_e, else global workspace).
size_t solve_ws_bytes(uint32_t e) {
    const uint32_t W2 = basis_width(e);
    return W2 + ((e + 15) & ~15u) + 4 * ((e + 7) & ~7u) + (size_t)e * W2;
}

#ifdef RQHIP_EXPERIMENTS
// Experiments builds: the solver variants measured and not shipped (rq_kernels_exp.hip) behind knobs.
// RQHIP_SOLVE_PM=0: alpha-multiple tables (k_solve_fast) instead of GF(256) multiplication; RQHIP_SOLVE_LUT=0:
// per-step table builds (k_solve_pm<..., false>); RQHIP_SOLVE_PQ=0: k_solve_pm instead of k_solve_pq;
// RQHIP_SOLVE_PF=1: k_solve_pq's pinfo column buffer; RQHIP_SOLVE_LEAN=1: k_solve_lean; RQHIP_SOLVE_NW:
// waves per block (1, 2, 4, 8; 0 = k_solve_reg).  Measurements: profiles/r02ag, r02r, r03_solve2, r04j, r04l.
int launch_solve_exp_first(const SolveArgs& first, const SolveArgs& a, uint32_t n_blocks, bool pm, bool lut, bool pq,
                           bool lean, int nw, void* stream);
int launch_solve_exp_wide(const SolveArgs& a, uint32_t n_blocks, bool pm, bool lut, bool pq, void* stream);
static bool knob_on(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    return e ? e[0] != '0' : dflt;
}
static bool rr_knob() {
    static const bool r = knob_on("RQHIP_SOLVE_RR", false);
    return r;
}
static bool ipx_knob() {
    static const bool r = knob_on("RQHIP_SOLVE_IPX", false);
    return r;
}
static bool sv_knob() {
    static const bool r = knob_on("RQHIP_SOLVE_SV", true);
    return r;
}
#endif

// The first solve in place (k_solve_ip, experiments library) or on [M | I] (k_solve_pq<1, 4>);
// rq_debug_solve_mode switches it in experiments builds.
uint32_t g_solve_ip = 0;
#ifdef RQHIP_EXPERIMENTS
static bool solve_in_place() { return g_solve_ip != 0; }
#else
static bool solve_in_place() { return false; }
#endif

int launch_solve(const SolveArgs& a_in, uint32_t n_blocks, bool need_general, bool wide, uint32_t max_lds_e,
                 void* stream, bool* xbits_done, bool* sx_done) {
    // the first solver launch copies the host-decided statuses (a_in.status_init); later launches never do
    SolveArgs first = a_in;
    // the syndrome workgroups (a_in.sx_wgs) ride on the shipped first solver only (sx below)
    first.sx_wgs = 0;
    if (sx_done) *sx_done = false;
    // k_solve_pq and k_solve write the apply's stream themselves (xb_on); any other first solver writes X
    // only, and the caller runs k_xbits
    bool stream_ok = solve_in_place() == false;
#ifdef RQHIP_EXPERIMENTS
    stream_ok = stream_ok && !std::getenv("RQHIP_SOLVE_PM") && !std::getenv("RQHIP_SOLVE_LUT") &&
                !std::getenv("RQHIP_SOLVE_PQ") && !std::getenv("RQHIP_SOLVE_PF") && !std::getenv("RQHIP_SOLVE_LEAN") &&
                !std::getenv("RQHIP_SOLVE_NW");
#endif
    if (!stream_ok) first.xb_on = 0;
    if (xbits_done) *xbits_done = first.xb_on != 0;
    first.diag_steps = 0;
    first.diag = 0;
    // inline_general (no block with e > 64): the first solver finishes everything and writes the host
    // statuses; only the shipped k_solve_pq<1, 4> implements it
    first.inline_general = a_in.inline_general && !wide ? 1u : 0u;
    const hipStream_t st = (hipStream_t)stream;
#ifdef RQHIP_EXPERIMENTS
    static const uint32_t dsteps = [] { const char* e = std::getenv("RQHIP_SOLVE_STEPS"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    static const uint32_t sdiag = [] { const char* e = std::getenv("RQHIP_SOLVE_DIAG"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    first.diag_steps = dsteps;
    first.diag = sdiag;
#endif
    SolveArgs a = first;
    a.status_init = nullptr;
    a.inline_general = 0;
#ifdef RQHIP_EXPERIMENTS
    if (!stream_ok || rr_knob()) first.inline_general = 0;  // the variants defer as before
    static const bool pm = knob_on("RQHIP_SOLVE_PM", true), lut = knob_on("RQHIP_SOLVE_LUT", true),
                      pq = knob_on("RQHIP_SOLVE_PQ", true), pf = knob_on("RQHIP_SOLVE_PF", false),
                      lean = knob_on("RQHIP_SOLVE_LEAN", false), rr = rr_knob();
    static const int nw = [] { const char* e = std::getenv("RQHIP_SOLVE_NW"); return e ? std::atoi(e) : 4; }();
    // solvers that take `a` (statuses uploaded first): k_solve_fast and k_solve_reg
    const bool takes_a = !lean && ((nw == 1 && !pm) || (nw == 4 && !pm) || (nw != 1 && nw != 2 && nw != 4 && nw != 8));
    if (a_in.status_init && takes_a &&
        hipMemcpyAsync(a.status, a_in.status_init, (size_t)a_in.n_all * 4, hipMemcpyHostToDevice, st) != hipSuccess)
        return (int)hipGetLastError();
    int rx = launch_solve_exp_first(first, a, n_blocks, pm, lut, pq, lean, nw, stream);
    if (rx == -1) {
        if (nw == 1) hipLaunchKernelGGL((k_solve_pq<1, 1>), dim3(n_blocks), dim3(64), 0, st, first);
        else if (nw == 2) hipLaunchKernelGGL((k_solve_pq<1, 2>), dim3(n_blocks), dim3(128), 0, st, first);
        else if (nw == 8) hipLaunchKernelGGL((k_solve_pq<1, 8>), dim3(n_blocks), dim3(512), 0, st, first);
        else if (pf) hipLaunchKernelGGL((k_solve_pq<1, 4, true>), dim3(n_blocks), dim3(256), 0, st, first);
        else if (rr) hipLaunchKernelGGL((k_solve_pq<1, 4, false, true>), dim3(n_blocks), dim3(256), 0, st, first);
        else if (solve_in_place()) hipLaunchKernelGGL((k_solve_ip<4>), dim3(n_blocks), dim3(256), 0, st, first);
        else if (!sv_knob()) hipLaunchKernelGGL((k_solve_pq<1, 4, false, false, false>), dim3(n_blocks), dim3(256), 0, st, first);
        else if (ipx_knob()) hipLaunchKernelGGL(k_solve_ipx, dim3(n_blocks), dim3(256), 0, st, first);
        else {
            SolveArgs sx = first;
            sx.sx_wgs = a_in.sx_wgs;
            hipLaunchKernelGGL((k_solve_pq<1, 4>), dim3(n_blocks + sx.sx_wgs), dim3(256), 0, st, sx);
            if (sx_done) *sx_done = sx.sx_wgs != 0;
        }
        rx = (int)hipGetLastError();
    }
    if (rx != hipSuccess || !need_general || first.inline_general) return rx;
    if (wide) {  // blocks with 64 < e <= 128; the rare rank-deficient-on-64-rows block goes to k_solve
        int rw = launch_solve_exp_wide(a, n_blocks, pm, lut, pq, stream);
        if (rw == -1) {
            hipLaunchKernelGGL((k_solve_pq<2, 4>), dim3(n_blocks), dim3(256), 0, st, a);
            rw = (int)hipGetLastError();
        }
        if (rw != hipSuccess) return rw;
    }
#else
    // e <= 64 on the first e + margin received repairs (statuses copied in by this launch)
    hipLaunchKernelGGL((k_solve_pq<1, 4>), dim3(n_blocks), dim3(256), 0, st, first);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !need_general || first.inline_general) return (int)e;
    if (wide) {  // blocks with 64 < e <= 128; the rare rank-deficient-on-64-rows block goes to k_solve
        hipLaunchKernelGGL((k_solve_pq<2, 4>), dim3(n_blocks), dim3(256), 0, st, a);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
#endif
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
#ifndef RQHIP_EXPERIMENTS
    // the shipped shapes: syndromes in pairs, KC = 4 at four waves per SIMD, KC = 8 at three (under four's
    // 128 VGPRs the KC = 8 pair loop spills 11 at CPL 5: 170.9 against 177.1 us, profiles/r03_apply2/occ).
    // launch_apply's cap keeps kc at 4 or 8.
    static_assert(PD == 2 && KCMAX == 8, "release k_apply shape");
    if (kc <= 4) hipLaunchKernelGGL((k_apply<4, CPL, 2, OCC, true>), g, dim3(64), lds + 40 * 4, st, a, nu, np, mc);
    else hipLaunchKernelGGL((k_apply<8, CPL, 2, 3, true>), g, dim3(64), lds + 40 * 8, st, a, nu, np, mc);
#else
    // experiments: RQHIP_APPLY_PAIR=0 restores the one-syndrome-at-a-time loop, RQHIP_APPLY_PAIROCC=4 the
    // KC = 8 pair loop at four waves per SIMD, RQHIP_APPLY_KC the wider slices (KC 12..24)
    static const bool pair = [] { const char* e = std::getenv("RQHIP_APPLY_PAIR"); return !(e && e[0] == '0'); }();
    if constexpr (PD == 2 && KCMAX == 8) {
        if (pair && kc <= 4) {
            hipLaunchKernelGGL((k_apply<4, CPL, 2, OCC, true>), g, dim3(64), lds + 40 * 4, st, a, nu, np, mc);
            return;
        }
        if (pair && kc == 8) {
            static const bool occ4p = [] { const char* e = std::getenv("RQHIP_APPLY_PAIROCC"); return e && e[0] == '4'; }();
            if (occ4p) {
                hipLaunchKernelGGL((k_apply<8, CPL, 2, OCC, true>), g, dim3(64), lds + 40 * 8, st, a, nu, np, mc);
                return;
            }
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
#endif
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
    uint32_t cpl = 1;
#ifdef RQHIP_EXPERIMENTS
    // fewest padded columns, then the widest lanes (1, 2, 4 or 5 dword columns per lane)
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t c : {1u, 2u, 4u, 5u}) {
        const uint32_t w = 64 * c, pad = (Td + w - 1) / w * w - Td;
        if (pad <= best) { best = pad; cpl = c; }
    }
#endif
    // The release library runs k_apply only for the batches beyond the register-table apply's stream
    // bound (rq_engine.cpp gi_stream_fits: some block with e > 512) and rq_debug_apply_mode(0): one dword
    // column per lane.
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
#ifdef RQHIP_EXPERIMENTS
    switch (cpl) {
        case 1: launch_apply_pd<1>(a, kc, g, ec, lds, st, nu, np, MC); break;
        case 2: launch_apply_pd<2>(a, kc, g, ec, lds, st, nu, np, MC); break;
        case 4: launch_apply_pd<4>(a, kc, g, ec, lds, st, nu, np, MC); break;
        default: launch_apply_pd<5>(a, kc, g, ec, lds, st, nu, np, MC); break;
    }
#else
    launch_apply_pd<1>(a, kc, g, ec, lds, st, nu, np, MC);
#endif
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
