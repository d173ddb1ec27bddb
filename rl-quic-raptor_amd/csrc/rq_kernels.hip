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

#include <algorithm>
#include <cstdint>

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
__device__ __forceinline__ uint32_t xtime4(uint32_t x) {
    const uint32_t hi = (x >> 7) & 0x01010101u;
    const uint32_t mask = (hi << 8) - hi;  // 0x00 / 0xFF per byte (no multiply)
    return ((x & 0x7F7F7F7Fu) << 1) ^ (mask & 0x1D1D1D1Du);
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

// ------------------------------ decode: zero the erased source rows --------------------------
// grid = (n erased rows), 64 threads: the syndrome pass reads erased rows as zero.
__global__ void __launch_bounds__(64) k_zero_rows(ZeroArgs a) {
    const uint32_t i = blockIdx.x;
    if (i >= a.n) return;
    uint8_t* row = a.data + (size_t)a.blk[i] * a.data_stride + (size_t)a.row[i] * a.T;
    uint32_t* r4 = reinterpret_cast<uint32_t*>(row);
    for (uint32_t c = threadIdx.x; c < a.T / 4; c += 64) r4[c] = 0;
}

int launch_zero_rows(const ZeroArgs& a, void* stream) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_zero_rows, dim3(a.n), dim3(64), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

// ------------------------------ decode: per-block GF(256) solve ------------------------------
// M[j][k] = mrep[uidx_j][e_k] (received repair j, erased source e_k); Gauss-Jordan on [M | I]
// (replaces GaussianElimination, RQ/discmath/gauss.go:7-45, on the e erased columns only):
// rank e <=> the reference's system is full rank.
// Output: X (e x e) and the e received repairs it combines: x_k = sum_m X[k][m] s_{piv[m]}.
__device__ __forceinline__ uint8_t gmul_t(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[lg[a] + lg[b]] : (uint8_t)0;
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
    const uint32_t* U = a.rep_uidx + a.rep_off[b];
    const uint32_t ws = e + nr;
    if (tid == 0) {
        uint32_t x = 1;
        for (int i = 0; i < 255; ++i) {
            ex[i] = (uint8_t)x; ex[i + 255] = (uint8_t)x; lg[x] = (uint8_t)i;
            x <<= 1; if (x & 0x100) x ^= 0x11D;
        }
        ex[510] = ex[0]; ex[511] = ex[1]; lg[0] = 0;
    }
    for (uint32_t r = tid; r < nr; r += nthr) rowid[r] = (uint16_t)r;
    for (uint32_t idx = tid; idx < nr * ws; idx += nthr) {
        const uint32_t j = idx / ws, k = idx - j * ws;
        sm[idx] = (k < e) ? a.mrep[(size_t)U[j] * a.mrep_stride + E[k]] : (uint8_t)(k - e == j);
    }
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
    // X as bit planes: xb[(kc * e + m) * 8 + bit] has bit k of X[64*kc + k][m]'s bit `bit`
    const uint32_t nkc = (a.max_e + 63) / 64;
    uint64_t* xb = a.xbits + (size_t)blockIdx.x * nkc * a.max_e * 8;
    uint16_t* XP = a.xpiv + (size_t)blockIdx.x * a.max_e;
    for (uint32_t m = tid; m < e; m += nthr) XP[m] = rowid[m];
    __syncthreads();
    for (uint32_t idx = tid; idx < ((e + 63) / 64) * e * 8; idx += nthr) {
        const uint32_t bt = idx & 7, m = (idx >> 3) % e, kc = (idx >> 3) / e;
        uint64_t w = 0;
        for (uint32_t k = 0; k < 64 && kc * 64 + k < e; ++k)
            w |= (uint64_t)((sm[(kc * 64 + k) * ws + e + rowid[m]] >> bt) & 1u) << k;
        xb[idx] = w;
    }
    if (tid == 0) a.status[b] = 1;
}

int launch_solve(const SolveArgs& a, uint32_t n_blocks, uint32_t lds_bytes, void* stream) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_solve, dim3(n_blocks), dim3(256), lds_bytes, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

// ------------------------------ decode: x_E = X * s ------------------------------------------
// grid = (strips of 64 dwords, solved blocks), one wave.  s_m = recv_{piv m} ^ r0_{piv m} (the
// syndrome, formed on the fly).  GF(256) by bit decomposition: for each source m the eight
// multiples alpha^b s_m are built by xtime and XORed into every output k whose coefficient has
// bit b set (uniform masks) -- 8 bitwise ops per mul-add, no tables.
constexpr uint32_t APPLY_KC = 64;  // outputs per pass (registers)

__global__ void __launch_bounds__(64) k_apply(ApplyArgs a) {
    const uint32_t b = a.blk_map[blockIdx.y];
    if (a.status[b] != 1) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t e = a.erased_off[b + 1] - a.erased_off[b];
    const uint32_t Td = a.T >> 2, c = blockIdx.x * 64 + lane;
    const bool live = c < Td;
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t nkc = (a.max_e + 63) / 64;
    const uint64_t* xb = a.xbits + (size_t)blockIdx.y * nkc * a.max_e * 8;
    const uint16_t* XP = a.xpiv + (size_t)blockIdx.y * a.max_e;
    const uint32_t r0b = a.rep_off[b];
    uint8_t* blk = a.data + (size_t)b * a.data_stride;
    for (uint32_t kc = 0; kc * APPLY_KC < e; ++kc) {
        const uint32_t k0 = kc * APPLY_KC, kn = min(APPLY_KC, e - k0);
        uint32_t acc[APPLY_KC];
#pragma unroll
        for (uint32_t k = 0; k < APPLY_KC; ++k) acc[k] = 0;
        for (uint32_t m = 0; m < e; ++m) {
            const uint32_t j = r0b + XP[m];
            uint32_t s = 0;
            if (live) {
                s = reinterpret_cast<const uint32_t*>(a.recv + (size_t)j * a.T)[c] ^
                    reinterpret_cast<const uint32_t*>(a.r0 + ((size_t)b * a.n_union + a.rep_uidx[j]) * a.T)[c];
            }
            const uint64_t* w = xb + ((size_t)kc * e + m) * 8;
#pragma unroll
            for (uint32_t bt = 0; bt < 8; ++bt) {
                const uint64_t wb = w[bt];
                const uint32_t lo = (uint32_t)wb, hi = (uint32_t)(wb >> 32);
#pragma unroll
                for (uint32_t k = 0; k < APPLY_KC; ++k) {
                    const uint32_t word = k < 32 ? lo : hi;
                    const uint32_t msk = 0u - ((word >> (k & 31)) & 1u);
                    acc[k] ^= s & msk;
                }
                s = xtime4(s);
            }
        }
        if (live)
            for (uint32_t k = 0; k < kn; ++k) reinterpret_cast<uint32_t*>(blk + (size_t)E[k0 + k] * a.T)[c] = acc[k];
    }
}

int launch_apply(const ApplyArgs& a, uint32_t n_strips, uint32_t n_blocks, uint32_t /*lds_bytes*/, void* stream) {
    hipLaunchKernelGGL(k_apply, dim3(n_strips, n_blocks), dim3(64), 0, (hipStream_t)stream, a);
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
