// rq_kernels_common.hpp -- device helpers shared by the shipped decode kernels (rq_kernels.hip) and the
// experiments-only solver variants (rq_kernels_exp.hip): GF(256) on packed dwords, the exp/log and v_perm
// coefficient tables, the solvers' row gather.  Device code only; the tables are internal to each
// translation unit (namespace-scope const).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rq_device.hpp"

namespace rq {

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

}  // namespace rq
