// rq_gistream.hpp -- the register-table apply's index stream for one block (GiLayout, rq_device.hpp).
// Host and device: the solvers and k_xbits write it on the GPU (rq_kernels.hip); rq_debug_gi_stream runs
// the same code on the host so the CPU tests can check every index number and offset it produces
// (tests/test_applygi.py), including for the blocks that end rank-deficient.
#pragma once
#include <cstddef>
#include <cstdint>

#include "rq_device.hpp"

namespace rq {

// One 16-byte store on the device (the stream's records are 16-byte aligned), four dword stores on the host.
__host__ __device__ inline void gi_put4(uint32_t* p, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
    *reinterpret_cast<uint4*>(p) = make_uint4(x, y, z, w);
#else
    p[0] = x; p[1] = y; p[2] = z; p[3] = w;
#endif
}

// One workgroup per block of the solve list: X (bytes, row m = syndrome in pivot order, byte k =
// output) becomes the dword stream of rq_device.hpp GiLayout: a header (status, e, the block's row
// bases), per slice of KC outputs their row offsets, per group of G syndromes their row offsets, and per
// slice, group and output the eight G-bit subsets idx_b = sum_t bit_b(X[k][G g + t]) << t, so that
// sum_m X[k][m] s_m = sum_b alpha^b sum_g Tab_g[idx_b], where Tab_g holds the 2^G XORs of group g's
// syndromes (the apply kernel, rq_applygi.cpp).  Unsolved blocks get a header with status 0 only.
// Block bi's part of the stream from X given as X(k, m) (coefficient byte of syndrome m in output k) and
// XP(m) (the received row, within the block, of syndrome m); nthr threads from tid.  An unsolved block
// (solved = false) gets its header only.
template <int KC, int G, int PDG, class XF, class PF, int PK = 0>
__host__ __device__ inline void gi_stream(const XbitsArgs& a, uint32_t bi, uint32_t b, uint32_t e, bool solved, uint32_t tid,
                          uint32_t nthr, XF X, PF XP) {
    const GiLayout& L = a.L;
    uint32_t* base = a.gi + (size_t)bi * L.block;
    const uint32_t ngr = (e + G - 1) / G, nsl = (e + KC - 1) / KC;
    if (tid < 16) {
        uint64_t v = 0;
        if (tid >= 4 && tid < 10) {
            const uint32_t w = (tid - 4) >> 1;
            const uint64_t addr = w == 0 ? (uint64_t)(a.recv + (size_t)a.rep_off[b] * a.T)
                                : w == 1 ? (uint64_t)(a.r0 + (size_t)b * a.n_union * a.T)
                                         : (uint64_t)(a.data + (size_t)b * a.data_stride);
            v = (tid & 1) ? addr >> 32 : addr & 0xFFFFFFFFu;
        }
        base[tid] = tid == 0 ? (uint32_t)solved : tid == 1 ? e : tid == 2 ? ngr : (uint32_t)v;
    }
    if (!solved) return;
    const uint32_t* E = a.erased + a.erased_off[b];
    const uint32_t* RU = a.rep_uidx + a.rep_off[b];
    const uint32_t T = a.T;
    for (uint32_t i = tid; i < nsl * 16; i += nthr) {
        const uint32_t sl = i >> 4, k = i & 15, ko = sl * KC + k;
        base[L.er + i] = (k < (uint32_t)KC && ko < e) ? E[ko] * T : 0u;
    }
    for (uint32_t i = tid; i < (ngr + PDG + 1) * 16; i += nthr) {
        const uint32_t q = i >> 4, w = i & 15, t = w >> 1, m = G * q + t;
        uint32_t v = 0;
        if (t < (uint32_t)G && m < e) {
            const uint32_t j = XP(m);
            v = (w & 1) ? RU[j] * T : j * T;
        }
        base[L.of + i] = v;
    }
    for (uint32_t i = tid; i < nsl * ngr * KC; i += nthr) {
        const uint32_t k = i % KC, r = i / KC, g = r % ngr, sl = r / ngr, ko = sl * KC + k;
        uint32_t x[G];
#pragma unroll
        for (int t = 0; t < G; ++t) {
            const uint32_t m = G * g + t;
            x[t] = (ko < e && m < e) ? (uint32_t)X(ko, m) : 0u;
        }
        uint32_t v[8];
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            uint32_t sb = 0;
#pragma unroll
            for (int t = 0; t < G; ++t) sb |= ((x[t] >> bit) & 1u) << t;
            v[bit] = sb;
        }
        if (PK) {  // two per dword: bits b = 2i (low half) and 2i + 1 (high half)
            uint32_t* d = base + L.ix + sl * L.ix_slice + g * 4 * KC + k * 4;
            gi_put4(d, v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
        } else {
            uint32_t* d = base + L.ix + sl * L.ix_slice + g * 8 * KC + k * 8;
            gi_put4(d, v[0], v[1], v[2], v[3]);
            gi_put4(d + 4, v[4], v[5], v[6], v[7]);
        }
    }
}

}  // namespace rq
