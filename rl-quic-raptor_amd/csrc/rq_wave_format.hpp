// rq_wave_format.hpp -- the per-wave instruction stream k_encode executes (shared by the host
// packer rq_wave.cpp, the kernel rq_kernels.hip and the Python emulator tests/plan_replay.py).
//
// A wave's stream is a sequence of 64-word pages; a page holds 8 groups of 8 words.  Words 0-3 of
// a group are read by lanes 0-31 (half A), words 4-7 by lanes 32-63 (half B), with one
// ds_read_b128 from a per-wave LDS ring that holds the current and the next page (refilled by
// LDS-DMA at each page switch).  Each op runs
// one statement per half side by side (XOR, MUL) or one statement on the whole wave (HORNER).
// Slot fields are LDS byte offsets of the slot row (slot * sd * 4) for the lane's half, so a
// source costs one add (lane column) and one ds_read_b32.
//
//   header group   A: [hdr, dstA, gA, 0]   B: [hdr, dstB, gB, 0]
//     hdr = type | flags | n << 16   (n = payload groups that follow)
//     g   = source row re-read from global memory (isi; 0xFFFFFFFF none), if FLAG_G
//   XOR payload    per group 4 source offsets per half; dst is a source when it accumulates,
//                  padding reads the zero slot.
//   MUL payload    per source two groups per half: [src, t0, t1, t2] [t3, t4, 0, 0] with the
//                  v_perm tables of its coefficient (rq_core.hpp gf_perm_tables)
//   HORNER         n groups of 8 column words (A: columns 0-3, B: 4-7), each
//                  off(18) | a << 18 | b << 22: t = alpha*t ^ y(off); partial[a] ^= t; partial[b] ^= t
//                  (a == b: nothing).  FLAG_HSTART zeroes t and the partials first; a piece
//                  without FLAG_HFINISH stores its partials to dst + h*sd*4 for the next piece of
//                  the chunk (same wave) to reload; FLAG_HFINISH is followed by one group of tau
//                  bytes (A words) and stores partial[h] ^ tau_h*t there (half B: trash slots).
//   END            FLAG_BARRIER: end of a dependency level (workgroup barrier);
//                  FLAG_ADVANCE: the stream continues at the start of the next page.
// An op never crosses a page; every page except the last ends with an END(ADVANCE) group.
#pragma once
#include <cstdint>

namespace rq {

constexpr uint32_t WV_PAGE = 64;                     // words per page
constexpr uint32_t WV_GROUP = 8;                     // words per group (4 per half)
constexpr uint32_t WV_GPP = WV_PAGE / WV_GROUP;      // groups per page
constexpr uint32_t WV_MAX_PIECE = WV_GPP - 1;        // groups of one op piece (an END must still fit)

constexpr uint32_t OP_XOR = 0, OP_MUL = 1, OP_HORNER = 4, OP_END = 7;
constexpr uint32_t FLAG_G = 1u << 5, FLAG_HSTART = 1u << 6, FLAG_HFINISH = 1u << 7;
constexpr uint32_t FLAG_BARRIER = 1u << 8, FLAG_ADVANCE = 1u << 9;
constexpr uint32_t WV_NO_ISI = 0xFFFFFFFFu;

}  // namespace rq
