// rq_applygi.cpp -- the decode's apply, x_E = g_E ^ X s, as register-table lookups (gfx950 assembly).
//
// Replaces the byte-table mul-add of the reference's decoder (asmSSSE3MulAdd,
// RQ/discmath/optimizations.s:36-78, under GaussianElimination's row operations) for the e erased rows.
//
// X is per block (it depends on the erasure pattern), so every coefficient is wave-uniform and the
// product can be split by bits instead of by bytes:
//   sum_m X[k][m] s_m = sum_b alpha^b P[k][b],  P[k][b] = XOR of the s_m whose X[k][m] has bit b set.
// Syndromes are taken G at a time; the 2^G XORs of a group's syndromes are built once per wave (2^G - 1
// VOP2 XORs into a table of VGPRs), and each bit plane P[k][b] takes one table entry per group: the
// entry's number (the G-bit subset, k_xbits) is an SGPR, and the lookup is one VOP2 XOR whose first
// source is read through the VGPR index mode (s_set_gpr_idx_on / _idx; gfx950 has no v_movrels).  A
// mul-add of four bytes then costs 8/G lookups plus (2^G - 1)/(G KC) table XORs instead of three
// v_perm and 1.5 XOR3 (rq_kernels.hip k_apply); the eight planes of an output are folded by Horner's
// rule, seven alpha-multiplies, at the end.
//
// One wave per (solved block, slice of KC outputs, strip of 64 dword columns); grid (8, slices x strips,
// ceil(blocks / 8)), so a block's waves share an XCD (workgroups are dealt to the XCDs round-robin by
// linear id, x fastest) and its syndrome rows are read from HBM once.  The index dwords and syndrome row
// offsets arrive through scalar loads, two 16-dword pieces per wait (SMEM returns out of order, so each
// wait is lgkmcnt(0) and a load issued right after one has a whole pair of pieces to land).
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "rq_applygi.hpp"

namespace rq {

namespace {
struct Asm {
    std::string s;
    char buf[256];
    void line(const char* t) { s += '\t'; s += t; s += '\n'; }
    template <class... A>
    void f(const char* fmt, A... a) {
        std::snprintf(buf, sizeof buf, fmt, a...);
        line(buf);
    }
};
}  // namespace

bool gi_shape_ok(const GiShape& sh) {
    return sh.KC >= 4 && sh.KC <= 16 && sh.KC % (sh.PACK ? 8 : 4) == 0 && sh.G >= 4 && sh.G <= 6 && sh.PDG >= 1 &&
           sh.PDG <= 2 && sh.CPL >= 1 && sh.CPL <= 2 && sh.PACK <= 1 && sh.SX <= 1 && gi_vgprs(sh) <= 256;
}

// VGPRs: v0 lane (prologue only), v1 the lane's byte offset in a row (column c at + 256 c), the syndrome
// ring from v2 (per column, PDG slots of G received-row + G r0-row values, or of G syndromes with SX; v2..v7
// double as Horner temporaries at the end), per column a table of 2^G entries (entry 0 = 0), then per
// column the KC x 8 bit planes (plane 0 starts as g_E).
namespace {
uint32_t gi_tb(const GiShape& sh) { return (2 + (sh.SX ? 1 : 2) * sh.G * sh.PDG * sh.CPL + 3) & ~3u; }
}  // namespace

uint32_t gi_vgprs(const GiShape& sh) { return gi_tb(sh) + sh.CPL * ((1u << sh.G) + 8 * sh.KC); }

std::string gi_kernel_name(const GiShape& sh) {
    return "rq_apply_gi_k" + std::to_string(sh.KC) + "_g" + std::to_string(sh.G) + "_p" + std::to_string(sh.PDG) +
           "_c" + std::to_string(sh.CPL) + (sh.PACK ? "_x2" : "") + (sh.SX ? "_s" : "") + (sh.stpol ? "_st" + std::to_string(sh.stpol) : std::string()) + (sh.diag ? "_d" + std::to_string(sh.diag) : std::string());
}

std::string emit_apply_gi_asm(const GiShape& sh) {
    const uint32_t KC = sh.KC, G = sh.G, PDG = sh.PDG, CPL = sh.CPL, NT = 1u << G;
    const uint32_t RING = 2, TB = gi_tb(sh), AC = TB + CPL * NT, NV = gi_vgprs(sh);
    const uint32_t PK = sh.PACK, PAIRS = PK ? KC / 8 : KC / 4;  // 32 index dwords per pair of 16-dword pieces
    const uint32_t UNR = (PDG * PAIRS) % 2 ? 2 * PDG : PDG;  // groups per loop body: ring slots, and pieces A/B alternate
    const std::string kname = gi_kernel_name(sh);
    // ring slot (c, p): G received-row values (RA) then G r0-row values (RB); with SX only the G syndromes (RB)
    const uint32_t SX = sh.SX, RW = SX ? 1 : 2;
    auto RA = [&](uint32_t c, uint32_t p, uint32_t t) { return RING + (c * PDG + p) * RW * G + t; };
    auto RB = [&](uint32_t c, uint32_t p, uint32_t t) { return RING + (c * PDG + p) * RW * G + (SX ? 0 : G) + t; };
    auto TBC = [&](uint32_t c) { return TB + c * NT; };
    auto ACC = [&](uint32_t c, uint32_t k, uint32_t b) { return AC + (c * KC + k) * 8 + b; };
    // column c's memory operations: the row offset + 256 c, under column c's exec mask (s[96:97] for c = 1)
    auto col_exec = [&](Asm& a, uint32_t c, bool on) {
        if (c) a.line(on ? "s_mov_b64 exec, s[96:97]" : "s_mov_b64 exec, s[98:99]");
    };
    Asm a;
    a.s += "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.amdhsa_code_object_version 6\n\t.text\n";
    a.s += "\t.globl " + kname + "\n\t.p2align 8\n\t.type " + kname + ",@function\n" + kname + ":\n";
    // ---- prologue: which block / slice / column group, and whether it has work.  Round 1: the arguments;
    // round 2: the block's header, the slice's output rows and the first PDG groups' row offsets.
    a.line("s_load_dwordx8 s[8:15], s[0:1], 0x0");     // gi(8:9) block_bytes of_bytes ix_bytes ix_slice n_blocks T
    a.line("s_load_dwordx4 s[16:19], s[0:1], 0x20");   // strips nsg sg_magic ws
    a.line("v_lshrrev_b32_e32 v2, 6, v0");             // the wave within the workgroup
    a.line("v_and_b32_e32 v0, 63, v0");
    a.line("s_nop 4");                                 // VALU write -> v_readfirstlane of it
    a.line("v_readfirstlane_b32 s36, v2");
    a.line("s_waitcnt lgkmcnt(0)");
    a.line("s_lshl_b32 s33, s4, 3");
    a.line("s_add_u32 s33, s33, s2");                  // bi = z * 8 + x
    a.line("s_cmp_ge_u32 s33, s14");
    a.line("s_cbranch_scc1 .Lend");
    a.line("s_lshl_b32 s34, s3, 1");
    a.line("s_mul_hi_u32 s34, s34, s18");              // slice = y / nsg = (2y * ceil(2^31 / nsg)) >> 32
    a.line("s_mul_i32 s35, s34, s17");
    a.line("s_sub_u32 s35, s3, s35");                  // strip group
    a.line("s_mul_i32 s35, s35, s19");
    a.line("s_add_u32 s35, s35, s36");                 // strip: CPL x 64 dword columns
    a.line("s_cmp_ge_u32 s35, s16");
    a.line("s_cbranch_scc1 .Lend");
    // the lane's dword column(s); lanes past T / 4 run with exec off (column 1: its own mask s[96:97])
    a.f("s_lshl_b32 s36, s35, %u", CPL == 2 ? 7 : 6);
    a.line("v_add_u32_e32 v1, s36, v0");
    a.line("s_lshr_b32 s36, s15, 2");
    a.line("v_cmp_gt_u32_e64 s[42:43], s36, v1");
    a.line("s_and_b64 exec, exec, s[42:43]");
    if (CPL == 2) {
        a.line("s_sub_u32 s37, s36, 64");
        a.line("v_cmp_gt_i32_e64 s[96:97], s37, v1");  // (signed: T / 4 < 64 leaves it empty)
        a.line("s_and_b64 s[96:97], s[96:97], exec");
        a.line("s_mov_b64 s[98:99], exec");
    }
    a.line("v_lshlrev_b32_e32 v1, 2, v1");
    // the block's stream at gi + bi * block_bytes: offsets -> s[62:63], this slice's index records ->
    // s[44:45], its output rows -> s[60:61]
    a.line("s_mul_i32 s38, s33, s10");
    a.line("s_mul_hi_u32 s39, s33, s10");
    a.line("s_add_u32 s38, s8, s38");
    a.line("s_addc_u32 s39, s9, s39");                 // block base
    a.line("s_add_u32 s62, s38, s11");
    a.line("s_addc_u32 s63, s39, 0");
    a.line("s_mul_i32 s36, s34, s13");
    a.line("s_add_u32 s36, s36, s12");
    a.line("s_add_u32 s44, s38, s36");
    a.line("s_addc_u32 s45, s39, 0");
    a.line("s_lshl_b32 s36, s34, 6");
    a.line("s_add_u32 s36, s36, 64");
    a.line("s_add_u32 s60, s38, s36");
    a.line("s_addc_u32 s61, s39, 0");
    a.f("s_mul_i32 s43, s34, %u", KC);                 // k0
    a.line("s_load_dwordx16 s[64:79], s[38:39], 0x0");  // header
    a.line("s_load_dwordx16 s[80:95], s[60:61], 0x0");  // output rows
    for (uint32_t p = 0; p < PDG; ++p) a.f("s_load_dwordx16 s[%u:%u], s[62:63], 0x%x", 16 * p, 16 * p + 15, 64 * p);
    a.line("s_waitcnt lgkmcnt(0)");
    a.line("s_cmp_eq_u32 s64, 1");
    a.line("s_cbranch_scc0 .Lend");                    // not solved: the block keeps its bytes
    a.line("s_cmp_ge_u32 s43, s65");
    a.line("s_cbranch_scc1 .Lend");                    // no outputs in this slice
    a.line("s_sub_u32 s47, s65, s43");
    a.f("s_min_u32 s47, s47, %u", KC);                 // kn: outputs of this slice
    a.line("s_mov_b32 s46, s66");                      // ngr
    // buffer resources (num_records unbounded, as the HIP kernels' make_buffer_rsrc(p, 0, -1, 0x20000)):
    // the block's received repairs, its r0 rows, its data rows
    a.line("s_mov_b32 s48, s68");
    a.line("s_and_b32 s49, s69, 0xffff");
    a.line("s_mov_b32 s50, -1");
    a.line("s_mov_b32 s51, 0x20000");
    a.line("s_mov_b32 s52, s70");
    a.line("s_and_b32 s53, s71, 0xffff");
    a.line("s_mov_b32 s54, -1");
    a.line("s_mov_b32 s55, 0x20000");
    a.line("s_mov_b32 s56, s72");
    a.line("s_and_b32 s57, s73, 0xffff");
    a.line("s_mov_b32 s58, -1");
    a.line("s_mov_b32 s59, 0x20000");
    for (uint32_t c = 0; c < CPL; ++c) {
        a.f("v_mov_b32_e32 v%u, 0", TBC(c));
        for (uint32_t k = 0; k < KC; ++k)
            for (uint32_t b = 1; b < 8; ++b) a.f("v_mov_b32_e32 v%u, 0", ACC(c, k, b));
    }
    // g_E (the erased rows as they are) into plane 0; then the first PDG groups' syndrome rows
    for (uint32_t c = 0; c < CPL; ++c) {
        col_exec(a, c, true);
        for (uint32_t k = 0; k < KC; ++k)
            a.f("buffer_load_dword v%u, v1, s[56:59], s%u offen offset:%u", ACC(c, k, 0), 80 + k, 256 * c);
        for (uint32_t p = 0; p < PDG; ++p)
            for (uint32_t t = 0; t < G; ++t) {
                if (!SX) a.f("buffer_load_dword v%u, v1, s[48:51], s%u offen offset:%u", RA(c, p, t), 16 * p + 2 * t, 256 * c);
                a.f("buffer_load_dword v%u, v1, s[52:55], s%u offen offset:%u", RB(c, p, t), 16 * p + 2 * t + 1, 256 * c);
            }
        col_exec(a, c, false);
    }
    a.f("s_add_u32 s62, s62, 0x%x", 64 * PDG);
    a.line("s_addc_u32 s63, s63, 0");
    // C = s[32:43]: the offsets of the group PDG ahead; pieces A = s[0:31], B = s[64:95]
    auto load_c = [&]() {
        a.line("s_load_dwordx8 s[32:39], s[62:63], 0x0");
        if (2 * G > 8) a.line("s_load_dwordx4 s[40:43], s[62:63], 0x20");
        a.line("s_add_u32 s62, s62, 64");
        a.line("s_addc_u32 s63, s63, 0");
    };
    auto load_pair = [&](uint32_t buf) {
        a.f("s_load_dwordx16 s[%u:%u], s[44:45], 0x0", buf, buf + 15);
        a.f("s_load_dwordx16 s[%u:%u], s[44:45], 0x40", buf + 16, buf + 31);
        a.line("s_add_u32 s44, s44, 0x80");
        a.line("s_addc_u32 s45, s45, 0");
    };
    load_c();
    load_pair(0);
    if (sh.diag & 1) {  // no index loads: both pieces hold valid (stale) indices, never an address
        a.line("s_waitcnt lgkmcnt(0)");
        for (uint32_t r = 64; r < 96; r += 2) a.f("s_mov_b64 s[%u:%u], 0", r, r + 1);
    }
    // ---- the groups: UNR copies of the body (ring slot p = u mod PDG), each ending in the exit test
    const uint32_t loads_per_group = RW * G * CPL;
    a.s += ".Lgroup:\n";
    uint32_t pair_no = 0;  // pieces alternate A, B over the whole body
    for (uint32_t u = 0; u < UNR; ++u) {
        const uint32_t p = u % PDG;
        a.f("s_waitcnt vmcnt(%u)", loads_per_group * (PDG - 1));
        for (uint32_t c = 0; c < CPL; ++c) {
            for (uint32_t t = 0; t < G; ++t) {
                if (SX) a.f("v_mov_b32_e32 v%u, v%u", TBC(c) + (1u << t), RB(c, p, t));
                else a.f("v_xor_b32_e32 v%u, v%u, v%u", TBC(c) + (1u << t), RA(c, p, t), RB(c, p, t));
            }
            for (uint32_t i = 3; i < NT; ++i) {
                if ((i & (i - 1)) == 0) continue;
                const uint32_t lo = i & (0u - i);
                a.f("v_xor_b32_e32 v%u, v%u, v%u", TBC(c) + i, TBC(c) + (i ^ lo), TBC(c) + lo);
            }
        }
        a.line("s_waitcnt lgkmcnt(0)");  // C and this group's first pair
        if (!(sh.diag & 2))
            for (uint32_t c = 0; c < CPL; ++c) {  // the group PDG ahead into the slot just consumed
                col_exec(a, c, true);
                for (uint32_t t = 0; t < G; ++t) {
                    if (!SX) a.f("buffer_load_dword v%u, v1, s[48:51], s%u offen offset:%u", RA(c, p, t), 32 + 2 * t, 256 * c);
                    a.f("buffer_load_dword v%u, v1, s[52:55], s%u offen offset:%u", RB(c, p, t), 33 + 2 * t, 256 * c);
                }
                col_exec(a, c, false);
            }
        for (uint32_t j = 0; j < PAIRS; ++j, ++pair_no) {
            const uint32_t cur = (pair_no & 1) ? 64 : 0, nxt = (pair_no & 1) ? 0 : 64;
            if (!(sh.diag & 1)) {
                if (j == 0) load_c();
                else a.line("s_waitcnt lgkmcnt(0)");
                load_pair(nxt);
            }
            if (sh.diag & 4) continue;
            for (uint32_t q = 0; q < 32; ++q) {
                // unpacked: dword q = output 4j + q / 8, bit q % 8; packed: output 8j + q / 4, bits 2 (q % 4) + 0, 1
                const uint32_t k = PK ? 8 * j + q / 4 : 4 * j + q / 8, b = PK ? 2 * (q % 4) : q % 8;
                if (j == 0 && q == 0) a.f("s_set_gpr_idx_on s%u, gpr_idx(SRC0)", cur + q);
                else a.f("s_set_gpr_idx_idx s%u", cur + q);
                for (uint32_t c = 0; c < CPL; ++c) a.f("v_xor_b32_e32 v%u, v%u, v%u", ACC(c, k, b), TBC(c), ACC(c, k, b));
                if (PK) {  // the high half: S0[7:0] after the shift (the idx instruction reads only bits 7:0)
                    a.f("s_lshr_b32 s%u, s%u, 16", cur + q, cur + q);
                    a.f("s_set_gpr_idx_idx s%u", cur + q);
                    for (uint32_t c = 0; c < CPL; ++c)
                        a.f("v_xor_b32_e32 v%u, v%u, v%u", ACC(c, k, b + 1), TBC(c), ACC(c, k, b + 1));
                }
            }
        }
        if (!(sh.diag & 4)) a.line("s_set_gpr_idx_off");
        // issue probe (diag 8 / 16): 32 dependent scalar / vector instructions more per group, results unused
        // (s97 is free at CPL 1, v0 after the prologue)
        if ((sh.diag & 8) && CPL == 1)
            for (int t = 0; t < 32; ++t) a.line("s_add_u32 s97, s97, 1");
        if (sh.diag & 16)
            for (int t = 0; t < 32; ++t) a.line("v_add_u32_e32 v0, 1, v0");
        a.line("s_sub_u32 s46, s46, 1");
        a.line("s_cmp_eq_u32 s46, 0");
        a.line("s_cbranch_scc1 .Lepi");
    }
    a.line("s_branch .Lgroup");
    // ---- Horner: x = P7; x = alpha x ^ P_b for b = 6..0 (plane 0 holds g_E), three outputs at a time;
    // alpha * a ^ c in 5 VALU as in the column program (rq_colasm.cpp MI_XTX)
    a.s += ".Lepi:\n";
    a.line("s_waitcnt vmcnt(0) lgkmcnt(0)");
    a.line("s_mov_b32 s36, 0x090b080a");
    a.line("s_mov_b32 s37, 0xfefefefe");
    a.line("s_mov_b32 s38, 0x1d1d1d1d");
    std::vector<std::pair<uint32_t, uint32_t>> outs;  // (column, output)
    for (uint32_t c = 0; c < CPL; ++c)
        for (uint32_t k = 0; k < KC; ++k) outs.push_back({c, k});
    for (size_t o0 = 0; o0 < outs.size(); o0 += 3) {
        const uint32_t n = (uint32_t)std::min<size_t>(3, outs.size() - o0);
        auto P = [&](uint32_t u, uint32_t b) { return ACC(outs[o0 + u].first, outs[o0 + u].second, b); };
        for (int b = 6; b >= 0; --b) {
            for (uint32_t u = 0; u < n; ++u) a.f("v_lshlrev_b32_e32 v%u, 8, v%u", 2 + 2 * u, P(u, b + 1));
            for (uint32_t u = 0; u < n; ++u) a.f("v_perm_b32 v%u, v%u, v%u, s36", 2 + 2 * u, 2 + 2 * u, P(u, b + 1));
            for (uint32_t u = 0; u < n; ++u)
                a.f("v_bitop3_b32 v%u, v%u, v%u, s38 bitop3:0x6c", 2 + 2 * u, 2 + 2 * u, P(u, b));
            for (uint32_t u = 0; u < n; ++u) a.f("v_lshlrev_b32_e32 v%u, 1, v%u", 3 + 2 * u, P(u, b + 1));
            for (uint32_t u = 0; u < n; ++u)
                a.f("v_bitop3_b32 v%u, v%u, v%u, s37 bitop3:0x6c", P(u, b), 3 + 2 * u, 2 + 2 * u);
        }
    }
    a.line("s_load_dwordx16 s[64:79], s[60:61], 0x0");
    a.line("s_waitcnt lgkmcnt(0)");
    for (uint32_t k = 0; k < KC; ++k) {
        a.f("s_cmp_le_u32 s47, %u", k);
        a.line("s_cbranch_scc1 .Lend");
        for (uint32_t c = 0; c < CPL; ++c) {
            col_exec(a, c, true);
            static const char* const pol[] = {"", " nt", " sc1", " sc0 sc1"};
            a.f("buffer_store_dword v%u, v1, s[56:59], s%u offen offset:%u%s", ACC(c, k, 0), 64 + k, 256 * c,
                pol[sh.stpol & 3]);
            col_exec(a, c, false);
        }
    }
    a.s += ".Lend:\n\ts_endpgm\n";
    a.s += ".Lfunc_end:\n\t.size " + kname + ", .Lfunc_end-" + kname + "\n";
    a.s += "\t.section .rodata,\"a\",@progbits\n\t.p2align 6, 0x0\n\t.amdhsa_kernel " + kname + "\n";
    a.s += "\t\t.amdhsa_group_segment_fixed_size 0\n\t\t.amdhsa_private_segment_fixed_size 0\n";
    a.s += "\t\t.amdhsa_kernarg_size 48\n\t\t.amdhsa_user_sgpr_count 2\n";
    a.s += "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1\n\t\t.amdhsa_system_sgpr_workgroup_id_x 1\n";
    a.s += "\t\t.amdhsa_system_sgpr_workgroup_id_y 1\n\t\t.amdhsa_system_sgpr_workgroup_id_z 1\n";
    a.s += "\t\t.amdhsa_system_vgpr_workitem_id 0\n\t\t.amdhsa_next_free_vgpr " + std::to_string(NV) + "\n";
    a.s += "\t\t.amdhsa_next_free_sgpr 100\n\t\t.amdhsa_accum_offset " + std::to_string((NV + 3) & ~3u) + "\n";
    a.s += "\t\t.amdhsa_reserve_vcc 0\n\t\t.amdhsa_ieee_mode 0\n\t\t.amdhsa_dx10_clamp 0\n\t.end_amdhsa_kernel\n\t.text\n";
    a.s += "\t.amdgpu_metadata\n---\namdhsa.kernels:\n  - .agpr_count: 0\n    .args:\n";
    a.s += "      - .offset: 0\n        .size: 48\n        .value_kind: by_value\n";
    a.s += "    .group_segment_fixed_size: 0\n    .kernarg_segment_align: 8\n    .kernarg_segment_size: 48\n";
    a.s += "    .max_flat_workgroup_size: 512\n    .name: " + kname + "\n    .private_segment_fixed_size: 0\n";
    a.s += "    .sgpr_count: 100\n    .symbol: " + kname + ".kd\n    .vgpr_count: " + std::to_string(NV) +
           "\n    .wavefront_size: 64\n";
    a.s += "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n";
    return a.s;
}

// The index-mode guard.  In the VGPR index mode (s_set_gpr_idx_on) every VALU
// instruction's enabled operand is offset by M0[7:0], and M0[15:12] holds the enable bits (SRC0, SRC1,
// SRC2, DST).  So (1) a VALU instruction other than a lookup inside a region reads a shifted register;
// (2) a whole-dword write of M0 replaces the index AND the enable bits -- a packed pair of subset numbers
// written that way puts the second number's bits into the enables or into bits 7:5 of the index, and an
// enabled DST or an index past the table reaches VGPRs beyond the allocation (the round-5 variant "M0
// written by SALU moves to carry two indices per dword" faulted; its code was never committed, and this
// generator has no such path); (3) the index itself is bits 7:0 of an SGPR the kernel loaded from the
// stream, which k_xbits / the solvers (gi_stream) build from G bits, so it is < 2^G
// (tests/test_applygi.py emulates that stream on the host).
bool check_apply_gi_asm(const std::string& text, const GiShape& sh, std::string* err) {
    const uint32_t NT = 1u << sh.G, NV = gi_vgprs(sh), TB = gi_tb(sh);
    auto bad = [&](const std::string& why, const std::string& l) {
        if (err) *err = "apply kernel index-mode check: " + why + ": `" + l + "`";
        return false;
    };
    std::istringstream in(text);
    std::string l;
    bool on = false, body = false;
    while (std::getline(in, l)) {
        if (l.rfind(".amdhsa_kernel", 1) != std::string::npos || l.find(".section") != std::string::npos) break;
        size_t a = l.find_first_not_of(" \t");
        if (a == std::string::npos) continue;
        const std::string t = l.substr(a);
        if (t[0] == '.' && t.find(':') == std::string::npos) continue;  // directives
        if (t.find(':') != std::string::npos && t.find(' ') == std::string::npos) {  // a label
            if (on) return bad("label inside an index-mode region", t);
            body = true;
            continue;
        }
        if (!body && t.find(':') != std::string::npos) { body = true; continue; }  // the kernel symbol
        std::string op = t.substr(0, t.find_first_of(" \t"));
        // M0: never written or read by name (the index mode keeps its state there)
        for (size_t at = t.find("m0"); at != std::string::npos; at = t.find("m0", at + 1)) {
            const bool lft = at == 0 || !std::isalnum((unsigned char)t[at - 1]);
            const bool rgt = at + 2 >= t.size() || !std::isalnum((unsigned char)t[at + 2]);
            if (lft && rgt) return bad("M0 named while the kernel uses the VGPR index mode", t);
        }
        if (op == "s_set_gpr_idx_on") {
            if (on) return bad("nested s_set_gpr_idx_on", t);
            if (t.find("gpr_idx(SRC0)") == std::string::npos || t.find("DST") != std::string::npos ||
                t.find("SRC1") != std::string::npos || t.find("SRC2") != std::string::npos)
                return bad("index mode other than SRC0", t);
            on = true;
            continue;
        }
        if (op == "s_set_gpr_idx_off") {
            if (!on) return bad("s_set_gpr_idx_off outside a region", t);
            on = false;
            continue;
        }
        if (op == "s_set_gpr_idx_idx") {
            if (!on) return bad("s_set_gpr_idx_idx outside a region", t);
            continue;
        }
        if (!on) continue;
        if (op == "s_endpgm" || op.rfind("s_branch", 0) == 0 || op.rfind("s_cbranch", 0) == 0 || op == "s_setpc_b64")
            return bad("control flow inside an index-mode region", t);
        if (op.rfind("buffer_", 0) == 0 || op.rfind("global_", 0) == 0 || op.rfind("ds_", 0) == 0 ||
            op.rfind("flat_", 0) == 0 || op.rfind("scratch_", 0) == 0)
            return bad("memory instruction inside an index-mode region", t);
        if (op[0] != 'v') continue;  // SALU (the index loads' bookkeeping)
        unsigned d = 0, s0 = 0, s1 = 0;
        if (op != "v_xor_b32_e32" || std::sscanf(t.c_str(), "v_xor_b32_e32 v%u, v%u, v%u", &d, &s0, &s1) != 3)
            return bad("vector instruction other than a table lookup inside an index-mode region", t);
        bool table = false;
        for (uint32_t c = 0; c < sh.CPL; ++c) table |= s0 == TB + c * NT;
        if (!table) return bad("indexed source is not a table base", t);
        if (s0 + NT > NV) return bad("table end past the VGPR allocation", t);
        if (d != s1 || (d >= s0 && d < s0 + NT)) return bad("lookup destination is not an accumulator outside the table", t);
    }
    if (on) return bad("index-mode region not closed", "end of kernel");
    return true;
}

}  // namespace rq
