// rq_colasm_exp.cpp -- column-program variants measured and not shipped (DESIGN.md sec. 5.2,
// profiles/r04_pair), compiled into the experiments library only (make EXPERIMENTS=1):
//   four-row staging of a single-wave program's source rows (compile_colprog_dma4 and its emitter hooks;
//     K=1024: 0.40-0.42 ms against 0.38 for the shipped program)
//   the two-wave pair split (compile_pair, emulate_pair, emit_pair_asm; 0.49-0.51 ms)
// The engine takes them only through RQHIP_DMA4 / RQHIP_PAIR (rq_engine.cpp compile_engine_program).
#ifndef RQHIP_EXPERIMENTS
#error "rq_colasm_exp.cpp belongs to the experiments build only"
#endif
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "rq_colasm.hpp"
#include "rq_colasm_internal.hpp"

namespace rq {

bool compile_colprog_dma4(const ColIR& ir, const AllocOpts& o, uint32_t quads, uint32_t la, MProg* mp,
                          std::string* err) {
    constexpr uint32_t WAVE_SLOTS = 160;  // 40 KiB per one-wave workgroup: four per CU
    uint32_t n_loads = 0;
    for (const IrNode& d : ir.nodes) n_loads += d.k == IR_LOAD;
    const uint32_t tbl_est = ((n_loads + 3) / 4 + 32) * 16 / 256 + 1;
    if (!quads || tbl_est + 4 * quads + 16 > WAVE_SLOTS) {
        if (err) *err = "compile_colprog_dma4: LDS budget";
        return false;
    }
    AllocOpts so = o;
    so.cip = 0;
    so.dma4 = quads;
    so.la_dma = la;
    so.n_vgpr = std::min<uint32_t>(o.n_vgpr, V_ALLOC - (N_RESERVED_DMA4 - N_RESERVED));
    so.n_lds = WAVE_SLOTS - tbl_est;  // spill slots, then the quads at the top
    if (!allocate_colprog(ir, so, mp, err)) return false;
    mp->lds_base = (uint32_t)((mp->dma4_rows.size() / 4 * 16 + 255) / 256);
    mp->wg_waves = 1;
    if (mp->lds_base + mp->n_lds_slots > WAVE_SLOTS) {
        if (err) *err = "compile_colprog_dma4: LDS budget";
        return false;
    }
    return true;
}


// Four-row staging, once per wave: the group table (16 B per group: the four rows' offsets row * T)
// into LDS 0 by LDS-DMA, 1 KiB per instruction, range-checked at the table's size through the VGPR
// offset; then the lane's table offset (lane group l / 16 reads entry l / 16 of a group).  v0 = lane.
void emit_dma4_prologue(const MProg& mp, const Reserved& rv, std::string& s) {
    char buf[160];
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    const uint32_t tbl_bytes = (uint32_t)(mp.dma4_rows.size() / 4 * 16);
    std::snprintf(buf, sizeof buf, "s_add_u32 s40, s50, %u", colprog_dma4_table_offset(mp)); line(buf);
    line("s_addc_u32 s41, s51, 0");
    line("s_and_b32 s41, s41, 0xffff");
    std::snprintf(buf, sizeof buf, "s_mov_b32 s42, %u", tbl_bytes); line(buf);
    line("s_mov_b32 s43, 0x20000");
    line("v_lshlrev_b32_e32 v1, 4, v0");
    for (uint32_t k = 0; k * 1024 < tbl_bytes; ++k) {
        if (k) line("v_add_u32_e32 v1, 0x400, v1");
        std::snprintf(buf, sizeof buf, "s_mov_b32 m0, %u", k * 1024); line(buf);
        line("s_nop 0");
        line("buffer_load_dwordx4 v1, s[40:43], 0 offen lds");
    }
    line("s_waitcnt vmcnt(0)");
    std::snprintf(buf, sizeof buf, "v_lshrrev_b32_e32 v%d, 4, v0", rv.grp4); line(buf);
    std::snprintf(buf, sizeof buf, "v_lshlrev_b32_e32 v%d, 2, v%d", rv.grp4, rv.grp4); line(buf);
}

// Four-row staging, per item (before the item's column map; v0 = lane, s20 = the item's first column):
// lane l's 16-B chunk is dword columns 4 (l % 16) .. + 3 of the item (T % 16 == 0 keeps a chunk inside
// one block); its base offset, 0 (valid memory, unused) beyond the last column.  All lanes: the staging
// runs with exec = -1, the item's mask is in s[22:23].  Uses v1..v4, s21, s[46:47].
void emit_dma4_item_base(const Reserved& rv, std::string& s) {
    char buf[160];
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    line("s_lshr_b32 s21, s12, 2");
    line("v_and_b32_e32 v1, 15, v0");
    line("v_lshlrev_b32_e32 v1, 2, v1");
    line("v_add_u32_e32 v1, s20, v1");
    line("v_cmp_gt_u32_e64 s[46:47], s13, v1");
    line("v_mul_hi_u32 v2, v1, s14");
    line("v_lshrrev_b32_e32 v2, s15, v2");
    line("v_mul_lo_u32 v3, v2, s21");
    line("v_sub_u32_e32 v3, v1, v3");
    line("v_lshlrev_b32_e32 v3, 2, v3");
    line("v_mul_lo_u32 v4, v2, s10");
    std::snprintf(buf, sizeof buf, "v_add_u32_e32 v%d, v4, v3", rv.dmabase); line(buf);
    std::snprintf(buf, sizeof buf, "v_cndmask_b32_e64 v%d, 0, v%d, s[46:47]", rv.dmabase, rv.dmabase); line(buf);
}

// ------------------------------------------------------------------------------------------
// Two-wave (pair) programs.

bool compile_pair(const ColIR& ir, const AllocOpts& o, uint32_t bmask, uint32_t lag, uint32_t max_xfer, uint32_t ring,
                  PairProg* pp, std::string* err) {
    PairIR px;
    if (!split_pair(ir, bmask, lag, max_xfer, ring, &px, err)) return false;
    *pp = PairProg();
    pp->lag = lag;
    ring = px.ring;  // the smallest ring that passed split_pair's window check
    pp->ring = ring;
    pp->n_xfer = px.n_xfer;
    pp->n_cross = px.n_cross;
    pp->bmask = bmask;
    constexpr uint32_t WG_SLOTS = 320;  // 80 KiB of LDS per workgroup: two workgroups per CU
    if (ring + 16 > WG_SLOTS) {
        if (err) *err = "compile_pair: ring too large";
        return false;
    }
    // B first (small live set: a few LDS slots at most), then A with the LDS that is left
    AllocOpts ob = o;
    ob.cip = 0;
    ob.n_lds = std::min<uint32_t>(o.n_lds, 32);
    ob.la_dma = 0;
    ob.dma4 = 0;
    if (o.dma4) ob.n_vgpr = std::min<uint32_t>(o.n_vgpr, V_ALLOC - (N_RESERVED_DMA4 - N_RESERVED));  // same reserved VGPRs
    if (!allocate_colprog(px.B, ob, &pp->B, err)) return false;
    if (pp->B.n_slots) {
        if (err) *err = "compile_pair: wave B needs global scratch";
        return false;
    }
    AllocOpts oa = o;
    oa.cip = 0;
    // four-row staging: the group table (16 B per group; at most one group per load) sits at LDS 0
    uint32_t n_loads = 0;
    for (const IrNode& d : px.A.nodes) n_loads += d.k == IR_LOAD;
    // (groups hold four rows unless rows were already loaded directly: a few more than n_loads / 4)
    const uint32_t tbl_est = o.dma4 ? ((n_loads + 3) / 4 + 32) * 16 / 256 + 1 : 0;
    uint32_t quads = o.dma4;
    while (quads && ring + tbl_est + pp->B.n_lds_slots + 4 * quads + 32 > WG_SLOTS) quads /= 2;  // keep 32 spill slots
    oa.dma4 = quads;
    oa.n_lds = std::min<uint32_t>(o.n_lds + 4 * quads, WG_SLOTS - ring - tbl_est - pp->B.n_lds_slots);
    if (o.dma4) oa.n_vgpr = ob.n_vgpr;  // both waves: the same reserved VGPRs (the prologue sets them once)
    if (!quads) oa.la_dma = 0;
    if (!allocate_colprog(px.A, oa, &pp->A, err)) return false;
    if (pp->A.n_vgpr != pp->B.n_vgpr) {
        if (err) *err = "compile_pair: the waves' register layouts differ";
        return false;
    }
    pp->tbl_slots = (uint32_t)((pp->A.dma4_rows.size() / 4 * 16 + 255) / 256);
    pp->A.ring_base = pp->B.ring_base = pp->tbl_slots;
    pp->A.lds_base = pp->tbl_slots + ring;
    pp->B.lds_base = pp->tbl_slots + ring + pp->A.n_lds_slots;
    pp->A.wg_waves = pp->B.wg_waves = 2;
    if (pair_lds_bytes(*pp) > WG_SLOTS * 256u) {
        if (err) *err = "compile_pair: LDS budget";
        return false;
    }
    return true;
}

double pair_cost(const PairProg& pp) {
    // the two waves issue on different SIMDs: the longer one sets the item time (A's also carries
    // the memory instructions), plus a slot per barrier for the rendezvous
    return std::max(colprog_cost(pp.A), colprog_cost(pp.B));
}

uint32_t pair_lds_bytes(const PairProg& pp) {
    return (pp.tbl_slots + pp.ring + pp.A.n_lds_slots + pp.B.n_lds_slots) * 256u;
}

bool emulate_pair(const PairProg& pp, const uint8_t* src, uint32_t T, uint8_t* out, std::string* err, uint32_t iters) {
    const uint32_t Td = T / 4;
    // A's ring writes: per slot, (A barrier count at the write, data)
    std::vector<std::vector<std::pair<uint64_t, std::vector<uint32_t>>>> hist(pp.ring);
    uint64_t a_bars = 0, b_bars = pp.lag;  // B starts with `lag` barriers
    std::string e2;
    WaveEmu A(pp.A, src, T, out, &e2), B(pp.B, src, T, out, &e2);
    A.ring_store = [&](uint32_t sl, const std::vector<uint32_t>& v) {
        if (sl >= pp.ring) { e2 = "ring slot out of range"; return false; }
        hist[sl].push_back({a_bars, v});
        return true;
    };
    A.barrier = [&]() { ++a_bars; };
    B.barrier = [&]() { ++b_bars; };
    B.ring_load = [&](uint32_t sl, std::vector<uint32_t>* d) {
        if (sl >= pp.ring) { e2 = "ring slot out of range"; return false; }
        // visible: A's writes before A's barrier b_bars (A count <= b_bars - 1); a write in A's interval
        // b_bars runs concurrently with this read
        const std::vector<uint32_t>* v = nullptr;
        for (const auto& h : hist[sl]) {
            if (h.first == b_bars) { e2 = "ring race: A writes the slot in the interval B reads it"; return false; }
            if (h.first + 1 <= b_bars) v = &h.second;
        }
        if (!v) { e2 = "ring read of a slot A has not written"; return false; }
        *d = *v;
        return true;
    };
    for (uint32_t it = 0; it < iters; ++it)
        if (!A.run()) { if (err) *err = "wave A: " + e2; return false; }
    for (uint32_t it = 0; it < iters; ++it)
        if (!B.run()) { if (err) *err = "wave B: " + e2; return false; }
    (void)Td;
    // per item the two waves execute the same number of barriers
    if (a_bars != (uint64_t)pp.n_xfer * iters || b_bars != pp.lag + (uint64_t)pp.n_xfer * iters) {
        if (err) *err = "emulate_pair: barrier counts differ from the transfer count";
        return false;
    }
    return true;
}

std::string emit_pair_asm(const PairProg& pp, const std::string& kname) {
    static const uint32_t diag = diag_mask();
    const MProg& A = pp.A;
    const MProg& B = pp.B;
    const Reserved rv(A.n_vgpr);
    // one register layout for both waves: A's reservation (B never stages, but shares A's VGPR count)
    const uint32_t acc_off = std::max(colprog_acc_off(A), colprog_acc_off(B));
    const uint32_t n_regs = (acc_off + std::max<uint32_t>(std::max(A.n_agpr, B.n_agpr), 1) + 7) & ~7u;
    std::string s;
    s.reserve((A.ins.size() + B.ins.size()) * 48 + 16384);
    char buf[256];
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    auto put = [&](const char* p) {
        std::string l(p);
        const std::pair<const char*, int> names[] = {
            {"V_SRCOFF", rv.srcoff}, {"V_OUTOFF", rv.outoff}, {"V_SCROFF", rv.scroff}, {"V_LDS2", rv.lds2}};
        for (const auto& nm : names)
            for (size_t at = l.find(nm.first); at != std::string::npos; at = l.find(nm.first))
                l.replace(at, std::strlen(nm.first), "v" + std::to_string(nm.second));
        line(l.c_str());
    };
    s += "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.amdhsa_code_object_version 6\n\t.text\n";
    s += "\t.globl " + kname + "\n\t.p2align 8\n\t.type " + kname + ",@function\n" + kname + ":\n";
    // Common prologue: kernel arguments, buffer resources, constants; wave 0 of the workgroup runs A,
    // wave 1 runs B.  Workgroup g takes items g, g + n_wg, ... (s52 / s49 / s48), both waves alike.
    const char* pro[] = {
        "s_load_dwordx8 s[4:11], s[0:1], 0x0",
        "s_load_dwordx8 s[12:19], s[0:1], 0x20",
        "s_load_dwordx4 s[48:51], s[0:1], 0x40",
        "v_lshrrev_b32_e32 v1, 6, v0",
        "s_nop 4",
        "v_readfirstlane_b32 s53, v1",
        "v_and_b32_e32 v0, 63, v0",
        "v_lshlrev_b32_e32 V_SCROFF, 2, v0",
        "v_add_u32_e32 V_LDS2, 0x10000, V_SCROFF",
        "s_waitcnt lgkmcnt(0)",
        "s_mov_b32 s24, s4",
        "s_and_b32 s25, s5, 0xffff",
        "s_mov_b32 s26, s19",
        "s_mov_b32 s27, 0x20000",
        "s_mov_b32 s28, s6",
        "s_and_b32 s29, s7, 0xffff",
        "s_mov_b32 s30, -1",
        "s_mov_b32 s31, 0x20000",
        "s_mul_i32 s32, s2, s16",
        "s_mul_hi_u32 s33, s2, s16",
        "s_add_u32 s32, s8, s32",
        "s_addc_u32 s33, s9, s33",
        "s_and_b32 s33, s33, 0xffff",
        "s_mov_b32 s34, -1",
        "s_mov_b32 s35, 0x20000",
        "s_mov_b32 s36, 0x090b080a",
        "s_mov_b32 s37, 0xfefefefe",
        "s_mov_b32 s38, 0x1d1d1d1d",
        "s_mov_b32 s52, s2",
        "s_cmp_eq_u32 s53, 0",
        "s_cbranch_scc1 .LA",
        // wave B: a far jump (the A program is longer than a 16-bit branch reaches)
        "s_getpc_b64 s[54:55]",
    };
    for (const char* p : pro) put(p);
    s += ".Lpcb:\n";
    line("s_add_u32 s54, s54, .LB-.Lpcb");
    line("s_addc_u32 s55, s55, 0");
    line("s_setpc_b64 s[54:55]");
    // the item's lane -> (block, dword column) map (as emit_colprog_asm's W = 1 loop head)
    const char* iter[] = {
        "s_mov_b64 exec, -1",
        "s_and_b32 s39, s52, 7",
        "s_mul_i32 s39, s39, s17",
        "s_lshr_b32 s40, s52, 3",
        "s_add_u32 s39, s39, s40",
        "s_cmp_lt_u32 s52, s18",
        "s_cselect_b32 s39, s39, s52",
        "s_lshl_b32 s20, s39, 6",
        "v_lshrrev_b32_e32 v0, 2, V_SCROFF",
        "v_add_u32_e32 v1, s20, v0",
        "v_cmp_gt_u32_e64 s[22:23], s13, v1",
        "s_and_b64 exec, exec, s[22:23]",
        "v_mul_hi_u32 v2, v1, s14",
        "v_lshrrev_b32_e32 v2, s15, v2",
        "s_lshr_b32 s21, s12, 2",
        "v_mul_lo_u32 v3, v2, s21",
        "v_sub_u32_e32 v3, v1, v3",
        "v_lshlrev_b32_e32 v3, 2, v3",
        "v_mul_lo_u32 v4, v2, s10",
        "v_add_u32_e32 V_SRCOFF, v4, v3",
        "v_mul_lo_u32 v4, v2, s11",
        "v_add_u32_e32 V_OUTOFF, v4, v3",
    };
    const bool dma4 = A.dma4_quads > 0;
    auto wave = [&](const MProg& mp, const char* tag, bool is_a) {
        s += std::string(".L") + tag + ":\n";
        const uint32_t nb = std::min<uint32_t>(SCR_BASES, mp.n_slots > 16 ? (mp.n_slots - 1) / 16 : 0);
        for (uint32_t j = 0; j < nb; ++j) {
            std::snprintf(buf, sizeof buf, "s_mov_b32 s%u, %u", 56 + j, 4096u * (j + 1));
            line(buf);
        }
        if (is_a && dma4) emit_dma4_prologue(A, rv, s);
        if (!is_a && !(diag & 128))  // B trails A by `lag` transfers: its first `lag` barriers pair with A's first
            for (uint32_t j = 0; j < pp.lag; ++j) line("s_barrier");
        s += std::string(".L") + tag + "_loop:\n";
        line("s_cmp_lt_u32 s52, s48");
        std::snprintf(buf, sizeof buf, "s_cbranch_scc1 .L%s_body", tag);
        line(buf);
        if (is_a && !(diag & 128))  // A's last `lag` barriers pair with B's of the last item's last transfers
            for (uint32_t j = 0; j < pp.lag; ++j) line("s_barrier");
        line("s_endpgm");
        s += std::string(".L") + tag + "_body:\n";
        for (const char* p : iter) {
            if (is_a && dma4 && std::strcmp(p, "v_add_u32_e32 v1, s20, v0") == 0) emit_dma4_item_base(rv, s);
            put(p);
        }
        emit_colprog_body(mp, 1, s);
        line("s_waitcnt lgkmcnt(0)");
        line("s_add_u32 s52, s52, s49");
        line("s_getpc_b64 s[54:55]");
        s += std::string(".L") + tag + "_pc:\n";
        std::snprintf(buf, sizeof buf, "s_sub_u32 s54, s54, .L%s_pc-.L%s_loop", tag, tag);
        line(buf);
        line("s_subb_u32 s55, s55, 0");
        line("s_setpc_b64 s[54:55]");
    };
    wave(A, "A", true);
    wave(B, "B", false);
    s += ".Lfunc_end:\n\t.size " + kname + ", .Lfunc_end-" + kname + "\n";
    s += "\t.p2alignl 6, 3212836864\n\t.fill 256, 4, 3212836864\n";
    s += "\t.section .rodata,\"a\",@progbits\n\t.p2align 6, 0x0\n\t.amdhsa_kernel " + kname + "\n";
    const std::string lds = std::to_string(pair_lds_bytes(pp));
    s += "\t\t.amdhsa_group_segment_fixed_size " + lds + "\n\t\t.amdhsa_private_segment_fixed_size 0\n";
    s += "\t\t.amdhsa_kernarg_size 104\n\t\t.amdhsa_user_sgpr_count 2\n";
    s += "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1\n\t\t.amdhsa_system_sgpr_workgroup_id_x 1\n";
    s += "\t\t.amdhsa_system_vgpr_workitem_id 0\n\t\t.amdhsa_next_free_vgpr " + std::to_string(n_regs) + "\n";
    s += "\t\t.amdhsa_next_free_sgpr " + std::to_string(ROW_WIN + 32) + "\n\t\t.amdhsa_accum_offset " + std::to_string(acc_off) +
         "\n\t\t.amdhsa_reserve_vcc 0\n";
    s += "\t\t.amdhsa_ieee_mode 0\n\t\t.amdhsa_dx10_clamp 0\n\t.end_amdhsa_kernel\n\t.text\n";
    s += "\t.amdgpu_metadata\n---\namdhsa.kernels:\n  - .agpr_count: " + std::to_string(n_regs - acc_off) + "\n    .args:\n";
    s += "      - .offset: 0\n        .size: 104\n        .value_kind: by_value\n";
    s += "    .group_segment_fixed_size: " + lds + "\n    .kernarg_segment_align: 8\n    .kernarg_segment_size: 104\n";
    s += "    .max_flat_workgroup_size: 128\n    .name: " + kname + "\n    .private_segment_fixed_size: 0\n";
    s += "    .sgpr_count: " + std::to_string(ROW_WIN + 32) + "\n    .symbol: " + kname + ".kd\n    .vgpr_count: " + std::to_string(n_regs) +
         "\n    .wavefront_size: 64\n";
    s += "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n";
    return s;
}

}  // namespace rq
