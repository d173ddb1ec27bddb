// rq_colasm_internal.hpp -- pieces of the column-program emitter and emulator shared by rq_colasm.cpp
// (the shipped single-wave programs) and rq_colasm_exp.cpp (the two-wave pair and four-row-staging
// variants, experiments builds only).  Not part of the library's interface.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "rq_colasm.hpp"

namespace rq {

inline bool is_agpr_reg(int r) { return r >= REG_A0; }

// Cache-policy suffixes of the memory instructions (gfx950 sc0/sc1/nt bits).  Output rows stream
// once (nt).  Source rows take the default policy: the waves of adjacent items read the two
// 128-B lines at their 256-B segment edges, which a streaming (nt) load marks for early eviction
// (interleaved A/B on one box, profiles/r02aj: K=1024 0.511 -> 0.496 ms, K=256 0.085 -> 0.075 ms).
// Scratch lines are re-read soon.  RQHIP_POLICY="src;out;scr_st;scr_ld" overrides them for
// experiments.
struct Policy {
    std::string src = "", out = " nt", scr_st = "", scr_ld = " sc1";
    Policy() {
        if (const char* e = knob("RQHIP_POLICY")) {
            std::string v(e), f[4];
            int i = 0;
            for (char c : v) {
                if (c == ';') { if (++i == 4) break; continue; }
                f[i] += c;
            }
            std::string* dst[4] = {&src, &out, &scr_st, &scr_ld};
            for (int k = 0; k < 4; ++k) *dst[k] = f[k].empty() ? "" : " " + f[k];
        }
    }
};

// Diagnostic builds (wrong bytes, timing only): RQHIP_DIAG bit 1 drops global scratch traffic,
// 2 drops LDS spill traffic, 4 replaces source loads by register writes, 8 drops output stores,
// 16 loads source rows in increasing row order (wrong rows; measures the cost of the random order),
// 32 drops the XOR / xtime instructions (memory traffic and register moves only), 64 drops the vmcnt
// waits (loads then race their uses: wrong bytes, but every address stays valid), 128 drops the pair
// programs' barriers (the two waves run decoupled: wrong bytes, same instructions, nothing waits).
inline uint32_t diag_mask() {
    const char* e = knob("RQHIP_DIAG");
    return e ? (uint32_t)std::atoi(e) : 0u;
}


// SGPR map of the emitted kernel beyond the prologue's s0..s55: s56..s63 scratch soffset bases,
// s64..s79 / s80..s95 the two halves of the double-buffered source row-offset window.
constexpr uint32_t SCR_BASES = 8;
constexpr uint32_t ROW_WIN = 64;

uint32_t scratch_bases(const MProg& mp);
// The per-item instruction stream of an allocated program (see rq_colasm.cpp).
void emit_colprog_body(const MProg& mp, uint32_t W, std::string& s);
#ifdef RQHIP_EXPERIMENTS
// four-row staging hooks of the single-wave emitter (rq_colasm_exp.cpp)
void emit_dma4_prologue(const MProg& mp, const Reserved& rv, std::string& s);
void emit_dma4_item_base(const Reserved& rv, std::string& s);
#endif

inline uint32_t xtime4(uint32_t x) {
    const uint32_t hi = (x >> 7) & 0x01010101u;
    return ((x & 0x7F7F7F7Fu) << 1) ^ (hi * 0x1Du);
}

// One wave's machine state for the emulators: registers, scratch, its LDS spill slots, the vmcnt / lgkmcnt
// bookkeeping.  Ring stores / loads and barriers (pair programs) go to the hooks.
struct WaveEmu {
    const MProg& mp;
    const uint8_t* src;
    uint32_t T, Td;
    uint64_t src_bytes = UINT64_MAX;  // buffer-resource extent: source dwords at or beyond it read 0
    uint8_t* out;
    std::string* err;
    std::vector<std::vector<uint32_t>> R, scr, lds;
    std::vector<uint64_t> pend, slot_st, lpend, lds_dma;
    uint64_t seq = 0, retired = 0, lseq = 0, lretired = 0;
    std::function<bool(uint32_t, const std::vector<uint32_t>&)> ring_store;
    std::function<bool(uint32_t, std::vector<uint32_t>*)> ring_load;
    std::function<void()> barrier;
    // cross-item prefetch: pass 2 runs the item again as the wave's next item (MI_HEAD then finds the row
    // the previous MI_PFX loaded; vmcnt keeps counting across the boundary); rows loaded into the head
    // registers by MI_PFX, and those registers handed over (nothing may write them until MI_HEAD)
    bool second = false;
    std::vector<int64_t> pfx_row = std::vector<int64_t>(512, -1);
    std::vector<uint8_t> handed = std::vector<uint8_t>(512, 0);
    uint64_t tbl_seq[2] = {0, 0};           // four-row staging: the table read into each table VGPR
    uint32_t tbl_grp[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    char buf[200];

    WaveEmu(const MProg& m, const uint8_t* s, uint32_t t, uint8_t* o, std::string* e)
        : mp(m), src(s), T(t), Td(t / 4), out(o), err(e), R(512, std::vector<uint32_t>(t / 4, 0)),
          scr(m.n_slots, std::vector<uint32_t>(t / 4, 0)),
          lds(std::max<uint32_t>(m.n_lds_slots, 1), std::vector<uint32_t>(t / 4, 0)), pend(512, 0),
          slot_st(m.n_slots, 0), lpend(512, 0), lds_dma(std::max<uint32_t>(m.n_lds_slots, 1), 0) {}

    bool bad(size_t i, const char* what) {
        std::snprintf(buf, sizeof buf, "emulate: instruction %zu: %s", i, what);
        if (err) *err = buf;
        return false;
    }
    bool ready(int r) const {
        return r < 0 || ((pend[r] == 0 || pend[r] <= retired) && (lpend[r] == 0 || lpend[r] <= lretired));
    }
    // at 63 outstanding the hardware holds issue until the oldest retires (pass 2 starts with the previous
    // item's tail in flight); the allocator itself never lets more than max_vmem be outstanding
    bool vmem() {
        if (second && seq - retired >= 63) retired = seq - 62;
        return ++seq - retired <= 63;
    }
    // source row `row` into dst (T/4 dwords) through the bounded buffer resource
    void read_row(uint32_t row, uint32_t* dst) const {
        const uint64_t base = (uint64_t)row * T;
        for (uint32_t c = 0; c < Td; ++c) {
            const uint64_t at = base + 4ull * c;
            if (at + 4 <= src_bytes) std::memcpy(&dst[c], src + at, 4);
            else dst[c] = 0;
        }
    }

    bool step(size_t i, const MInst& m) {
        if (!ready(m.a) || !ready(m.b) || !ready(m.c)) return bad(i, "operand read before its load completed");
        if (m.op != MI_DMA && m.op != MI_DMA4 && m.op != MI_DMAT && m.op != MI_HEAD && m.d >= 0 && !ready(m.d))
            return bad(i, "register overwritten while a load into it is pending");
        if (m.op != MI_DMA && m.op != MI_DMA4 && m.op != MI_DMAT && m.op != MI_HEAD && m.d >= 0 && handed[m.d])
            return bad(i, "write to a register handed to the next item");
        switch (m.op) {
            case MI_XOR2:
                for (uint32_t c = 0; c < Td; ++c) R[m.d][c] = R[m.a][c] ^ R[m.b][c];
                break;
            case MI_XOR3:
                for (uint32_t c = 0; c < Td; ++c) R[m.d][c] = R[m.a][c] ^ R[m.b][c] ^ R[m.c][c];
                break;
            case MI_XT:
                for (uint32_t c = 0; c < Td; ++c) R[m.d][c] = xtime4(R[m.a][c]);
                break;
            case MI_XTX:
                for (uint32_t c = 0; c < Td; ++c) R[m.d][c] = xtime4(R[m.a][c]) ^ R[m.b][c];
                break;
            case MI_ZERO:
                std::fill(R[m.d].begin(), R[m.d].end(), 0u);
                break;
            case MI_LDSRC:
                if (m.imm >= mp.K) return bad(i, "source row >= K");
                read_row(m.imm, R[m.d].data());
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                pend[m.d] = seq;
                break;
            case MI_STOUT:
                if (m.imm >= mp.n_out) return bad(i, "output index out of range");
                std::memcpy(out + (size_t)m.imm * T, R[m.a].data(), (size_t)Td * 4);
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                break;
            case MI_SPST:
                scr[m.imm] = R[m.a];
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                slot_st[m.imm] = seq;
                break;
            case MI_SPLD:
                if (slot_st[m.imm] > retired) return bad(i, "reload of a slot whose store is still in flight");
                R[m.d] = scr[m.imm];
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                pend[m.d] = seq;
                break;
            case MI_ACCW:
                if (m.d < REG_A0 || m.a >= REG_A0) return bad(i, "accvgpr_write operands");
                R[m.d] = R[m.a];
                break;
            case MI_ACCR:
                if (m.d >= REG_A0 || m.a < REG_A0) return bad(i, "accvgpr_read operands");
                R[m.d] = R[m.a];
                break;
            case MI_WAIT:
                if (seq > m.imm) retired = std::max(retired, seq - m.imm);
                break;
            case MI_NOP:
                break;
            case MI_LDST:
                if (m.imm >= mp.n_lds_slots) return bad(i, "LDS slot out of range");
                if (lds_dma[m.imm] > retired) return bad(i, "LDS write over a pending DMA");
                lds[m.imm] = R[m.a];
                if (++lseq - lretired > 15) return bad(i, "more than 15 LDS operations outstanding");
                break;
            case MI_LDLD:
                if (m.imm >= mp.n_lds_slots) return bad(i, "LDS slot out of range");
                if (lds_dma[m.imm] > retired) return bad(i, "LDS read before its DMA completed");
                R[m.d] = lds[m.imm];
                if (++lseq - lretired > 15) return bad(i, "more than 15 LDS operations outstanding");
                lpend[m.d] = lseq;
                break;
            case MI_WAITL:
                if (lseq > m.imm) lretired = std::max(lretired, lseq - m.imm);
                break;
            case MI_DMA:
                if (m.imm >= mp.K) return bad(i, "source row >= K");
                if (m.d < 0 || (uint32_t)m.d >= mp.n_lds_slots) return bad(i, "DMA slot out of range");
                if (lds_dma[m.d] > retired) return bad(i, "DMA over a pending DMA");
                read_row(m.imm, lds[m.d].data());
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                lds_dma[m.d] = seq;
                break;
            case MI_RST:
                if (!ring_store) return bad(i, "ring store outside a pair program");
                if (!ring_store(m.imm, R[m.a])) return bad(i, err && !err->empty() ? err->c_str() : "ring store");
                if (++lseq - lretired > 15) return bad(i, "more than 15 LDS operations outstanding");
                break;
            case MI_RLD:
                if (!ring_load) return bad(i, "ring load outside a pair program");
                if (!ring_load(m.imm, &R[m.d])) return bad(i, err && !err->empty() ? err->c_str() : "ring load");
                if (++lseq - lretired > 15) return bad(i, "more than 15 LDS operations outstanding");
                lpend[m.d] = lseq;
                break;
            case MI_BAR:
                if (lseq != lretired) return bad(i, "barrier with LDS operations outstanding");
                if (!barrier) return bad(i, "barrier outside a pair program");
                barrier();
                break;
            case MI_HEAD:
                if (m.imm >= mp.K) return bad(i, "source row >= K");
                if (second) {  // loaded by the previous item's MI_PFX
                    if (pfx_row[m.d] != (int64_t)m.imm) return bad(i, "head register does not hold its prefetched row");
                    handed[m.d] = 0;
                    pfx_row[m.d] = -1;
                    break;
                }
                read_row(m.imm, R[m.d].data());
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                pend[m.d] = seq;
                break;
            case MI_PFX: {
                const uint32_t f = m.imm >> 16, n = m.imm & 0xFFFFu;
                if ((size_t)f + n > mp.cip_reg.size()) return bad(i, "prefetch beyond the head list");
                for (uint32_t k = f; k < f + n; ++k) {
                    const int r = mp.cip_reg[k];
                    if (handed[r] || !ready(r)) return bad(i, "prefetch into a busy register");
                    read_row(mp.cip_row[k], R[r].data());
                    if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                    pend[r] = seq;
                    pfx_row[r] = mp.cip_row[k];
                    handed[r] = 1;
                }
                break;
            }
            case MI_DMAT:
                if (m.d < 0 || m.d > 1) return bad(i, "table register out of range");
                if ((size_t)m.imm * 4 + 4 > mp.dma4_rows.size()) return bad(i, "table read beyond the group table");
                if (++lseq - lretired > 15) return bad(i, "more than 15 LDS operations outstanding");
                tbl_seq[m.d] = lseq;
                tbl_grp[m.d] = m.imm;
                break;
            case MI_DMA4: {
                const uint32_t tr = m.imm & 1u;
                if (tbl_grp[tr] != m.imm) return bad(i, "four-row DMA without its table read");
                if (tbl_seq[tr] > lretired) return bad(i, "four-row DMA before its table read completed");
                if (m.d < 0 || (uint32_t)m.d >= mp.dma4_quads) return bad(i, "quad out of range");
                for (uint32_t g = 0; g < 4; ++g) {
                    const uint32_t sl = mp.dma4_slot0 + 4u * (uint32_t)m.d + g;
                    if (sl >= mp.n_lds_slots) return bad(i, "quad slot out of range");
                    if (lds_dma[sl] > retired) return bad(i, "DMA over a pending DMA");
                    const uint32_t row = mp.dma4_rows[(size_t)m.imm * 4 + g];
                    if (row >= mp.K) return bad(i, "source row >= K");
                    read_row(row, lds[sl].data());
                }
                if (!vmem()) return bad(i, "more than 63 vector-memory operations outstanding");
                for (uint32_t g = 0; g < 4; ++g) lds_dma[mp.dma4_slot0 + 4u * (uint32_t)m.d + g] = seq;
                tbl_grp[tr] = 0xFFFFFFFFu;  // the add consumed the table register
                break;
            }
        }
        if ((m.op == MI_XOR2 || m.op == MI_XOR3 || m.op == MI_XT || m.op == MI_XTX || m.op == MI_ZERO) &&
            (m.d >= REG_A0 || m.a >= REG_A0 || m.b >= REG_A0 || m.c >= REG_A0))
            return bad(i, "VALU operand in an AGPR");
        const int nva = (int)mp.n_vgpr;
        if ((m.op <= MI_ZERO) && (m.d >= nva || (m.a >= nva && m.a < REG_A0) || (m.b >= nva && m.b < REG_A0) ||
                                  (m.c >= nva && m.c < REG_A0)))
            return bad(i, "VALU operand in a reserved VGPR");
        return true;
    }
    bool run() {
        // each item's allocation assumes no vector-memory operation outstanding at its start (the
        // previous item's last ones are stores; at 63 outstanding the hardware holds further issue).  With
        // cross-item prefetch the item runs twice, the second time as its own next item (the counters
        // carry over: its waits must also cover the previous item's prefetch and last stores).
        retired = seq;
        for (size_t i = 0; i < mp.ins.size(); ++i)
            if (!step(i, mp.ins[i])) return false;
        lretired = lseq;  // the loop end's lgkmcnt(0)
        if (mp.cip_reg.empty()) return true;
        for (size_t k = 0; k < mp.cip_reg.size(); ++k)
            if (!handed[mp.cip_reg[k]] || pfx_row[mp.cip_reg[k]] != (int64_t)mp.cip_row[k])
                return bad(mp.ins.size(), "a head register not prefetched for the next item");
        second = true;
        for (size_t i = 0; i < mp.ins.size(); ++i)
            if (!step(i, mp.ins[i])) return false;
        lretired = lseq;
        return true;
    }
};

}  // namespace rq
