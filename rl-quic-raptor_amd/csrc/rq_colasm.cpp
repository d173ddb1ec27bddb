// rq_colasm.cpp -- allocation, emission and emulation of the column program (rq_colasm.hpp).
#include "rq_colasm.hpp"
#include "rq_colasm_internal.hpp"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <queue>
#include <set>

namespace rq {

namespace {

constexpr uint32_t INF = 0xFFFFFFFFu;
inline bool is_agpr(int r) { return r >= REG_A0; }

struct Allocator {
    const ColIR& ir;
    const AllocOpts& o;
    MProg* mp;
    std::string* err;
    uint32_t nv = 0;                                // IR nodes
    std::vector<std::vector<uint32_t>> uses;        // value -> use positions (ascending)
    std::vector<uint32_t> uptr;
    std::vector<int16_t> reg;                       // value -> register or -1
    std::vector<int32_t> slot;                      // value -> scratch slot with a valid copy or -1
    std::vector<int32_t> lslot;                     // value -> LDS slot with a valid copy or -1
    std::vector<uint8_t> issued;                    // LOAD value already issued
    std::vector<uint64_t> dma_seq;                  // LOAD value staged in LDS by DMA: its vmem seq
    // four-row staging: quads of LDS slots [slot0 + 4q, +4), rows still to be read per quad, free quads,
    // the next group and its table read (lgkm seq)
    uint32_t slot0 = 0;
    std::vector<uint32_t> quad_left;
    std::deque<uint32_t> free_quads;
    uint32_t gj = 0;
    uint64_t tseq = 0;
    int32_t owner[512];
    uint64_t inflight[512];                         // vector-memory load into the register (seq) or 0
    uint64_t linflight[512];                        // LDS load into the register (lgkm seq) or 0
    uint8_t pinned[512];
    uint8_t reserved[512];                          // cross-item prefetch: head register handed to the next item
    int last_accw[512];                             // instruction index of the last ACCW into an AGPR
    std::vector<int> freeV, freeA;
    std::vector<int32_t> free_slots, free_lslots;
    std::set<std::pair<uint32_t, uint32_t>> lds_res;  // (next use, value) of values held in LDS
    std::vector<uint64_t> slot_st, slot_ld;         // last store / load seq per slot
    uint64_t seq = 0, retired = 0;
    std::deque<std::pair<uint64_t, int>> pend_loads;  // (seq, reg)
    uint64_t lseq = 0, lretired = 0;                // LDS operations (lgkmcnt, in order, max 15)
    std::deque<std::pair<uint64_t, int>> pend_lds;
    std::vector<size_t> vm_ins{0}, l_ins{0};        // seq -> instruction index at issue
    using HE = std::pair<uint32_t, uint32_t>;       // (next use, value)
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> reload_q;
    bool failed = false;
    uint32_t cur = 0;                               // IR node being allocated

    Allocator(const ColIR& i, const AllocOpts& op, MProg* m, std::string* e) : ir(i), o(op), mp(m), err(e) {}

    uint32_t nu(uint32_t v) const { return uptr[v] < uses[v].size() ? uses[v][uptr[v]] : INF; }
    // a source row always has its home copy in the source buffer: evicted, it is re-read from there
    // instead of being written to scratch
    bool is_src(uint32_t v) const { return ir.nodes[v].k == IR_LOAD; }
    bool has_copy(uint32_t v) const { return slot[v] >= 0 || lslot[v] >= 0 || is_src(v); }

    void emit(uint8_t op, int d = -1, int a = -1, int b = -1, int c = -1, uint32_t imm = 0) {
        MInst m;
        m.op = op; m.d = (int16_t)d; m.a = (int16_t)a; m.b = (int16_t)b; m.c = (int16_t)c; m.imm = imm;
        mp->ins.push_back(m);
    }
    void fail(const char* m) {
        if (!failed && err) *err = m;
        failed = true;
    }

    // ---- vector-memory counters ----
    void retire_to(uint64_t s) {
        if (s <= retired) return;
        retired = s;
        while (!pend_loads.empty() && pend_loads.front().first <= retired) {
            const int r = pend_loads.front().second;
            if (inflight[r] == pend_loads.front().first) inflight[r] = 0;
            pend_loads.pop_front();
        }
    }
    // Make op `s` complete.  The wait also covers the younger operations issued at least
    // wait_age instructions ago (done by now in all likelihood), so the next uses find them retired
    // and need no s_waitcnt of their own.
    void wait_seq(uint64_t s) {
        if (s == 0 || s <= retired) return;
        const size_t now = mp->ins.size();
        while (s < seq && vm_ins[s + 1] + o.wait_age <= now) ++s;
        const uint64_t n = std::min<uint64_t>(seq - s, 63);
        emit(MI_WAIT, -1, -1, -1, -1, (uint32_t)n);
        mp->st.wait++;
        retire_to(seq - n);
    }
    uint64_t issue_vmem() {  // call before emitting a VMEM instruction; returns its seq
        if (seq - retired >= o.max_vmem) {  // full: also retire what was issued wait_age instructions ago
            const size_t now = mp->ins.size();
            uint64_t s = retired + 1;
            while (s < seq && vm_ins[s + 1] + o.wait_age <= now) ++s;
            const uint64_t n = std::min<uint64_t>(seq - s, o.max_vmem - 1);
            emit(MI_WAIT, -1, -1, -1, -1, (uint32_t)n);
            mp->st.wait++;
            retire_to(seq - n);
        }
        vm_ins.push_back(mp->ins.size());
        return ++seq;
    }

    void retire_l(uint64_t s) {
        if (s <= lretired) return;
        lretired = s;
        while (!pend_lds.empty() && pend_lds.front().first <= lretired) {
            const int r = pend_lds.front().second;
            if (linflight[r] == pend_lds.front().first) linflight[r] = 0;
            pend_lds.pop_front();
        }
    }
    void wait_lseq(uint64_t s) {
        if (s == 0 || s <= lretired) return;
        const size_t now = mp->ins.size();
        while (s < lseq && l_ins[s + 1] + o.lwait_age <= now) ++s;
        const uint64_t n = std::min<uint64_t>(lseq - s, 15);
        emit(MI_WAITL, -1, -1, -1, -1, (uint32_t)n);
        mp->st.waitl++;
        retire_l(lseq - n);
    }
    uint64_t issue_lgkm() {
        // full (15 outstanding): retire everything issued lwait_age instructions ago or more at once, so
        // the next LDS operations do not each need a wait of their own (-106 waits per item at K=1024)
        if (lseq - lretired >= 15) {
            const size_t now = mp->ins.size();
            uint64_t s = lretired + 1;
            while (s < lseq && l_ins[s + 1] + o.lwait_age <= now) ++s;
            const uint64_t n = std::min<uint64_t>(lseq - s, 14);
            emit(MI_WAITL, -1, -1, -1, -1, (uint32_t)n);
            mp->st.waitl++;
            retire_l(lseq - n);
        }
        l_ins.push_back(mp->ins.size());
        return ++lseq;
    }
    bool busy(int r) const { return inflight[r] || linflight[r]; }

    // ---- scratch ----
    int32_t new_slot() {
        int32_t s;
        if (!free_slots.empty()) { s = free_slots.back(); free_slots.pop_back(); }
        else { s = (int32_t)mp->n_slots++; slot_st.push_back(0); slot_ld.push_back(0); }
        wait_seq(slot_ld[s]);  // WAR: an older reload of this slot must have read it
        wait_seq(slot_st[s]);  // WAW
        return s;
    }
    void to_global(uint32_t v, int r) {  // store register r (holding v) into a new scratch slot
        const int32_t s = new_slot();
        const uint64_t q = issue_vmem();
        emit(MI_SPST, -1, r, -1, -1, (uint32_t)s);
        mp->st.spst++;
        slot_st[s] = q;
        slot[v] = s;
    }
    void lds_put(uint32_t v, int r, int32_t s) {
        mp->n_lds_slots = std::max<uint32_t>(mp->n_lds_slots, (uint32_t)s + 1);
        issue_lgkm();
        emit(MI_LDST, -1, r, -1, -1, (uint32_t)s);
        mp->st.ldst++;
        lslot[v] = s;
        lds_res.insert({nu(v), v});
    }
    // value in register r -> a copy in LDS or global scratch (if none); r becomes free (not pushed
    // to a free list).  Registers + LDS act as one Belady cache in front of global scratch: a value
    // enters LDS if a slot is free, or by pushing the LDS resident with the furthest next use out to
    // global scratch when its own next use is nearer (through the reserved temp VGPR).
    void spill_out(int r) {
        const int32_t v = owner[r];
        if (slot[v] < 0 && lslot[v] < 0 && o.n_lds && (o.src_lds || !is_src((uint32_t)v))) {
            const uint32_t n = nu((uint32_t)v);
            if (!free_lslots.empty()) {
                const int32_t s = free_lslots.back();
                free_lslots.pop_back();
                lds_put((uint32_t)v, r, s);
            } else if (!lds_res.empty() && std::prev(lds_res.end())->first > n + o.lds_horizon) {
                const uint32_t w = std::prev(lds_res.end())->second;
                const int32_t s = lslot[w];
                const int t = Reserved(o.n_vgpr).t1;
                lds_res.erase(std::prev(lds_res.end()));
                if (dma_seq[w]) { wait_seq(dma_seq[w]); dma_seq[w] = 0; }
                lslot[w] = -1;
                if (!is_src(w)) {  // a source row is simply dropped: it is re-read from the source
                    const uint64_t q = issue_lgkm();
                    emit(MI_LDLD, t, -1, -1, -1, (uint32_t)s);
                    mp->st.ldld++;
                    wait_lseq(q);
                    to_global(w, t);
                }
                mp->st.migrate++;
                lds_put((uint32_t)v, r, s);
            }
        }
        if (!has_copy((uint32_t)v)) to_global((uint32_t)v, r);
        reg[v] = -1;
        owner[r] = -1;
        reload_q.push({nu((uint32_t)v), (uint32_t)v});
    }
    int victim(int lo, int hi) const {  // max-next-use resident value in [lo, hi), unpinned, not in flight
        int best = -1;
        uint64_t bn = 0;
        for (int r = lo; r < hi; ++r) {
            const int32_t v = owner[r];
            if (v < 0 || pinned[r] || busy(r)) continue;
            // source rows leave for free (no store): their next use counts src_bias % as far
            const uint64_t n = (uint64_t)nu((uint32_t)v) * (is_src((uint32_t)v) ? o.src_bias : 100u);
            if (best < 0 || n > bn) { best = r; bn = n; }
        }
        return best;
    }
    // a VGPR for an operand / result
    int take_vgpr() {
        if (!freeV.empty()) { const int r = freeV.back(); freeV.pop_back(); return r; }
        int r = victim(0, (int)o.n_vgpr);
        while (r < 0 && (!pend_loads.empty() || !pend_lds.empty())) {  // every VGPR awaits a load
            if (!pend_lds.empty()) wait_lseq(pend_lds.front().first);
            else wait_seq(pend_loads.front().first);
            r = victim(0, (int)o.n_vgpr);
        }
        if (r < 0) { fail("colasm: no evictable VGPR"); return 0; }
        const uint32_t n = nu((uint32_t)owner[r]);
        int a = -1;
        if (!freeA.empty()) { a = freeA.back(); freeA.pop_back(); }
        else {
            const int ra = victim(REG_A0, REG_A0 + (int)o.n_agpr);
            if (ra >= 0 && nu((uint32_t)owner[ra]) > n) { spill_out(ra); a = ra; }
        }
        if (a >= 0) {
            const int32_t v = owner[r];
            emit(MI_ACCW, a, r);
            mp->st.accw++;
            last_accw[a] = (int)mp->ins.size() - 1;
            owner[a] = v; reg[v] = (int16_t)a; owner[r] = -1;
        } else {
            spill_out(r);
        }
        return r;
    }
    // any register for a value first needed at `need` (prefetch); -1 if not worth it
    int take_any(uint32_t need) {
        if (!freeV.empty()) { const int r = freeV.back(); freeV.pop_back(); return r; }
        if (!freeA.empty()) { const int r = freeA.back(); freeA.pop_back(); return r; }
        const int rv = victim(0, (int)o.n_vgpr), ra = victim(REG_A0, REG_A0 + (int)o.n_agpr);
        int r = rv;
        if (r < 0 || (ra >= 0 && nu((uint32_t)owner[ra]) >= nu((uint32_t)owner[rv]))) r = ra;
        if (r < 0 || nu((uint32_t)owner[r]) <= need) return -1;
        spill_out(r);
        return r;
    }
    void release(int r) {
        owner[r] = -1;
        if (!reserved[r]) (is_agpr(r) ? freeA : freeV).push_back(r);
    }
    void kill(uint32_t v) {  // value dead: free register and scratch slot
        if (reg[v] >= 0) { release(reg[v]); reg[v] = -1; }
        if (slot[v] >= 0) { free_slots.push_back(slot[v]); slot[v] = -1; }
        if (lslot[v] >= 0) free_lds(v);
    }
    void free_lds(uint32_t v) {
        lds_res.erase({nu(v), v});
        if (o.dma4 && (uint32_t)lslot[v] >= slot0) {  // a staged row read: its quad frees with its last row
            const uint32_t q = ((uint32_t)lslot[v] - slot0) / 4;
            if (--quad_left[q] == 0) free_quads.push_back(q);
        } else {
            free_lslots.push_back(lslot[v]);
        }
        lslot[v] = -1;
    }
    void reload_into(uint32_t v, int r) {
        if (lslot[v] >= 0) {  // the LDS slot is released at once: LDS operations run in order
            if (dma_seq[v]) { wait_seq(dma_seq[v]); dma_seq[v] = 0; }
            const uint64_t q = issue_lgkm();
            emit(MI_LDLD, r, -1, -1, -1, (uint32_t)lslot[v]);
            mp->st.ldld++;
            linflight[r] = q;
            pend_lds.push_back({q, r});
            free_lds(v);
            owner[r] = (int32_t)v; reg[v] = (int16_t)r;
            return;
        }
        if (slot[v] < 0) {  // a dropped source row: read it again from the source buffer
            const uint64_t q = issue_vmem();
            emit(MI_LDSRC, r, -1, -1, -1, ir.nodes[v].imm);
            mp->st.spld++;
            inflight[r] = q;
            pend_loads.push_back({q, r});
            owner[r] = (int32_t)v; reg[v] = (int16_t)r;
            return;
        }
        const int32_t s = slot[v];
        wait_seq(slot_st[s]);
        const uint64_t q = issue_vmem();
        emit(MI_SPLD, r, -1, -1, -1, (uint32_t)s);
        mp->st.spld++;
        slot_ld[s] = q;
        inflight[r] = q;
        pend_loads.push_back({q, r});
        owner[r] = (int32_t)v; reg[v] = (int16_t)r;
    }
    // source row v -> a free LDS slot by LDS-DMA (its data is valid once vmcnt covers the DMA)
    bool issue_dma(uint32_t v) {
        if (free_lslots.empty()) return false;
        const int32_t s = free_lslots.back();
        free_lslots.pop_back();
        mp->n_lds_slots = std::max<uint32_t>(mp->n_lds_slots, (uint32_t)s + 1);
        const uint64_t q = issue_vmem();
        emit(MI_DMA, s, -1, -1, -1, ir.nodes[v].imm);
        mp->st.dma++;
        mp->st.ldsrc++;
        dma_seq[v] = q;
        lslot[v] = s;
        lds_res.insert({nu(v), v});
        reload_q.push({nu(v), v});
        issued[v] = 1;
        return true;
    }
    void issue_load(uint32_t v, int r) {
        const uint64_t q = issue_vmem();
        emit(MI_LDSRC, r, -1, -1, -1, ir.nodes[v].imm);
        mp->st.ldsrc++;
        inflight[r] = q;
        pend_loads.push_back({q, r});
        owner[r] = (int32_t)v; reg[v] = (int16_t)r;
        issued[v] = 1;
    }
    // Cross-item prefetch: head register r is handed to the next item from here on.  Its value (if any)
    // moves to a free AGPR, else out like an eviction; a load still in flight into it completes first.
    void vacate(int r) {
        if (inflight[r]) wait_seq(inflight[r]);
        if (linflight[r]) wait_lseq(linflight[r]);
        if (owner[r] >= 0) {
            mp->st.cip_evict++;
            if (!is_agpr(r) && !freeA.empty()) {
                const int a = freeA.back();
                freeA.pop_back();
                const int32_t v = owner[r];
                emit(MI_ACCW, a, r);
                mp->st.accw++;
                last_accw[a] = (int)mp->ins.size() - 1;
                owner[a] = v; reg[v] = (int16_t)a; owner[r] = -1;
            } else if (is_agpr(r) && !freeV.empty()) {  // (an AGPR head row's register: to a free VGPR)
                const int t = freeV.back();
                freeV.pop_back();
                const int32_t v = owner[r];
                if (last_accw[r] >= (int)mp->ins.size() - 2) emit(MI_NOP, -1, -1, -1, -1, 1);
                emit(MI_ACCR, t, r);
                mp->st.accr++;
                owner[t] = v; reg[v] = (int16_t)t; owner[r] = -1;
            } else {
                spill_out(r);
            }
        } else {
            std::vector<int>& fl = is_agpr(r) ? freeA : freeV;
            fl.erase(std::remove(fl.begin(), fl.end(), r), fl.end());
        }
        reserved[r] = 1;
    }
    // head loads [f, f + nb) for the next item, issued back to back by one MI_PFX: room for all of them
    // in the vmcnt budget first
    void issue_pfx(uint32_t f, uint32_t nb) {
        for (uint32_t k = 0; k < nb; ++k) vacate(mp->cip_reg[f + k]);
        if (seq - retired + nb > o.max_vmem) wait_seq(seq + nb - o.max_vmem);
        for (uint32_t k = 0; k < nb; ++k) issue_vmem();
        emit(MI_PFX, -1, -1, -1, -1, (f << 16) | nb);
    }
    // operand v into a VGPR (pinned by the caller)
    int to_vgpr(uint32_t v) {
        int r = reg[v];
        if (r < 0) {  // not prefetched: synchronous reload
            if (!has_copy(v)) { fail("colasm: value lost"); return 0; }
            const int t = take_vgpr();
            reload_into(v, t);
            mp->st.sync_reload++;
            r = t;
        }
        if (inflight[r]) wait_seq(inflight[r]);
        if (linflight[r]) wait_lseq(linflight[r]);
        if (is_agpr(r)) {
            pinned[r] = 1;
            const int t = take_vgpr();
            pinned[r] = 0;
            if (last_accw[r] >= (int)mp->ins.size() - 2) emit(MI_NOP, -1, -1, -1, -1, 1);
            emit(MI_ACCR, t, r);
            mp->st.accr++;
            release(r);
            owner[t] = (int32_t)v; reg[v] = (int16_t)t;
            r = t;
        }
        return r;
    }

    bool run() {
        nv = (uint32_t)ir.nodes.size();
        uses.assign(nv, {});
        for (uint32_t i = 0; i < nv; ++i) {
            const IrNode& n = ir.nodes[i];
            for (uint32_t x : {n.a, n.b, n.c})
                if (x != NOVAL) uses[x].push_back(i);
        }
        uptr.assign(nv, 0);
        reg.assign(nv, -1);
        slot.assign(nv, -1);
        lslot.assign(nv, -1);
        slot0 = o.dma4 ? o.n_lds - 4 * o.dma4 : o.n_lds;  // quads at the top of the LDS budget
        for (int s = (int)slot0 - 1; s >= 0; --s) free_lslots.push_back(s);
        quad_left.assign(o.dma4, 0);
        for (uint32_t q = 0; q < o.dma4; ++q) free_quads.push_back(q);
        issued.assign(nv, 0);
        dma_seq.assign(nv, 0);
        for (int r = 0; r < 512; ++r) {
            owner[r] = -1; inflight[r] = 0; linflight[r] = 0; pinned[r] = 0; reserved[r] = 0; last_accw[r] = -100;
        }
        for (int r = (int)o.n_vgpr - 1; r >= 0; --r) freeV.push_back(r);
        for (int r = REG_A0 + (int)o.n_agpr - 1; r >= REG_A0; --r) freeA.push_back(r);
        std::vector<uint32_t> loads;
        for (uint32_t i = 0; i < nv; ++i)
            if (ir.nodes[i].k == IR_LOAD) loads.push_back(i);
        size_t lp = 0, dp = 0;
        mp->ins.clear();
        mp->n_slots = 0;
        mp->n_out = ir.n_out;
        mp->K = ir.p.K;

        std::vector<uint32_t> ld;  // loads with uses, in order: the four-row groups' rows
        for (uint32_t v : loads)
            if (!uses[v].empty()) ld.push_back(v);
        size_t lq = 0;  // next load not yet put in a group
        if (o.dma4) {
            mp->dma4_quads = o.dma4;
            mp->dma4_slot0 = slot0;
            mp->n_lds_slots = std::max<uint32_t>(mp->n_lds_slots, o.n_lds);
            if (!ld.empty()) {  // the first group's table read; each DMA then reads the next group's
                tseq = issue_lgkm();
                emit(MI_DMAT, 0, -1, -1, -1, 0);
            }
        }
        // Cross-item prefetch: the first cip rows (loads with uses) are in flight at the item's start,
        // issued by the previous item's tail into the top VGPRs (the allocator sees them as the item's first
        // loads: its vmcnt counts then also cover the previous item's last stores, conservatively).  From
        // the node after the last source load on, cip_batch of them every cip_gap nodes are re-issued for
        // the next item into the same registers, vacated first.
        const uint32_t n_cipv = o.cip && !o.dma4 && !o.la_dma ? std::min<uint32_t>({o.cip, (uint32_t)ld.size(), o.n_vgpr / 2}) : 0;
        // experiments (cip_agpr): further head rows into the top AGPRs (read back by v_accvgpr_read at use)
        const uint32_t n_cip = n_cipv ? n_cipv + std::min<uint32_t>({o.cip_agpr, (uint32_t)ld.size() - n_cipv, o.n_agpr / 2}) : 0;
        uint32_t t_pf = 0, cip_done = 0;
        for (uint32_t k = 0; k < n_cip; ++k) {
            const uint32_t v = ld[k];
            const int r = k < n_cipv ? (int)o.n_vgpr - 1 - (int)k : REG_A0 + (int)o.n_agpr - 1 - (int)(k - n_cipv);
            std::vector<int>& fl = is_agpr(r) ? freeA : freeV;
            fl.erase(std::remove(fl.begin(), fl.end(), r), fl.end());
            const uint64_t q = issue_vmem();
            emit(MI_HEAD, r, -1, -1, -1, ir.nodes[v].imm);
            mp->st.ldsrc++;
            inflight[r] = q;
            pend_loads.push_back({q, r});
            owner[r] = (int32_t)v; reg[v] = (int16_t)r;
            issued[v] = 1;
            mp->cip_reg.push_back((int16_t)r);
            mp->cip_row.push_back(ir.nodes[v].imm);
        }
        if (n_cip) t_pf = ld.back() + 1;
        for (uint32_t i = 0; i < nv && !failed; ++i) {
            cur = i;
            // -- cross-item prefetch: the next batch of the next item's head loads
            if (cip_done < n_cip && i >= t_pf + (cip_done / std::max<uint32_t>(1, o.cip_batch)) * o.cip_gap) {
                const uint32_t nb = std::min<uint32_t>(std::max<uint32_t>(1, o.cip_batch), n_cip - cip_done);
                issue_pfx(cip_done, nb);
                cip_done += nb;
            }
            // -- four-row staging far ahead: one buffer_load_dwordx4 ... lds per group of four rows
            while (o.dma4 && lq < ld.size() && ld[lq] <= i + o.la_dma) {
                if (free_quads.empty() || seq - retired >= o.max_vmem) break;
                size_t j = lq;
                std::vector<uint32_t> g;
                while (j < ld.size() && g.size() < 4) {
                    if (!issued[ld[j]]) g.push_back(ld[j]);
                    ++j;
                }
                lq = j;
                if (g.empty()) break;
                wait_lseq(tseq);  // this group's row offsets are in the table VGPR
                const uint32_t q = free_quads.front();
                free_quads.pop_front();
                const uint64_t sq = issue_vmem();
                emit(MI_DMA4, (int)q, -1, -1, -1, gj);
                mp->st.dma++;
                for (uint32_t k = 0; k < 4; ++k)
                    mp->dma4_rows.push_back(ir.nodes[g[k < g.size() ? k : 0]].imm);
                quad_left[q] = (uint32_t)g.size();
                for (size_t k = 0; k < g.size(); ++k) {
                    const uint32_t v = g[k];
                    lslot[v] = (int32_t)(slot0 + 4 * q + k);
                    dma_seq[v] = sq;
                    issued[v] = 1;
                    mp->st.ldsrc++;
                    reload_q.push({nu(v), v});
                }
                ++gj;
                if (lq < ld.size()) {  // the next group's table read, into the other table VGPR
                    tseq = issue_lgkm();
                    emit(MI_DMAT, (int)(gj & 1), -1, -1, -1, gj);
                }
            }
            // -- stage source rows in LDS by DMA far ahead (no register held while in flight)
            while (!o.dma4 && o.la_dma && dp < loads.size() && loads[dp] <= i + o.la_dma) {
                const uint32_t v = loads[dp];
                if (issued[v] || uses[v].empty()) { ++dp; continue; }
                if (seq - retired >= o.max_vmem) break;
                if (!issue_dma(v)) break;
                ++dp;
            }
            // -- prefetch source rows into registers (rows not staged).  load_batch = B > 1 (experiments):
            // hold the prefetches until B rows are due (or the next is needed within 8 nodes), then issue
            // B back to back (fewer load/VALU transitions of the in-order issue)
            {
                const uint32_t B = std::max<uint32_t>(1, o.load_batch);
                // experiments (la_extra): a deeper look-ahead while la_free registers are free (the head and
                // the tail of the program, where the live set is well below the file)
                const uint32_t la = o.la_load + (o.la_extra && freeV.size() + freeA.size() >= o.la_free ? o.la_extra : 0);
                size_t due = 0;
                while (lp + due < loads.size() && loads[lp + due] <= i + la) ++due;
                const bool go = B == 1 || due >= B || (lp < loads.size() && loads[lp] <= i + 8);
                size_t quota = go ? std::max<size_t>(due, B) : 0;
                while (quota && lp < loads.size()) {
                    const uint32_t v = loads[lp];
                    if (issued[v]) { ++lp; continue; }
                    if (uses[v].empty()) { issued[v] = 1; ++lp; continue; }
                    if (B == 1 && v > i + la) break;
                    if (seq - retired >= o.max_vmem && v > i) break;
                    const int r = take_any(uses[v][0]);
                    if (r < 0) break;
                    issue_load(v, r);
                    ++lp;
                    --quota;
                }
            }
            // -- prefetch scratch reloads
            while (!reload_q.empty() && reload_q.top().first <= i + o.la_reload) {
                const HE e = reload_q.top();
                const uint32_t v = e.second;
                if (reg[v] >= 0 || !has_copy(v) || nu(v) != e.first) { reload_q.pop(); continue; }
                if (seq - retired >= o.max_vmem && e.first > i + 8) break;
                const int r = take_any(e.first);
                if (r < 0) break;
                reload_q.pop();
                reload_into(v, r);
            }
            const IrNode& n = ir.nodes[i];
            switch (n.k) {
                case IR_LOAD: {
                    if (!issued[i] && !uses[i].empty()) {
                        const int r = take_vgpr();
                        issue_load(i, r);
                    }
                    break;
                }
                case IR_SEND: {  // pair programs, wave A: value -> ring slot (ds_write_b32; VGPR or AGPR data)
                    const uint32_t v = n.a;
                    int r = reg[v];
                    if (r < 0) {
                        if (!has_copy(v)) { fail("colasm: send of a lost value"); break; }
                        r = take_vgpr();
                        reload_into(v, r);
                        mp->st.sync_reload++;
                    }
                    if (inflight[r]) wait_seq(inflight[r]);
                    if (linflight[r]) wait_lseq(linflight[r]);
                    issue_lgkm();
                    emit(MI_RST, -1, r, -1, -1, n.imm);
                    mp->st.rst++;
                    uptr[v]++;
                    if (nu(v) == INF) kill(v);
                    break;
                }
                case IR_RECV: {  // pair programs, wave B: ring slot -> register (ds_read_b32)
                    if (uses[i].empty()) break;
                    int r = -1;
                    if (uses[i][0] > i + o.lds_horizon) r = take_any(uses[i][0]);  // used much later: any register
                    if (r < 0) r = take_vgpr();
                    const uint64_t q = issue_lgkm();
                    emit(MI_RLD, r, -1, -1, -1, n.imm);
                    mp->st.rld++;
                    linflight[r] = q;
                    pend_lds.push_back({q, r});
                    owner[r] = (int32_t)i; reg[i] = (int16_t)r;
                    break;
                }
                case IR_BAR: {  // pair programs: the transfer's LDS operations complete, then the barrier
                    if (lseq > lretired) {
                        emit(MI_WAITL, -1, -1, -1, -1, 0);
                        mp->st.waitl++;
                        retire_l(lseq);
                    }
                    emit(MI_BAR, -1, -1, -1, -1, n.imm);
                    mp->st.bar++;
                    break;
                }
                case IR_STORE: {
                    const uint32_t v = n.a;
                    int r = reg[v];
                    if (r < 0) {
                        if (!has_copy(v)) { fail("colasm: store of a lost value"); break; }
                        r = take_vgpr();
                        reload_into(v, r);
                        mp->st.sync_reload++;
                    }
                    if (inflight[r]) wait_seq(inflight[r]);
                    if (linflight[r]) wait_lseq(linflight[r]);
                    const uint64_t q = issue_vmem();
                    (void)q;
                    emit(MI_STOUT, -1, r, -1, -1, n.imm);
                    mp->st.stout++;
                    uptr[v]++;
                    if (nu(v) == INF) kill(v);
                    break;
                }
                default: {
                    uint32_t ops[3] = {n.a, n.b, n.c};
                    int nops = (n.k == IR_ZERO) ? 0 : (n.k == IR_XOR3 ? 3 : (n.k == IR_XT ? 1 : 2));
                    int rr[3] = {-1, -1, -1};
                    for (int q = 0; q < nops; ++q)
                        if (reg[ops[q]] >= 0) pinned[reg[ops[q]]] = 1;
                    for (int q = 0; q < nops; ++q) {
                        rr[q] = to_vgpr(ops[q]);
                        pinned[rr[q]] = 1;
                    }
                    // consume uses; find a dying operand register to reuse for the result
                    int dst = -1;
                    for (int q = 0; q < nops; ++q) {
                        const uint32_t v = ops[q];
                        bool dup = false;
                        for (int p = 0; p < q; ++p) dup |= (ops[p] == v);
                        if (dup) continue;
                        while (uptr[v] < uses[v].size() && uses[v][uptr[v]] == i) uptr[v]++;
                    }
                    for (int q = 0; q < nops && dst < 0; ++q)
                        if (nu(ops[q]) == INF) dst = rr[q];
                    if (dst < 0) dst = take_vgpr();
                    pinned[dst] = 1;
                    uint8_t op = MI_XOR2;
                    switch (n.k) {
                        case IR_ZERO: op = MI_ZERO; break;
                        case IR_XOR2: op = MI_XOR2; break;
                        case IR_XOR3: op = MI_XOR3; break;
                        case IR_XT: op = MI_XT; break;
                        case IR_XTX: op = MI_XTX; break;
                    }
                    emit(op, dst, rr[0], rr[1], rr[2]);
                    mp->st.valu++;
                    for (int q = 0; q < nops; ++q) {
                        const uint32_t v = ops[q];
                        pinned[rr[q]] = 0;
                        if (nu(v) == INF && reg[v] >= 0) {
                            if (reg[v] == dst) {
                                reg[v] = -1; owner[dst] = -1;
                                if (slot[v] >= 0) { free_slots.push_back(slot[v]); slot[v] = -1; }
                                if (lslot[v] >= 0) free_lds(v);
                            }
                            else kill(v);
                        }
                    }
                    pinned[dst] = 0;
                    owner[dst] = (int32_t)i; reg[i] = (int16_t)dst;
                    if (uses[i].empty()) kill(i);
                    break;
                }
            }
        }
        // a short tail: the rest of the prefetch at the end
        while (!failed && cip_done < n_cip) {
            const uint32_t nb = std::min<uint32_t>(std::max<uint32_t>(1, o.cip_batch), n_cip - cip_done);
            issue_pfx(cip_done, nb);
            cip_done += nb;
        }
        return !failed;
    }
};

}  // namespace

bool allocate_colprog(const ColIR& ir, const AllocOpts& o, MProg* mp, std::string* err) {
    *mp = MProg();
    if (o.n_vgpr < 8 || o.n_vgpr > V_ALLOC || o.n_agpr > 256 || o.n_lds > 512) {  // 2 LDS bases
        if (err) *err = "colasm: register budget out of range";
        return false;
    }
    mp->n_vgpr = o.n_vgpr;
    mp->n_agpr = o.n_agpr;
    Allocator a(ir, o, mp, err);
    return a.run();
}

// One wave per SIMD issues one instruction per 4-cycle slot whatever its kind, so the launch time is
// close to linear in issue slots (an xtime is 5 VALU instructions; an output store carries the SALU that
// forms its soffset, a source load 1/8 of an s_load + wait), plus a stall term per global-scratch spill or reload.  Least-squares fit
// over the K=1024 schedule sweep (profiles/r02g/passes_sweep.log): 7.6e-6 ms per slot and 12 slots
// per scratch access, within 2 % on all seven points.
double colprog_cost(const MProg& mp) {
    double slots = 0;
    for (const MInst& m : mp.ins) {
        switch (m.op) {
            case MI_XT: case MI_XTX: slots += 5; break;
            case MI_LDSRC: slots += 1.125; break;
            case MI_STOUT: slots += 2; break;
            case MI_HEAD: break;  // issued by the previous item's MI_PFX
            case MI_PFX: slots += 2.0 * (m.imm & 0xFFFFu) + 2 + ((m.imm >> 16) ? 0 : 18); break;
            default: slots += 1;
        }
    }
    return slots + 12.0 * (double)(mp.st.spst + mp.st.spld);
}

bool compile_colprog(const Params& p, const uint32_t* esi, uint32_t n_out, const AllocOpts& o, ColIR* ir, MProg* mp,
                     std::string* err, uint32_t* passes_out, bool search_waves) {
    double best = 0;
    bool have = false;
    // P Horner passes, or no scan at all (SCHED_4R: bh bit by bit, XOR now when the accumulator's
    // next push is more than 64 productions away); K=1024: P = 2 32.0 k slots, 4R 25.8 k (no spills)
    std::vector<uint32_t> cand{0u, 1u, 2u, 3u, 4u, 5u, 6u, SCHED_4R | 64u, SCHED_4R};
    if (const char* f = knob("RQHIP_PASSES")) cand = {(uint32_t)std::atoi(f)};  // experiments: fixed schedule
    for (uint32_t P : cand) {
        ColIR cir;
        MProg cmp;
        const bool ok = esi ? build_colprog(p, esi, n_out, &cir, err, P) : build_colprog_C(p, &cir, err, P);
        if (!ok || !allocate_colprog(cir, o, &cmp, err)) {
            if (P == 0) return false;
            continue;
        }
        const double c = colprog_cost(cmp);
        if (!have || c < best) {
            best = c;
            have = true;
            *ir = std::move(cir);
            *mp = std::move(cmp);
            if (passes_out) *passes_out = P;
        }
        if (P == 0 && cmp.st.spst == 0) break;  // fits on chip: the single scan is cheapest
    }
    if (!have || !search_waves || mp->st.spst) return have;
    // A program that fits on chip at one wave per SIMD may fit at 2, 4 or 8: another wave on the SIMD
    // then issues while one waits on memory.  Take the highest residency whose program still needs no
    // global scratch and at most 1.5x the instructions (measured: K=128 4 waves -24 %, K=256 2 waves
    // -13 %, K=512 spills at 2 waves and loses, profiles/r02ab).
    const size_t ins1 = mp->ins.size();
    // VGPR, AGPR, LDS slots for 2 / 4 / 8 waves per SIMD; experiments: RQHIP_W3=1 adds 3 (170 registers)
    static const std::vector<std::array<uint32_t, 3>> cap = [] {
        std::vector<std::array<uint32_t, 3>> c{{122, 128, 78}, {58, 64, 39}, {26, 32, 19}};
        if (const char* e = knob("RQHIP_W3"))
            if (e[0] == '1') c.insert(c.begin() + 1, {78, 86, 52});
        return c;
    }();
    for (const auto& c : cap) {
        AllocOpts w = o;
        w.cip = 0;  // the SIMD's other waves issue while one waits at its item's start
        w.n_vgpr = std::min(o.n_vgpr, c[0]);
        w.n_agpr = std::min(o.n_agpr, c[1]);
        w.n_lds = std::min(o.n_lds, c[2]);
        ColIR cir;
        MProg cmp;
        std::string e2;
        const bool ok = esi ? build_colprog(p, esi, n_out, &cir, &e2, 0) : build_colprog_C(p, &cir, &e2, 0);
        if (!ok || !allocate_colprog(cir, w, &cmp, &e2) || cmp.st.spst || cmp.ins.size() * 2 > ins1 * 3) break;
        *ir = std::move(cir);
        *mp = std::move(cmp);
        if (passes_out) *passes_out = 0;
    }
    return have;
}

bool divmagic(uint32_t d, uint32_t limit, uint32_t* magic, uint32_t* shift) {
    if (d == 0) return false;
    for (uint32_t s = 0; s < 32; ++s) {
        const uint64_t m = (((uint64_t)1 << (32 + s)) + d - 1) / d;
        if (m > 0xFFFFFFFFull) break;
        // exact for g < limit if the error term stays below one step
        const uint64_t e = m * d - ((uint64_t)1 << (32 + s));
        if ((uint64_t)limit * e < ((uint64_t)1 << (32 + s))) {
            *magic = (uint32_t)m;
            *shift = s;
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------------------------------
// First AGPR in the unified register file: above the allocatable VGPRs and the reserved ones (four more
// with four-row staging -- they must not alias an AGPR).
uint32_t colprog_acc_off(const MProg& mp) {
    return (mp.n_vgpr + (mp.dma4_quads ? N_RESERVED_DMA4 : N_RESERVED) + 3) & ~3u;
}

uint32_t colprog_regs(const MProg& mp) {
    return (colprog_acc_off(mp) + std::max<uint32_t>(mp.n_agpr, 1) + 7) & ~7u;
}

// SGPR map of the emitted kernel beyond the prologue's s0..s55: s56..s63 scratch soffset bases,
// s64..s79 / s80..s95 the two halves of the double-buffered source row-offset window.

std::vector<uint32_t> colprog_src_rows(const MProg& mp) {
    static const uint32_t diag = diag_mask();
    std::vector<uint32_t> rows;
    if (diag & 4) return rows;
    for (const MInst& m : mp.ins)
        if (m.op == MI_LDSRC) rows.push_back((diag & 16) ? (uint32_t)(rows.size() % mp.K) : m.imm);
    return rows;
}

uint32_t colprog_row_end(const MProg& mp) {
    uint32_t e = 1;
    for (const MInst& m : mp.ins)
        if (m.op == MI_LDSRC || m.op == MI_DMA || m.op == MI_HEAD) e = std::max(e, m.imm + 1);
    for (uint32_t r : mp.dma4_rows) e = std::max(e, r + 1);
    return e;
}

// Scratch slot s sits at soffset 4096 * (s / 16) + offset (s % 16) * 256: soffset 0 or one of
// SCR_BASES SGPRs s56.. loaded once by the prologue; slots beyond them (very large K) form their
// soffset with an s_mov.
uint32_t scratch_bases(const MProg& mp) {
    return std::min<uint32_t>(SCR_BASES, mp.n_slots > 16 ? (mp.n_slots - 1) / 16 : 0);
}

// Cross-item prefetch (MProg::cip_*): head loads [first, first + n) of the item at workgroup iteration
// s52 + s49 (the wave's next item; the prologue: s52, its first item).  The first batch forms the item's
// lane offset as the loop top forms V_SRCOFF, into V_LDS2 (free: the program's LDS slots stay below 256)
// through the xtime temporaries, and its lane mask (columns below n_cols) into s[54:55] (free until the
// loop end's s_getpc); later batches reuse both.  Each load's soffset is row * T by an s_mul (SALU
// temporaries s39 / s40 / s42..s47 are dead between the body's instructions at W = 1).  Past the wave's
// last item the loads re-read the current item's rows (V_SRCOFF under its own mask): the allocator counts
// them in its vmcnt waits, so they are issued either way.  The prologue skips a wave that has no item.
void emit_cip_loads(const MProg& mp, uint32_t first, uint32_t n, bool next, uint32_t label, std::string& s) {
    static const Policy pol;
    const Reserved rv(mp.n_vgpr);
    char buf[256];
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    auto lab = [&](const char* t) { std::snprintf(buf, sizeof buf, ".Lcip%s%u:\n", t, label); s += buf; };
    auto R = [&](int r) { return std::string(is_agpr(r) ? "a" : "v") + std::to_string(is_agpr(r) ? r - REG_A0 : r); };
    if (first == 0) {
        line(next ? "s_add_u32 s39, s52, s49" : "s_mov_b32 s39, s52");
        line("s_cmp_lt_u32 s39, s48");
        if (next) {
            std::snprintf(buf, sizeof buf, "s_cbranch_scc1 .Lcipn%u", label); line(buf);
            std::snprintf(buf, sizeof buf, "v_mov_b32_e32 v%d, v%d", rv.lds2, rv.srcoff); line(buf);
            line("s_mov_b64 s[54:55], s[22:23]");
            std::snprintf(buf, sizeof buf, "s_branch .Lcipg%u", label); line(buf);
            lab("n");
            line("s_mov_b64 exec, -1");  // the next item's offsets and mask on every lane, whatever this item's mask
        } else {
            std::snprintf(buf, sizeof buf, "s_cbranch_scc0 .Lcipe%u", label); line(buf);
        }
        line("s_and_b32 s40, s39, 7");
        line("s_mul_i32 s40, s40, s17");
        line("s_lshr_b32 s42, s39, 3");
        line("s_add_u32 s40, s40, s42");
        line("s_cmp_lt_u32 s39, s18");
        line("s_cselect_b32 s39, s40, s39");
        line("s_lshl_b32 s39, s39, 6");
        std::snprintf(buf, sizeof buf, "v_mbcnt_lo_u32_b32 v%d, -1, 0", rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_mbcnt_hi_u32_b32 v%d, -1, v%d", rv.t1, rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_add_u32_e32 v%d, s39, v%d", rv.t1, rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_cmp_gt_u32_e64 s[54:55], s13, v%d", rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_mul_hi_u32 v%d, v%d, s14", rv.t2, rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_lshrrev_b32_e32 v%d, s15, v%d", rv.t2, rv.t2); line(buf);
        std::snprintf(buf, sizeof buf, "v_mul_lo_u32 v%d, v%d, s21", rv.lds2, rv.t2); line(buf);
        std::snprintf(buf, sizeof buf, "v_sub_u32_e32 v%d, v%d, v%d", rv.t1, rv.t1, rv.lds2); line(buf);
        std::snprintf(buf, sizeof buf, "v_lshlrev_b32_e32 v%d, 2, v%d", rv.t1, rv.t1); line(buf);
        std::snprintf(buf, sizeof buf, "v_mul_lo_u32 v%d, v%d, s10", rv.lds2, rv.t2); line(buf);
        std::snprintf(buf, sizeof buf, "v_add_u32_e32 v%d, v%d, v%d", rv.lds2, rv.lds2, rv.t1); line(buf);
        if (next) lab("g");
    }
    line("s_mov_b64 exec, s[54:55]");
    for (uint32_t k = first; k < first + n; ++k) {
        // the prologue issues every head row at once: at most 48 outstanding before the next, well inside
        // the 6-bit vmcnt (the tail's batches are bounded by the allocator, issue_pfx)
        if (!next && k > first && (k - first) % 48 == 0) line("s_waitcnt vmcnt(24)");
        const int q = 42 + (int)(k % 6);
        std::snprintf(buf, sizeof buf, "s_mul_i32 s%d, s12, %u", q, mp.cip_row[k]); line(buf);
        std::snprintf(buf, sizeof buf, "buffer_load_dword %s, v%d, s[24:27], s%d offen%s", R(mp.cip_reg[k]).c_str(), rv.lds2, q,
                      pol.src.c_str());
        line(buf);
    }
    line(next ? "s_mov_b64 exec, s[22:23]" : "s_mov_b64 exec, -1");
    if (!next) lab("e");
}

// The per-item instruction stream of an allocated program (the body of the persistent loop): the
// source row-offset window (A / single-wave programs), scratch soffsets, and every MInst.  Shared by
// the single-wave kernel (emit_colprog_asm) and both waves of a pair kernel (emit_pair_asm).  W: waves
// per workgroup of the single-wave layout (MI_DMA's per-wave LDS base in s41 when W > 1).
void emit_colprog_body(const MProg& mp, uint32_t W, std::string& s) {
    static const Policy pol;
    static const uint32_t diag = diag_mask();
    static const uint32_t wgbar = [] { const char* e = knob("RQHIP_WGBAR"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    const Reserved rv(mp.n_vgpr);
    const int V_T1 = rv.t1, V_T2 = rv.t2, V_SCROFF = rv.scroff, V_OUTOFF = rv.outoff, V_SRCOFF = rv.srcoff;
    const uint32_t n_bases = scratch_bases(mp);
    char buf[256];
    auto R = [&](int r) {
        static thread_local char b[2][16];
        static thread_local int k = 0;
        k ^= 1;
        std::snprintf(b[k], sizeof b[k], is_agpr(r) ? "a%d" : "v%d", is_agpr(r) ? r - REG_A0 : r);
        return b[k];
    };
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    // LDS slot sl (256 B per lane row) of this program: offset (sl & 255) * 256 from V_SCROFF (the lane's
    // 4 B) or from V_LDS2 = V_SCROFF + 64 KiB (the ds offset field is 16 bits)
    auto lds_at = [&](uint32_t sl, int* vbase) {
        *vbase = sl < 256 ? V_SCROFF : rv.lds2;
        return (sl & 255u) * 256u;
    };
    // Source row j of the program (in issue order) is read at soffset row_off[j] = row * T, a
    // host-built table (colprog_src_rows) streamed into SGPRs 16 entries at a time by s_load_dwordx16,
    // one group ahead: a source load carries no SALU of its own, only one s_load and one
    // lgkmcnt(0) per 16 loads.  (LDS waits counted by the allocator only get stricter from the
    // extra outstanding scalar load.)
    const std::vector<uint32_t> src_rows = colprog_src_rows(mp);
    const uint32_t n_groups = (uint32_t)((src_rows.size() + 15) / 16);
    // experiments: RQHIP_SRC_SMUL=1 forms each source load's soffset with an s_mul (one SALU per load)
    // instead (no lgkmcnt(0) per 16 loads, which also drains the LDS operations in flight)
    static const bool src_smul = [] { const char* e = knob("RQHIP_SRC_SMUL"); return e && e[0] == '1'; }();
    if (n_groups && !src_smul) line("s_load_dwordx16 s[64:79], s[50:51], 0x0");
    uint32_t src_j = 0;
    int sr = 0;
    // s40..s47 rotate as short-lived SALU temporaries; at W > 1, s41 holds the wave's LDS base for the
    // whole kernel (MI_DMA's m0), so the rotation skips it
    auto srot = [&]() {
        do sr = (sr + 1) & 7; while (W > 1 && sr == 1);
        return 40 + sr;
    };
    auto scr_soff = [&](uint32_t slot) -> std::string {
        const uint32_t j = slot / 16;
        if (j == 0) return "0";
        if (j <= n_bases) return "s" + std::to_string(56 + j - 1);
        const int q = srot();
        std::snprintf(buf, sizeof buf, "s_mov_b32 s%d, %u", q, 4096u * j);
        line(buf);
        return "s" + std::to_string(q);
    };
    for (const MInst& m : mp.ins) {
        if ((diag & 32) && m.op <= MI_ZERO) continue;  // memory-only timing: no XOR / xtime work
        switch (m.op) {
            case MI_XOR2:
                std::snprintf(buf, sizeof buf, "v_xor_b32_e32 v%d, v%d, v%d", m.d, m.a, m.b); line(buf); break;
            case MI_XOR3:
                std::snprintf(buf, sizeof buf, "v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", m.d, m.a, m.b, m.c); line(buf); break;
            case MI_XT:
            case MI_XTX:
                // alpha*a (+ b) per byte in 5 VALU: m = 0xff where a byte's top bit is set (v_perm sign
                // select over {a << 8, a}); z = (m & 0x1d..) [^ b]; result = ((a << 1) & 0xfe..) ^ z.
                // bitop3 0x6c = (S0 & S2) ^ S1, symmetric in S0/S2 so operand order cannot flip it.
                std::snprintf(buf, sizeof buf, "v_lshlrev_b32_e32 v%d, 8, v%d", V_T1, m.a); line(buf);
                std::snprintf(buf, sizeof buf, "v_perm_b32 v%d, v%d, v%d, s36", V_T1, V_T1, m.a); line(buf);
                if (m.op == MI_XT) std::snprintf(buf, sizeof buf, "v_and_b32_e32 v%d, s38, v%d", V_T1, V_T1);
                else std::snprintf(buf, sizeof buf, "v_bitop3_b32 v%d, v%d, v%d, s38 bitop3:0x6c", V_T1, V_T1, m.b);
                line(buf);
                std::snprintf(buf, sizeof buf, "v_lshlrev_b32_e32 v%d, 1, v%d", V_T2, m.a); line(buf);
                std::snprintf(buf, sizeof buf, "v_bitop3_b32 v%d, v%d, v%d, s37 bitop3:0x6c", m.d, V_T2, V_T1); line(buf);
                break;
            case MI_ZERO:
                std::snprintf(buf, sizeof buf, "v_mov_b32_e32 v%d, 0", m.d); line(buf); break;
            case MI_LDSRC: {
                if (diag & 4) {
                    std::snprintf(buf, sizeof buf, is_agpr(m.d) ? "v_accvgpr_write_b32 %s, v%d" : "v_mov_b32_e32 %s, v%d",
                                  R(m.d), V_SRCOFF);
                    line(buf);
                    break;
                }
                if (src_smul) {
                    ++src_j;
                    const int q = srot();
                    std::snprintf(buf, sizeof buf, "s_mul_i32 s%d, s12, %u", q, m.imm); line(buf);
                    std::snprintf(buf, sizeof buf, "buffer_load_dword %s, v%d, s[24:27], s%d offen%s", R(m.d), V_SRCOFF, q,
                                  pol.src.c_str());
                    line(buf);
                    break;
                }
                const uint32_t g = src_j / 16, i = src_j % 16, win = ROW_WIN + 16 * (g & 1);
                if (i == 0) {
                    line("s_waitcnt lgkmcnt(0)");
                    if (g + 1 < n_groups) {
                        std::snprintf(buf, sizeof buf, "s_load_dwordx16 s[%u:%u], s[50:51], 0x%x", ROW_WIN + 16 * ((g + 1) & 1),
                                      ROW_WIN + 16 * ((g + 1) & 1) + 15, (g + 1) * 64);
                        line(buf);
                    }
                }
                // W > 1, experiments: an s_barrier every `wgbar` source loads keeps the workgroup's waves
                // at the same rows (every wave runs this same stream, so the barrier counts match)
                if (W > 1 && wgbar && src_j && src_j % wgbar == 0) line("s_barrier");
                ++src_j;
                std::snprintf(buf, sizeof buf, "buffer_load_dword %s, v%d, s[24:27], s%u offen%s", R(m.d), V_SRCOFF, win + i,
                              pol.src.c_str());
                line(buf);
                break;
            }
            case MI_DMA: {
                if (diag & 4) break;
                const int q = srot();
                std::snprintf(buf, sizeof buf, "s_mul_i32 s%d, s12, %u", q, m.imm); line(buf);
                const uint32_t dsl = (uint32_t)m.d + mp.lds_base;
                if (W > 1) std::snprintf(buf, sizeof buf, "s_add_u32 m0, s41, %u", dsl * 256u);
                else std::snprintf(buf, sizeof buf, "s_mov_b32 m0, %u", dsl * 256u);
                line(buf);
                line("s_nop 0");
                std::snprintf(buf, sizeof buf, "buffer_load_dword v%d, s[24:27], s%d offen%s lds", V_SRCOFF, q, pol.src.c_str());
                line(buf);
                break;
            }
            case MI_STOUT: {
                if (diag & 8) break;
                const int q = srot();
                std::snprintf(buf, sizeof buf, "s_mul_i32 s%d, s12, %u", q, m.imm); line(buf);
                std::snprintf(buf, sizeof buf, "buffer_store_dword %s, v%d, s[28:31], s%d offen%s", R(m.a), V_OUTOFF, q, pol.out.c_str()); line(buf);
                break;
            }
            case MI_SPST: {
                if (diag & 1) break;
                const std::string so = scr_soff(m.imm);
                std::snprintf(buf, sizeof buf, "buffer_store_dword %s, v%d, s[32:35], %s offen offset:%u%s", R(m.a), V_SCROFF,
                              so.c_str(), (m.imm & 15u) * 256u, pol.scr_st.c_str());
                line(buf);
                break;
            }
            case MI_SPLD: {
                if (diag & 1) break;
                const std::string so = scr_soff(m.imm);
                std::snprintf(buf, sizeof buf, "buffer_load_dword %s, v%d, s[32:35], %s offen offset:%u%s", R(m.d), V_SCROFF,
                              so.c_str(), (m.imm & 15u) * 256u, pol.scr_ld.c_str());
                line(buf);
                break;
            }
            case MI_ACCW:
                std::snprintf(buf, sizeof buf, "v_accvgpr_write_b32 %s, v%d", R(m.d), m.a); line(buf); break;
            case MI_ACCR:
                std::snprintf(buf, sizeof buf, "v_accvgpr_read_b32 v%d, %s", m.d, R(m.a)); line(buf); break;
            case MI_WAIT:
                if (diag & 64) break;  // diagnostic: no vmcnt waits (wrong bytes; addresses stay valid)
                std::snprintf(buf, sizeof buf, "s_waitcnt vmcnt(%u)", m.imm); line(buf); break;
            case MI_NOP:
                std::snprintf(buf, sizeof buf, "s_nop %u", m.imm); line(buf); break;
            case MI_DMAT: {  // row offsets of group imm for this lane's row group (table at LDS 0), all lanes
                line("s_mov_b64 exec, -1");
                std::snprintf(buf, sizeof buf, "ds_read_b32 v%d, v%d offset:%u", m.d ? rv.tbl1 : rv.tbl0, rv.grp4,
                              m.imm * 16u);
                line(buf);
                line("s_mov_b64 exec, s[22:23]");
                break;
            }
            case MI_DMA4: {  // lane l: 16 B of row (l / 16) of the group at its chunk base -> quad d, all lanes
                const int tr = (m.imm & 1u) ? rv.tbl1 : rv.tbl0;
                line("s_mov_b64 exec, -1");
                std::snprintf(buf, sizeof buf, "v_add_u32_e32 v%d, v%d, v%d", tr, rv.dmabase, tr); line(buf);
                std::snprintf(buf, sizeof buf, "s_mov_b32 m0, %u", (mp.lds_base + mp.dma4_slot0 + 4u * (uint32_t)m.d) * 256u);
                line(buf);
                line("s_nop 0");
                std::snprintf(buf, sizeof buf, "buffer_load_dwordx4 v%d, s[24:27], 0 offen lds%s", tr, pol.src.c_str());
                line(buf);
                line("s_mov_b64 exec, s[22:23]");
                break;
            }
            case MI_LDST:
            case MI_RST: {  // spill slots sit after the ring (lds_base); ring slots after the group table
                if (diag & 2 && m.op == MI_LDST) break;
                int vb;
                const uint32_t off = lds_at(m.op == MI_RST ? m.imm + mp.ring_base : m.imm + mp.lds_base, &vb);
                std::snprintf(buf, sizeof buf, "ds_write_b32 v%d, %s offset:%u", vb, R(m.a), off);
                line(buf);
                break;
            }
            case MI_LDLD:
            case MI_RLD: {
                if (diag & 2 && m.op == MI_LDLD) break;
                int vb;
                const uint32_t off = lds_at(m.op == MI_RLD ? m.imm + mp.ring_base : m.imm + mp.lds_base, &vb);
                std::snprintf(buf, sizeof buf, "ds_read_b32 %s, v%d offset:%u", R(m.d), vb, off);
                line(buf);
                break;
            }
            case MI_BAR:
                if (diag & 128) break;
                line("s_barrier");
                break;
            case MI_WAITL:
                std::snprintf(buf, sizeof buf, "s_waitcnt lgkmcnt(%u)", m.imm); line(buf); break;
            case MI_HEAD:
                break;  // in flight since the previous item's MI_PFX (or the prologue)
            case MI_PFX:
                if (diag & 4) break;
                emit_cip_loads(mp, m.imm >> 16, m.imm & 0xFFFFu, true, 1 + (m.imm >> 16), s);
                break;
        }
    }
}

std::vector<uint32_t> colprog_row_table(const MProg& mp, uint32_t T) {
    const std::vector<uint32_t> rows = colprog_src_rows(mp);
    std::vector<uint32_t> off((rows.size() + 15) / 16 * 16 + 16, 0);
    for (size_t j = 0; j < rows.size(); ++j) off[j] = rows[j] * T;
    for (uint32_t r : mp.dma4_rows) off.push_back(r * T);
    return off;
}

uint32_t colprog_dma4_table_offset(const MProg& mp) {
    return (uint32_t)((colprog_src_rows(mp).size() + 15) / 16 * 16 + 16) * 4u;
}

std::string emit_colprog_asm(const MProg& mp, const std::string& kname) {
    static const Policy pol;
    static const uint32_t diag = diag_mask();
    const Reserved rv(mp.n_vgpr);
    const int V_SCROFF = rv.scroff, V_OUTOFF = rv.outoff, V_SRCOFF = rv.srcoff;
    const uint32_t acc_off = colprog_acc_off(mp);  // first AGPR in the unified file
    const uint32_t n_regs = colprog_regs(mp);
    std::string s;
    s.reserve(mp.ins.size() * 48 + 8192);
    char buf[256];
    auto line = [&](const char* t) { s += '\t'; s += t; s += '\n'; };
    s += "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.amdhsa_code_object_version 6\n\t.text\n";
    s += "\t.globl " + kname + "\n\t.p2align 8\n\t.type " + kname + ",@function\n" + kname + ":\n";
    // Persistent loop: the grid holds as many waves as can be resident (the host sets n_wg = s49);
    // wave w processes items w, w + n_wg, ... < n_items (s48), so its scratch lines are reused by
    // its own next item instead of a fresh wave's, and the scratch footprint stays at the
    // resident set.  One item = 64 dword columns (the lane -> (block, column) map below).
    const char* pro_once[] = {
        "s_load_dwordx8 s[4:11], s[0:1], 0x0",
        "s_load_dwordx8 s[12:19], s[0:1], 0x20",
        "s_load_dwordx4 s[48:51], s[0:1], 0x40",
        "s_waitcnt lgkmcnt(0)",
        "CPFETCH",
        "v_lshlrev_b32_e32 V_SCROFF, 2, v0",
        "v_add_u32_e32 V_LDS2, 0x10000, V_SCROFF",
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
    };
    const char* pro_iter[] = {
        // (the program is longer than a 16-bit branch reaches: exit in place, loop back by s_setpc)
        "s_cmp_lt_u32 s52, s48",
        "s_cbranch_scc1 .Lbody",
        "s_endpgm",
        ".Lbody:",
        "s_mov_b64 exec, -1",
        // XCD-aware item order: workgroups are dealt to the 8 XCDs round-robin, so logical item
        // L = (w % 8) * q + w / 8 (for w < 8q; s17 = q, s18 = 8q, both 0 = identity) keeps the
        // items of one block, which share the 128-B lines at their 256-B segment edges, on one L2.
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
    const uint32_t W = std::max<uint32_t>(1, mp.wg_waves);
    if (!mp.cip_reg.empty() && (W > 1 || mp.dma4_quads || mp.lds_base + mp.n_lds_slots > 256))
        s += "\t.error \"cross-item prefetch needs W = 1 and LDS slots below 256 (V_LDS2 holds its offsets)\"\n";
    auto put = [&](const char* p) {
        std::string l(p);
        if (l == "CPFETCH") {
            if (mp.n_vgpr < 24) return;  // (v1..v23 below; the host launches no fetch workgroups then)
            // Descriptor fetch (ColKernArgs::cp_*, a decode's syndrome launch): workgroups past the
            // persistent grid (s2 >= n_wg = s49) copy their cp_chunk-byte piece of the descriptors from
            // pinned host memory to the device, four 16-byte loads per lane in flight (4 KiB per wave
            // per round trip; cp_bytes and cp_chunk are multiples of 4 KiB x W), and exit.  They run on
            // the SIMDs the grid leaves free, beside the program; the solve that reads the copy is the
            // next kernel in the stream.  Vector loads and stores only.
            const uint32_t WB = 1024u * W;  // bytes per workgroup per load
            line("s_cmp_lt_u32 s2, s49");
            line("s_cbranch_scc1 .Ldmain");
            line("s_load_dwordx4 s[56:59], s[0:1], 0x50");  // cp_src, cp_dst
            line("s_load_dwordx2 s[60:61], s[0:1], 0x60");  // cp_bytes, cp_chunk
            line("s_waitcnt lgkmcnt(0)");
            line("s_sub_u32 s62, s2, s49");
            line("s_mul_i32 s62, s62, s61");   // the piece's first byte
            line("s_add_u32 s63, s62, s61");
            line("s_min_u32 s63, s63, s60");   // its end
            line("v_lshlrev_b32_e32 v1, 4, v0");
            line("v_add_u32_e32 v1, s62, v1");
            s += ".Ldcp:\n";
            line("v_cmp_gt_u32_e32 vcc, s63, v1");
            line("s_and_b64 exec, exec, vcc");
            line("s_cbranch_execz .Ldcpend");
            for (uint32_t u = 1; u < 4; ++u) {
                std::snprintf(buf, sizeof buf, "v_add_u32_e32 v%u, 0x%x, v1", 1 + u, u * WB);
                line(buf);
            }
            // addresses in v1..v4, data in v[8:23] (disjoint: a store's address must survive the loads)
            for (uint32_t u = 0; u < 4; ++u) {
                std::snprintf(buf, sizeof buf, "global_load_dwordx4 v[%u:%u], v%u, s[56:57]", 8 + 4 * u, 11 + 4 * u, 1 + u);
                line(buf);
            }
            line("s_waitcnt vmcnt(0)");
            for (uint32_t u = 0; u < 4; ++u) {
                std::snprintf(buf, sizeof buf, "global_store_dwordx4 v%u, v[%u:%u], s[58:59]", 1 + u, 8 + 4 * u, 11 + 4 * u);
                line(buf);
            }
            std::snprintf(buf, sizeof buf, "v_add_u32_e32 v1, 0x%x, v1", 4u * WB);
            line(buf);
            line("s_branch .Ldcp");
            s += ".Ldcpend:\n";
            line("s_endpgm");
            s += ".Ldmain:\n";
            return;
        }
        const std::pair<const char*, int> names[] = {
            {"V_SRCOFF", V_SRCOFF}, {"V_OUTOFF", V_OUTOFF}, {"V_SCROFF", V_SCROFF}, {"V_LDS2", rv.lds2}};
        for (const auto& nm : names)
            for (size_t at = l.find(nm.first); at != std::string::npos; at = l.find(nm.first))
                l.replace(at, std::strlen(nm.first), "v" + std::to_string(nm.second));
        line(l.c_str());
    };
    const uint32_t LB = mp.n_lds_slots * 256u;  // LDS bytes per wave
    if (W == 1) {
        for (const char* p : pro_once) put(p);
    } else {
        // W waves per workgroup (one per SIMD of a CU) take W consecutive items, i.e. the W x 256-B
        // pieces of the same source rows (1 KiB at W = 4), which then reach the memory system close
        // together.  Wave w of the workgroup: LDS slots at w * LB (folded into V_SCROFF, the lane's
        // LDS / scratch voffset), scratch of global wave (wg * W + w), its base moved back by w * LB
        // because V_SCROFF carries that LDS offset too.
        for (const char* p : pro_once) {
            const std::string l(p);
            if (l.rfind("v_lshlrev_b32_e32 V_SCROFF", 0) == 0 || l.rfind("v_add_u32_e32 V_LDS2", 0) == 0 ||
                l.rfind("s_mul_i32 s32", 0) == 0 || l.rfind("s_mul_hi_u32 s33", 0) == 0)
                continue;
            if (l.rfind("s_add_u32 s32, s8, s32", 0) == 0) {
                put("v_lshrrev_b32_e32 v1, 6, v0");
                line("s_nop 4");  // VALU write -> v_readfirstlane of it (a missing wait state read v1 stale)
                line("v_readfirstlane_b32 s53, v1");
                put("v_and_b32_e32 v0, 63, v0");
                put("v_lshlrev_b32_e32 V_SCROFF, 2, v0");
                std::snprintf(buf, sizeof buf, "s_mul_i32 s41, s53, %u", LB); line(buf);
                put("v_add_u32_e32 V_SCROFF, s41, V_SCROFF");
                put("v_add_u32_e32 V_LDS2, 0x10000, V_SCROFF");
                std::snprintf(buf, sizeof buf, "s_mul_i32 s42, s2, %u", W); line(buf);
                line("s_add_u32 s42, s42, s53");
                line("s_mul_i32 s32, s42, s16");
                line("s_mul_hi_u32 s33, s42, s16");
                line("s_sub_u32 s32, s32, s41");
                line("s_subb_u32 s33, s33, 0");
            }
            put(p);
        }
    }
    // Scratch slot s sits at soffset 4096 * (s / 16) + offset (s % 16) * 256: soffset 0 or one of
    // SCR_BASES SGPRs s56.. loaded once, so a spill or reload carries no SALU; slots beyond them
    // (very large K) form their soffset with an s_mov.
    const uint32_t n_bases = scratch_bases(mp);
    for (uint32_t j = 0; j < n_bases; ++j) {
        std::snprintf(buf, sizeof buf, "s_mov_b32 s%u, %u", 56 + j, 4096u * (j + 1));
        line(buf);
    }
#ifdef RQHIP_EXPERIMENTS
    const bool dma4 = mp.dma4_quads > 0;  // (W = 1 only: compile_colprog_dma4)
    if (dma4) emit_dma4_prologue(mp, rv, s);
#endif
    // Code warm-up (W = 1): the program is ~180 KB of straight-line code that every wave starts at
    // once, and when the previous kernel was not a column program its lines are in neither L2 nor the
    // memory-side cache, so round 1's instruction fetches go to HBM one after another (12-15 us per
    // launch after a decode's apply, ~30 us after a large copy: profiles/r03_dense/r03pos).  Each wave
    // reads four 8 KiB strides of its own code (one dword per 128-B line; slice (wg / 8) % 32 within
    // its XCD), so the XCD's waves pull the whole program into their L2 in parallel, then wait once.
    // Bounds-checked buffer loads (num_records = code length): nothing beyond the code is read.
    // RQHIP_CODEPF=2 (experiments): the four loads land in a 256-byte LDS sink (buffer_load ... lds, no
    // VGPR written) and the wave starts its item without waiting for them.
    static const int code_pf = [] { const char* e = knob("RQHIP_CODEPF"); return e ? std::atoi(e) : 1; }();
    const bool pf_sink = code_pf == 2 && W == 1 && mp.lds_base + mp.n_lds_slots < 160;
    if (W == 1 && code_pf && !(diag & 4) && mp.n_vgpr >= 12) {  // v5, v6, v8..v11 are program registers
        line("s_getpc_b64 s[44:45]");
        s += ".Lcpf:\n";
        line(("s_sub_u32 s44, s44, .Lcpf-" + kname).c_str());
        line("s_subb_u32 s45, s45, 0");
        line("s_and_b32 s45, s45, 0xffff");
        line(("s_mov_b32 s46, .Lfunc_end-" + kname).c_str());
        line("s_mov_b32 s47, 0x20000");
        line("s_lshr_b32 s43, s2, 3");
        line("s_and_b32 s43, s43, 31");
        line("s_lshl_b32 s43, s43, 13");
        line("v_lshlrev_b32_e32 v5, 7, v0");
        line("v_add_u32_e32 v5, s43, v5");
        if (pf_sink) {
            std::snprintf(buf, sizeof buf, "s_mov_b32 m0, %u", (mp.lds_base + mp.n_lds_slots) * 256u);
            line(buf);
        }
        for (uint32_t k = 0; k < 4; ++k) {
            std::snprintf(buf, sizeof buf, "v_add_u32_e32 v6, 0x%x, v5", k * 32u * 8192u); line(buf);
            if (pf_sink) line("buffer_load_dword v6, s[44:47], 0 offen lds");
            else { std::snprintf(buf, sizeof buf, "buffer_load_dword v%u, v6, s[44:47], 0 offen", 8 + k); line(buf); }
        }
        if (!pf_sink) line("s_waitcnt vmcnt(0)");
    }
    // experiments: RQHIP_STAGGER=n delays the odd workgroups' start by n x 127 x 64 cycles (do the
    // first rounds' coinciding load bursts cost time?)
    static const uint32_t stagger = [] { const char* e = knob("RQHIP_STAGGER"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    if (stagger) {
        line("s_bitcmp1_b32 s2, 0");
        line("s_cbranch_scc0 .Lnostagger");
        for (uint32_t i = 0; i < stagger; ++i) line("s_sleep 127");
        s += ".Lnostagger:\n";
    }
    if (!mp.cip_reg.empty()) {
        // cross-item prefetch: the wave's first item's head loads (later items': the previous item's MI_PFX)
        line("s_lshr_b32 s21, s12, 2");
        if (!(diag & 4)) emit_cip_loads(mp, 0, (uint32_t)mp.cip_reg.size(), false, 0, s);
    }
    s += ".Lloop:\n";
    for (const char* p : pro_iter) {
        const std::string l(p);
        if (W > 1 && l.rfind("s_lshl_b32 s20, s39, 6", 0) == 0) {  // item = iteration * W + wave
            std::snprintf(buf, sizeof buf, "s_mul_i32 s39, s39, %u", W); line(buf);
            line("s_add_u32 s39, s39, s53");
        }
#ifdef RQHIP_EXPERIMENTS
        if (dma4 && l == "v_add_u32_e32 v1, s20, v0") emit_dma4_item_base(rv, s);
#endif
        if (W > 1 && l.rfind("v_lshrrev_b32_e32 v0, 2, V_SCROFF", 0) == 0) {  // lane id (V_SCROFF has w * LB)
            line("v_mbcnt_lo_u32_b32 v0, -1, 0");
            line("v_mbcnt_hi_u32_b32 v0, -1, v0");
            continue;
        }
        put(p);
    }
    emit_colprog_body(mp, W, s);
    // Loop end: no vmcnt drain.  The item's last memory operations are its output stores (every load
    // has been consumed), and the next item's program may run while they retire: vmcnt waits in it
    // then also cover these older stores (conservative, still exact), scratch slots are reused in
    // program order by the same wave (same-address order), and a store has read its data VGPR at
    // issue.  RQHIP_DRAIN=1 (experiments) restores the full drain.
    static const bool drain = [] { const char* e = knob("RQHIP_DRAIN"); return e && e[0] == '1'; }();
    line(drain ? "s_waitcnt vmcnt(0) lgkmcnt(0)" : "s_waitcnt lgkmcnt(0)");
    line("s_add_u32 s52, s52, s49");
    line("s_getpc_b64 s[54:55]");
    s += ".Lpc:\n";
    line("s_sub_u32 s54, s54, .Lpc-.Lloop");
    line("s_subb_u32 s55, s55, 0");
    line("s_setpc_b64 s[54:55]");
    s += ".Lend:\n\ts_endpgm\n";
    s += ".Lfunc_end:\n\t.size " + kname + ", .Lfunc_end-" + kname + "\n";
    s += "\t.p2alignl 6, 3212836864\n\t.fill 256, 4, 3212836864\n";
    s += "\t.section .rodata,\"a\",@progbits\n\t.p2align 6, 0x0\n\t.amdhsa_kernel " + kname + "\n";
    const std::string lds = std::to_string((mp.lds_base + mp.n_lds_slots) * 256u * W + (pf_sink ? 256u : 0u));
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
    s += "    .max_flat_workgroup_size: " + std::to_string(64 * W) + "\n    .name: " + kname + "\n    .private_segment_fixed_size: 0\n";
    s += "    .sgpr_count: " + std::to_string(ROW_WIN + 32) + "\n    .symbol: " + kname + ".kd\n    .vgpr_count: " + std::to_string(n_regs) +
         "\n    .wavefront_size: 64\n";
    s += "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n";
    return s;
}

// ------------------------------------------------------------------------------------------
bool emulate_colprog(const MProg& mp, const uint8_t* src, uint32_t T, uint8_t* out, std::string* err,
                     uint64_t src_bytes) {
    WaveEmu w(mp, src, T, out, err);
    w.src_bytes = src_bytes;
    return w.run();
}

}  // namespace rq
