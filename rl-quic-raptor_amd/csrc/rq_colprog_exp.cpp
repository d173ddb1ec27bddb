// rq_colprog_exp.cpp -- the two-wave (pair) split of a column program's IR (rq_colprog.hpp split_pair),
// the IR side of the pair programs measured and not shipped (profiles/r04_pair);
// compiled into the experiments library only (make EXPERIMENTS=1).
#ifndef RQHIP_EXPERIMENTS
#error "rq_colprog_exp.cpp belongs to the experiments build only"
#endif
#include <algorithm>
#include <cstring>

#include "rq_colprog.hpp"

namespace rq {

bool split_pair(const ColIR& ir, uint32_t bmask, uint32_t lag, uint32_t max_xfer, uint32_t ring, PairIR* out,
                std::string* err) {
    auto bad = [&](const char* m) {
        if (err) *err = m;
        return false;
    };
    const uint32_t n = (uint32_t)ir.nodes.size();
    if (!max_xfer || !ring) return bad("split_pair: empty transfer or ring");
    // side of every node: loads on A; a store beside the value it writes; the rest by grp
    std::vector<uint8_t> onB(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
        const IrNode& d = ir.nodes[i];
        if (d.k == IR_LOAD) onB[i] = 0;
        else if (d.k == IR_STORE) onB[i] = onB[d.a];
        else if (d.k > IR_STORE) return bad("split_pair: the IR is already split");
        else onB[i] = (bmask >> d.grp) & 1;
    }
    std::vector<uint8_t> cross(n, 0);  // A value used on B
    for (uint32_t i = 0; i < n; ++i) {
        const IrNode& d = ir.nodes[i];
        if (d.k == IR_STORE) continue;
        for (uint32_t x : {d.a, d.b, d.c}) {
            if (x == NOVAL) continue;
            if (onB[i] && !onB[x]) cross[x] = 1;
            if (!onB[i] && onB[x]) return bad("split_pair: a B value feeds an A node");
        }
    }
    *out = PairIR();
    out->lag = lag;
    out->ring = ring;
    ColIR& A = out->A;
    ColIR& Bv = out->B;
    A.p = Bv.p = ir.p;
    A.n_out = Bv.n_out = ir.n_out;
    std::vector<uint32_t> mapA(n, NOVAL), mapB(n, NOVAL);
    std::vector<uint8_t> sent(n, 0);
    std::vector<uint32_t> pending;       // A values for B, defined, not yet sent
    std::vector<uint32_t> sizes;         // per transfer
    uint32_t rp = 0;                     // position of the next value in the item's transfer sequence
    auto add = [](ColIR& c, uint8_t k, uint32_t a, uint32_t b, uint32_t cc, uint32_t imm, uint8_t grp) {
        IrNode d;
        d.k = k; d.a = a; d.b = b; d.c = cc; d.imm = imm; d.grp = grp;
        c.nodes.push_back(d);
        return (uint32_t)c.nodes.size() - 1;
    };
    std::vector<std::vector<uint32_t>> slots;  // ring slots of every transfer
    std::vector<std::vector<uint32_t>> xvals;  // the values of every transfer
    // B's stream is built as a sequence of its original nodes (>= 0) and transfers (-1 - t), then
    // every transfer is moved ahead of the B nodes that precede it back to the previous transfer: its
    // barrier and ring reads then run one transfer earlier in B's stream, so the reads' LDS latency
    // hides behind the previous transfer's work (B still reads transfer t only after its own barrier
    // t, so the ring rule below is unchanged).
    std::vector<int64_t> bseq;
    auto flush = [&]() {
        for (size_t s0 = 0; s0 < pending.size(); s0 += max_xfer) {
            const size_t s1 = std::min(pending.size(), s0 + max_xfer);
            const uint32_t t = (uint32_t)sizes.size();
            bseq.push_back(-1 - (int64_t)t);
            slots.emplace_back();
            xvals.emplace_back();
            for (size_t j = s0; j < s1; ++j) {
                const uint32_t v = pending[j];
                add(A, IR_SEND, mapA[v], NOVAL, NOVAL, rp, 0);
                sent[v] = 1;
                slots.back().push_back(rp);
                xvals.back().push_back(v);
                ++rp;
            }
            add(A, IR_BAR, NOVAL, NOVAL, NOVAL, t, 0);  // A: the barrier closes the transfer
            sizes.push_back((uint32_t)(s1 - s0));
        }
        pending.clear();
    };
    for (uint32_t i = 0; i < n; ++i) {
        const IrNode& d = ir.nodes[i];
        if (onB[i]) {
            bool need = false;
            for (uint32_t x : {d.a, d.b, d.c})
                if (x != NOVAL && cross[x] && !sent[x]) need = true;
            if (need) flush();
            bseq.push_back(i);
        } else {
            uint32_t o[3] = {NOVAL, NOVAL, NOVAL};
            const uint32_t in[3] = {d.a, d.b, d.c};
            for (int q = 0; q < 3; ++q)
                if (in[q] != NOVAL) {
                    o[q] = mapA[in[q]];
                    if (o[q] == NOVAL) return bad("split_pair: A operand missing");
                }
            mapA[i] = add(A, d.k, o[0], o[1], o[2], d.imm, d.grp);
            if (cross[i]) pending.push_back(i);
        }
    }
    {  // [pre, X0, n0, X1, n1, X2, ...] -> [pre, X0, X1, n0, X2, n1, ...]: X(t+1) ahead of n(t)
        std::vector<int64_t> h, run;
        h.reserve(bseq.size());
        bool seen = false;
        for (int64_t x : bseq) {
            if (x >= 0) {
                (seen ? run : h).push_back(x);
                continue;
            }
            h.push_back(x);  // this transfer, then the nodes that followed the previous one
            h.insert(h.end(), run.begin(), run.end());
            run.clear();
            seen = true;
        }
        h.insert(h.end(), run.begin(), run.end());
        bseq.swap(h);
    }
    for (int64_t x : bseq) {
        if (x < 0) {
            const uint32_t t = (uint32_t)(-1 - x);
            add(Bv, IR_BAR, NOVAL, NOVAL, NOVAL, t, 0);  // B: the barrier opens the transfer
            for (size_t j = 0; j < xvals[t].size(); ++j) {
                const uint32_t v = xvals[t][j];
                mapB[v] = add(Bv, IR_RECV, NOVAL, NOVAL, NOVAL, slots[t][j], ir.nodes[v].grp);
            }
            continue;
        }
        const IrNode& d = ir.nodes[(uint32_t)x];
        uint32_t o[3] = {NOVAL, NOVAL, NOVAL};
        const uint32_t in[3] = {d.a, d.b, d.c};
        for (int q = 0; q < 3; ++q)
            if (in[q] != NOVAL) {
                o[q] = mapB[in[q]];
                if (o[q] == NOVAL) return bad("split_pair: B operand missing");
            }
        mapB[(uint32_t)x] = add(Bv, d.k, o[0], o[1], o[2], d.imm, d.grp);
    }
    if (!pending.empty()) return bad("split_pair: A values never used by B");
    out->n_xfer = (uint32_t)sizes.size();
    for (uint32_t x : sizes) out->n_cross += x;
    // Ring slots.  While A writes transfer k + 1, B may still read transfers k - lag .. k (written, not
    // yet consumed), so every lag + 2 consecutive transfers must use pairwise distinct slots -- across
    // the item boundary too, where every item restarts the same code.  The item's values take
    // consecutive positions (transfer order) and slot = position % R; positions within lag + 2
    // consecutive transfers are then distinct mod R as long as they span at most R.  For the sequence
    // to continue across items the item's span must be a multiple of R, so a gap of
    // (R - n % R) % R positions goes before the transfer g where the windows containing it are
    // smallest.  The smallest R <= ring with a feasible gap is taken.
    const uint32_t nt = out->n_xfer, ncross = out->n_cross, wl = lag + 2;
    std::vector<uint32_t> win(nt, 0);  // window sum starting at transfer j (cyclic)
    for (uint32_t j = 0; j < nt; ++j)
        for (uint32_t q = 0; q < wl; ++q) win[j] += sizes[(j + q) % nt];
    for (uint32_t j = 0; j < nt; ++j) out->max_window = std::max(out->max_window, win[j]);
    if (nt && wl > nt) return bad("split_pair: too few transfers for the lag");
    uint32_t R = 0, gap = 0, gat = 0;
    for (uint32_t r = std::max<uint32_t>(out->max_window, 1); nt && r <= ring && !R; ++r) {
        const uint32_t gp = (r - ncross % r) % r;
        if (!gp) { R = r; break; }
        for (uint32_t g = 0; g < nt && !R; ++g) {  // windows holding the boundary g-1 | g start at g-lag-1 .. g-1
            uint32_t m = 0;
            for (uint32_t q = 1; q < wl; ++q) m = std::max(m, win[(g + nt - q) % nt]);
            if (m + gp <= r) { R = r; gap = gp; gat = g; }
        }
    }
    if (nt && !R) return bad("split_pair: ring too small for the lag");
    out->ring = nt ? R : 1;
    if (nt) {
        std::vector<uint32_t> pos_of(ncross, 0);  // item position of value index p (transfer order)
        uint32_t p = 0;
        for (uint32_t t = 0; t < nt; ++t)
            for (uint32_t j = 0; j < sizes[t]; ++j, ++p) pos_of[p] = p + (t >= gat && gap ? gap : 0);
        for (IrNode& d : A.nodes)
            if (d.k == IR_SEND) d.imm = pos_of[d.imm] % R;
        for (IrNode& d : Bv.nodes)
            if (d.k == IR_RECV) d.imm = pos_of[d.imm] % R;
    }
    for (ColIR* c : {&A, &Bv}) {
        for (const IrNode& d : c->nodes) {
            switch (d.k) {
                case IR_LOAD: ++c->st.load; break;
                case IR_ZERO: ++c->st.zero; break;
                case IR_XOR2: ++c->st.xor2; break;
                case IR_XOR3: ++c->st.xor3; break;
                case IR_XT: ++c->st.xt; break;
                case IR_XTX: ++c->st.xtx; break;
                case IR_STORE: ++c->st.store; break;
                default: break;
            }
        }
    }
    return true;
}

}  // namespace rq
