// rq_colprog.cpp -- builds the column program IR (see rq_colprog.hpp).
//
// Constraint system (RQ/solver.go:25-65, RQ/params.go:116-160):
//   S LDPC rows (circulant B part, identity on B..B+S-1, two PI columns), rhs 0
//   K' LT rows (ISI 0..K'-1), rhs = zero-padded source symbol
//   H HDPC rows [MT*Gamma | I_H], rhs 0
// Elimination: peeling with inactivation over the sparse GF(2) rows (cf. RQ/inactivate.go:25-170),
// then a dense solve on the u inactive columns (replaces RQ/discmath/gauss.go:7-45).
#include "rq_colprog.hpp"

#include <algorithm>
#include <array>
#include <cstring>
#include <functional>
#include <map>
#include <queue>
#include <set>

namespace rq {

namespace {

using Bits = std::vector<uint64_t>;

struct Elim {
    uint32_t L = 0, S = 0, H = 0, Kp = 0, W = 0, P = 0, KS = 0, NR = 0;
    std::vector<std::vector<uint32_t>> rows;    // GF(2) rows: LDPC 0..S-1, LT S..S+K'-1
    std::vector<uint8_t> cstate;                // 1 pivoted, 2 inactive
    std::vector<uint32_t> piv_row, piv_col;     // peeling order
    std::vector<int32_t> col_order;             // column -> pivot index or -1
    std::vector<std::vector<uint32_t>> deps;    // pivot -> earlier pivots in its row
    std::vector<uint32_t> ucols;                // inactive columns
    std::vector<int32_t> uidx;                  // column -> index in ucols or -1
    std::vector<uint32_t> rem;                  // remaining (unpeeled) GF(2) rows
    uint32_t u = 0, nw = 0;
    std::vector<uint64_t> Wb;                   // npiv x nw: C[c_k] = y_k ^ W_k * C_U
    const uint64_t* wrow(uint32_t k) const { return &Wb[(size_t)k * nw]; }
    // HDPC: G[h][j] = sum_{i>=j} MT[h][i] alpha^(i-j); ma/mb = the two ones of MT column j
    std::vector<uint8_t> G, ma, mb;
    // dense solve
    uint32_t n2 = 0;
    std::vector<int32_t> pc_of_row;             // rem row i -> U index of its pivot column
    std::vector<uint32_t> fcols;                // H free U indices
    std::vector<Bits> E2, R;                    // n2 x n2, n2 x H (GF(2))
    std::vector<uint8_t> Zi;                    // H x H GF(256)
    std::vector<uint8_t> Q;                     // H x n2 GF(256): C_F = Zi*bh ^ Q*b2
};

inline bool bit(const uint64_t* b, uint32_t i) { return (b[i >> 6] >> (i & 63)) & 1; }
inline void flip(uint64_t* b, uint32_t i) { b[i >> 6] ^= 1ull << (i & 63); }

bool eliminate(const Params& p, Elim* e, std::string* err) {
    const GF& g = gf();
    e->L = p.L; e->S = p.S; e->H = p.H; e->Kp = p.Kp; e->W = p.W; e->P = p.P;
    const uint32_t L = p.L, S = p.S, H = p.H, W = p.W, P = p.P, KS = p.Kp + p.S, NR = p.S + p.Kp;
    e->KS = KS; e->NR = NR;
    auto& rows = e->rows;
    rows.assign(NR, {});
    for (uint32_t i = 0; i < p.B; ++i) {
        const uint32_t a = 1 + i / S;
        uint32_t r = i % S;
        rows[r].push_back(i);
        r = (r + a) % S; rows[r].push_back(i);
        r = (r + a) % S; rows[r].push_back(i);
    }
    for (uint32_t i = 0; i < S; ++i) {
        rows[i].push_back(p.B + i);
        rows[i].push_back(W + (i % P));
        rows[i].push_back(W + ((i + 1) % P));
    }
    uint32_t cols[64];
    for (uint32_t i = 0; i < p.Kp; ++i) {
        const int n = lt_cols(p, i, cols);
        rows[S + i].assign(cols, cols + n);
    }
    for (auto& r : rows) {  // Set(...,1) semantics: duplicates are idempotent
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
    }
    std::vector<std::vector<uint32_t>> col_rows(L);
    for (uint32_t r = 0; r < NR; ++r)
        for (uint32_t c : rows[r]) col_rows[c].push_back(r);

    // ---- peeling with inactivation: take a row of minimum active degree (FIFO per degree);
    // its pivot is the active column with the most unfinished rows, the others go inactive.
    enum : uint8_t { ACTIVE = 0, PIVOTED = 1, INACTIVE = 2 };
    auto& cstate = e->cstate;
    cstate.assign(L, ACTIVE);
    for (uint32_t c = W; c < L; ++c) cstate[c] = INACTIVE;  // PI columns start inactive
    std::vector<uint32_t> cnt(NR, 0);
    std::vector<uint8_t> rdone(NR, 0);
    for (uint32_t r = 0; r < NR; ++r)
        for (uint32_t c : rows[r]) cnt[r] += (cstate[c] == ACTIVE);
    std::vector<uint32_t> live_deg(L, 0);
    for (uint32_t c = 0; c < L; ++c) live_deg[c] = (uint32_t)col_rows[c].size();
    std::vector<std::vector<uint32_t>> bucket(64);
    std::vector<size_t> bhead(64, 0);
    for (uint32_t r = 0; r < NR; ++r) bucket[std::min<uint32_t>(cnt[r], 63)].push_back(r);
    e->ucols.clear();
    for (uint32_t c = W; c < L; ++c) e->ucols.push_back(c);
    e->col_order.assign(L, -1);
    auto drop_col = [&](uint32_t c, uint32_t except_row) {
        for (uint32_t r : col_rows[c]) {
            if (rdone[r] || r == except_row) continue;
            --cnt[r];
            bucket[std::min<uint32_t>(cnt[r], 63)].push_back(r);
        }
    };
    // degree-1 rows by smallest column (peel_mode 1): peeling then runs roughly in column order
    static const int peel_mode = [] { const char* m = knob("RQHIP_PEEL"); return m ? std::atoi(m) : 0; }();
    std::priority_queue<std::pair<uint32_t, uint32_t>, std::vector<std::pair<uint32_t, uint32_t>>,
                        std::greater<std::pair<uint32_t, uint32_t>>> deg1;
    auto active_col = [&](uint32_t r) -> uint32_t {
        for (uint32_t c : rows[r]) if (cstate[c] == ACTIVE) return c;
        return UINT32_MAX;
    };
    for (;;) {
        int32_t r = -1;
        if (peel_mode) {
            auto& bk = bucket[1];
            while (bhead[1] < bk.size()) {  // move new degree-1 rows into the column / row ordered heap
                const uint32_t x = bk[bhead[1]++];
                if (!rdone[x] && cnt[x] == 1) deg1.push({peel_mode == 1 ? active_col(x) : x, x});
            }
            while (!deg1.empty() && r < 0) {
                const auto top = deg1.top();
                deg1.pop();
                if (!rdone[top.second] && cnt[top.second] == 1 &&
                    (peel_mode != 1 || cstate[top.first] == ACTIVE))
                    r = (int32_t)top.second;
            }
        }
        for (uint32_t b = 1; b < 64 && r < 0; ++b) {
            auto& bk = bucket[b];
            while (bhead[b] < bk.size()) {
                const uint32_t x = bk[bhead[b]++];
                if (!rdone[x] && std::min<uint32_t>(cnt[x], 63) == b) { r = (int32_t)x; break; }
            }
        }
        if (r < 0) break;
        uint32_t best = UINT32_MAX, best_deg = 0;
        for (uint32_t c : rows[r])
            if (cstate[c] == ACTIVE && (best == UINT32_MAX || live_deg[c] > best_deg)) { best = c; best_deg = live_deg[c]; }
        for (uint32_t c : rows[r]) {
            if (cstate[c] != ACTIVE || c == best) continue;
            cstate[c] = INACTIVE;
            e->ucols.push_back(c);
            drop_col(c, UINT32_MAX);
        }
        cstate[best] = PIVOTED;
        e->col_order[best] = (int32_t)e->piv_col.size();
        e->piv_row.push_back((uint32_t)r);
        e->piv_col.push_back(best);
        rdone[r] = 1;
        drop_col(best, (uint32_t)r);
        for (uint32_t c : rows[r]) --live_deg[c];
    }
    for (uint32_t c = 0; c < L; ++c)
        if (cstate[c] == ACTIVE) { cstate[c] = INACTIVE; e->ucols.push_back(c); }
    const uint32_t u = e->u = (uint32_t)e->ucols.size();
    const uint32_t npiv = (uint32_t)e->piv_col.size();
    for (uint32_t r = 0; r < NR; ++r)
        if (!rdone[r]) e->rem.push_back(r);
    const uint32_t n2 = e->n2 = (uint32_t)e->rem.size();
    if (n2 + H != u) { if (err) *err = "colprog: remaining rows != inactive columns"; return false; }
    e->uidx.assign(L, -1);
    for (uint32_t j = 0; j < u; ++j) e->uidx[e->ucols[j]] = (int32_t)j;

    // ---- forward-substitution structure and W (C[c_k] = y_k ^ W_k C_U)
    const uint32_t nw = e->nw = (u + 63) / 64;
    e->Wb.assign((size_t)npiv * nw, 0);
    e->deps.assign(npiv, {});
    for (uint32_t k = 0; k < npiv; ++k) {
        uint64_t* wk = &e->Wb[(size_t)k * nw];
        for (uint32_t c : rows[e->piv_row[k]]) {
            if (c == e->piv_col[k]) continue;
            if (cstate[c] == PIVOTED) {
                const uint32_t j = (uint32_t)e->col_order[c];
                e->deps[k].push_back(j);
                const uint64_t* wd = e->wrow(j);
                for (uint32_t x = 0; x < nw; ++x) wk[x] ^= wd[x];
            } else {
                flip(wk, (uint32_t)e->uidx[c]);
            }
        }
    }

    // ---- HDPC coefficients
    e->ma.assign(KS, 0); e->mb.assign(KS, 0);
    for (uint32_t j = 0; j + 1 < KS; ++j) {
        const uint32_t a = rand_(j + 1, 6, H);
        e->ma[j] = (uint8_t)a;
        e->mb[j] = (uint8_t)((a + rand_(j + 1, 7, H - 1) + 1) % H);
    }
    auto MT = [&](uint32_t h, uint32_t j) -> uint8_t {
        if (j == KS - 1) return g.pow_alpha(h);
        return (e->ma[j] == h || e->mb[j] == h) ? 1 : 0;
    };
    e->G.assign((size_t)H * KS, 0);
    for (uint32_t h = 0; h < H; ++h) {
        uint8_t acc = 0;
        for (int64_t j = (int64_t)KS - 1; j >= 0; --j) {
            acc = (uint8_t)(g.mul(acc, 2) ^ MT(h, (uint32_t)j));
            e->G[(size_t)h * KS + j] = acc;
        }
    }

    // ---- dense matrix Mu (u x u): rem rows (GF(2)) then HDPC rows (GF(256))
    std::vector<uint8_t> Mu((size_t)u * u, 0);
    for (uint32_t i = 0; i < n2; ++i) {
        std::vector<uint64_t> acc(nw, 0);
        for (uint32_t c : rows[e->rem[i]]) {
            if (cstate[c] == PIVOTED) {
                const uint64_t* wd = e->wrow((uint32_t)e->col_order[c]);
                for (uint32_t x = 0; x < nw; ++x) acc[x] ^= wd[x];
            } else {
                flip(acc.data(), (uint32_t)e->uidx[c]);
            }
        }
        for (uint32_t j = 0; j < u; ++j) Mu[(size_t)i * u + j] = bit(acc.data(), j);
    }
    for (uint32_t h = 0; h < H; ++h) {
        uint8_t* mrow = &Mu[(size_t)(n2 + h) * u];
        for (uint32_t j = 0; j < u; ++j) {
            const uint32_t c = e->ucols[j];
            uint8_t v = (c < KS) ? e->G[(size_t)h * KS + c] : 0;
            if (c == KS + h) v ^= 1;
            mrow[j] = v;
        }
        for (uint32_t k = 0; k < npiv; ++k) {
            const uint8_t gc = e->G[(size_t)h * KS + e->piv_col[k]];
            if (!gc) continue;
            const uint64_t* wk = e->wrow(k);
            for (uint32_t j = 0; j < u; ++j)
                if (bit(wk, j)) mrow[j] ^= gc;
        }
    }
    auto mu = [&](uint32_t r, uint32_t c) -> uint8_t { return Mu[(size_t)r * u + c]; };

    // ---- GF(2) Gauss-Jordan on [Mu2 | I]: pivot columns Pc, E2 = Mu2[:,Pc]^-1, R = E2 Mu2[:,Fc]
    const uint32_t bw = (u + n2 + 63) / 64;
    std::vector<uint64_t> aug((size_t)n2 * bw, 0);
    for (uint32_t i = 0; i < n2; ++i) {
        uint64_t* ar = &aug[(size_t)i * bw];
        for (uint32_t j = 0; j < u; ++j)
            if (mu(i, j)) flip(ar, j);
        flip(ar, u + i);
    }
    e->pc_of_row.assign(n2, -1);
    std::vector<uint8_t> is_pc(u, 0);
    for (uint32_t i = 0; i < n2; ++i) {
        uint64_t* ai = &aug[(size_t)i * bw];
        int32_t jc = -1;
        for (uint32_t j = 0; j < u; ++j)
            if (!is_pc[j] && bit(ai, j)) { jc = (int32_t)j; break; }
        if (jc < 0) { if (err) *err = "colprog: singular GF(2) block"; return false; }
        e->pc_of_row[i] = jc;
        is_pc[jc] = 1;
        for (uint32_t q = 0; q < n2; ++q) {
            uint64_t* aq = &aug[(size_t)q * bw];
            if (q != i && bit(aq, (uint32_t)jc))
                for (uint32_t x = 0; x < bw; ++x) aq[x] ^= ai[x];
        }
    }
    for (uint32_t j = 0; j < u; ++j)
        if (!is_pc[j]) e->fcols.push_back(j);
    if (e->fcols.size() != H) { if (err) *err = "colprog: free column count != H"; return false; }
    const uint32_t nb2 = (n2 + 63) / 64, nbh = (H + 63) / 64;
    e->E2.assign(n2, Bits(nb2, 0));
    e->R.assign(n2, Bits(nbh, 0));
    for (uint32_t i = 0; i < n2; ++i) {
        const uint64_t* ai = &aug[(size_t)i * bw];
        for (uint32_t m = 0; m < n2; ++m)
            if (bit(ai, u + m)) flip(e->E2[i].data(), m);
        for (uint32_t f = 0; f < H; ++f)
            if (bit(ai, e->fcols[f])) flip(e->R[i].data(), f);
    }
    // Z = Mh[:,Fc] ^ Mh[:,Pc] R, Zi = Z^-1 (GF(256) Gauss-Jordan)
    std::vector<uint8_t> Z((size_t)H * H, 0), Zi((size_t)H * H, 0);
    for (uint32_t h = 0; h < H; ++h)
        for (uint32_t f = 0; f < H; ++f) {
            uint8_t z = mu(n2 + h, e->fcols[f]);
            for (uint32_t i = 0; i < n2; ++i)
                if (bit(e->R[i].data(), f)) z ^= mu(n2 + h, (uint32_t)e->pc_of_row[i]);
            Z[(size_t)h * H + f] = z;
        }
    for (uint32_t i = 0; i < H; ++i) Zi[(size_t)i * H + i] = 1;
    for (uint32_t c = 0; c < H; ++c) {
        uint32_t pr = H;
        for (uint32_t r = c; r < H; ++r)
            if (Z[(size_t)r * H + c]) { pr = r; break; }
        if (pr == H) { if (err) *err = "colprog: singular HDPC block"; return false; }
        for (uint32_t x = 0; x < H; ++x) {
            std::swap(Z[(size_t)pr * H + x], Z[(size_t)c * H + x]);
            std::swap(Zi[(size_t)pr * H + x], Zi[(size_t)c * H + x]);
        }
        const uint8_t inv = g.inv(Z[(size_t)c * H + c]);
        for (uint32_t x = 0; x < H; ++x) {
            Z[(size_t)c * H + x] = g.mul(Z[(size_t)c * H + x], inv);
            Zi[(size_t)c * H + x] = g.mul(Zi[(size_t)c * H + x], inv);
        }
        for (uint32_t r = 0; r < H; ++r) {
            const uint8_t f = Z[(size_t)r * H + c];
            if (r == c || !f) continue;
            for (uint32_t x = 0; x < H; ++x) {
                Z[(size_t)r * H + x] ^= g.mul(f, Z[(size_t)c * H + x]);
                Zi[(size_t)r * H + x] ^= g.mul(f, Zi[(size_t)c * H + x]);
            }
        }
    }
    e->Zi = Zi;
    // Q = Zi * Mh[:,Pc] * E2  (H x n2)
    std::vector<uint8_t> MP((size_t)H * n2, 0);  // Mh[:,Pc] E2
    for (uint32_t h = 0; h < H; ++h)
        for (uint32_t m = 0; m < n2; ++m) {
            uint8_t v = 0;
            for (uint32_t i = 0; i < n2; ++i)
                if (bit(e->E2[i].data(), m)) v ^= mu(n2 + h, (uint32_t)e->pc_of_row[i]);
            MP[(size_t)h * n2 + m] = v;
        }
    e->Q.assign((size_t)H * n2, 0);
    for (uint32_t f = 0; f < H; ++f)
        for (uint32_t m = 0; m < n2; ++m) {
            uint8_t v = 0;
            for (uint32_t h = 0; h < H; ++h) v ^= g.mul(Zi[(size_t)f * H + h], MP[(size_t)h * n2 + m]);
            e->Q[(size_t)f * n2 + m] = v;
        }
    return true;
}

// ---- IR construction helpers ----
struct Builder {
    ColIR* ir;
    uint8_t grp = 0;  // tag of the nodes added (IrNode::grp)
    uint32_t add(uint8_t k, uint32_t a = NOVAL, uint32_t b = NOVAL, uint32_t c = NOVAL, uint32_t imm = 0) {
        IrNode n;
        n.k = k; n.a = a; n.b = b; n.c = c; n.imm = imm; n.grp = grp;
        ir->nodes.push_back(n);
        return (uint32_t)ir->nodes.size() - 1;
    }
    // XOR of a term list (NOVAL = zero terms are skipped); NOVAL if every term is zero.
    uint32_t xsum(const std::vector<uint32_t>& terms) {
        uint32_t acc = NOVAL;
        std::vector<uint32_t> t;
        for (uint32_t v : terms)
            if (v != NOVAL) t.push_back(v);
        size_t i = 0;
        if (t.empty()) return NOVAL;
        if (t.size() == 1) return t[0];
        if (t.size() % 2 == 0) { acc = add(IR_XOR2, t[0], t[1]); i = 2; }
        else { acc = t[0]; i = 1; }
        for (; i < t.size(); i += 2) acc = add(IR_XOR3, acc, t[i], t[i + 1]);
        return acc;
    }
    uint32_t xt(uint32_t a, uint32_t b = NOVAL) {  // alpha*a ^ b
        if (a == NOVAL) return b;
        return b == NOVAL ? add(IR_XT, a) : add(IR_XTX, a, b);
    }
};

// Accumulator: pushes are XORed in pairs (one XOR3 per two pushes).
struct Acc {
    uint32_t val = NOVAL, pend = NOVAL;
    // may_pend = false: the next push is far off, so XOR now rather than keep v alive as the pending
    // operand of a later XOR3
    void push(Builder& B, uint32_t v, bool may_pend = true) {
        if (v == NOVAL) return;
        if (val == NOVAL) { val = v; return; }
        if (!may_pend && pend == NOVAL) { val = B.add(IR_XOR2, val, v); return; }
        if (pend == NOVAL) { pend = v; return; }
        val = B.add(IR_XOR3, val, pend, v);
        pend = NOVAL;
    }
    uint32_t get(Builder& B) {
        if (pend != NOVAL) { val = B.add(IR_XOR2, val, pend); pend = NOVAL; }
        return val;
    }
    // the accumulated terms as operands of a larger sum (no XOR of their own): val, then pend
    void append_to(std::vector<uint32_t>& t) {
        if (val != NOVAL) t.push_back(val);
        if (pend != NOVAL) t.push_back(pend);
        val = pend = NOVAL;
    }
};

// Output specification: the set of C columns XORed (XOR semantics) or a source row.
struct OutDesc {
    bool source = false;
    uint32_t row = 0;
    std::vector<uint32_t> cols;
};

// passes = 0: demand-driven order (each y_k emitted when the single column scan first needs it).
// passes = P >= 1: y_k in peeling order, each pushed at once into the rows that depend on it (their
// accumulators), into the remaining-row sums and into the output sums; the HDPC Horner scan runs P
// times, pass q over the y values produced since pass q-1 (the others count as zero: the scan is
// linear, so the P chains' pushes and end values add up to the single scan's).  A y value then lives
// only until its pass instead of until its column comes up in one global scan, which bounds the live
// set by about npiv / P plus the open accumulators, at 2 ops per column per extra pass.
// Group size of the four-Russians dense part and outputs (0: the direct sums of rounds 1-2;
// RQHIP_DENSE_GROUP in experiments builds).
static uint32_t dense_group() {
    static const uint32_t g = [] {
        const char* m = knob("RQHIP_DENSE_GROUP");
        return m ? (uint32_t)std::min(6, std::max(0, std::atoi(m))) : 4u;
    }();
    return g;
}

static bool interleave_passes() {
    static const bool on = [] { const char* m = knob("RQHIP_WEAVE"); return m && m[0] == '1'; }();
    return on;
}

bool build(const Params& p, const std::vector<OutDesc>& outs, uint32_t passes, ColIR* ir, std::string* err) {
    Elim e;
    if (!eliminate(p, &e, err)) return false;
    *ir = ColIR();
    ir->p = p;
    ir->n_out = (uint32_t)outs.size();
    Builder B{ir};
    const uint32_t npiv = (uint32_t)e.piv_col.size(), u = e.u, n2 = e.n2, H = e.H, S = e.S, KS = e.KS;
    const uint32_t K = p.K;
    auto D = [&](uint32_t row) -> uint32_t {  // rhs of GF(2) row `row` (LT rows: source ISI row - S)
        if (row < S) return NOVAL;
        const uint32_t isi = row - S;
        return isi < K ? B.add(IR_LOAD, NOVAL, NOVAL, NOVAL, isi) : NOVAL;
    };
    // ---- forward pass, demand-driven: y_k = D(row_k) ^ XOR of its deps is emitted just before the
    // column scan first needs it (deps first, iterative DFS), so few y values wait in registers.
    ir->phase_start[0] = 0;
    std::vector<uint32_t> y(npiv, NOVAL);
    std::vector<uint8_t> ystate(npiv, 0);  // 0 todo, 1 deps pushed, 2 done
    std::vector<uint32_t> stk;
    auto getY = [&](uint32_t k0) -> uint32_t {
        if (ystate[k0] == 2) return y[k0];
        stk.push_back(k0);
        while (!stk.empty()) {
            const uint32_t k = stk.back();
            if (ystate[k] == 2) { stk.pop_back(); continue; }
            if (ystate[k] == 0) {
                ystate[k] = 1;
                for (auto it = e.deps[k].rbegin(); it != e.deps[k].rend(); ++it)
                    if (ystate[*it] != 2) stk.push_back(*it);
                continue;
            }
            std::vector<uint32_t> t;
            t.push_back(D(e.piv_row[k]));
            for (uint32_t j : e.deps[k]) t.push_back(y[j]);
            y[k] = B.xsum(t);
            ystate[k] = 2;
            stk.pop_back();
        }
        return y[k0];
    };
    // ---- per output: y-part (pivoted columns) and W-hat (U part) -> V1 (n2 bits), V2 (H bits)
    const uint32_t no = (uint32_t)outs.size();
    std::vector<std::vector<uint32_t>> col_outs(e.L);  // column -> outputs using it (odd multiplicity)
    std::vector<Bits> V1(no, Bits((n2 + 63) / 64, 0)), V2(no, Bits((H + 63) / 64, 0));
    for (uint32_t o = 0; o < no; ++o) {
        if (outs[o].source) continue;
        std::vector<uint32_t> cs = outs[o].cols;
        std::sort(cs.begin(), cs.end());
        std::vector<uint32_t> kept;
        for (size_t i = 0; i < cs.size();) {
            size_t j = i;
            while (j < cs.size() && cs[j] == cs[i]) ++j;
            if ((j - i) & 1) kept.push_back(cs[i]);
            i = j;
        }
        Bits what(e.nw, 0);
        for (uint32_t c : kept) {
            if (e.cstate[c] == 1) {
                col_outs[c].push_back(o);
                const uint64_t* wk = e.wrow((uint32_t)e.col_order[c]);
                for (uint32_t x = 0; x < e.nw; ++x) what[x] ^= wk[x];
            } else {
                flip(what.data(), (uint32_t)e.uidx[c]);
            }
        }
        for (uint32_t i = 0; i < n2; ++i) {
            if (!bit(what.data(), (uint32_t)e.pc_of_row[i])) continue;
            for (uint32_t x = 0; x < V1[o].size(); ++x) V1[o][x] ^= e.E2[i][x];
            for (uint32_t x = 0; x < V2[o].size(); ++x) V2[o][x] ^= e.R[i][x];
        }
        for (uint32_t f = 0; f < H; ++f)
            if (bit(what.data(), e.fcols[f])) flip(V2[o].data(), f);
    }
    // rem rows per column
    std::vector<std::vector<uint32_t>> col_rem(e.L);
    for (uint32_t i = 0; i < n2; ++i)
        for (uint32_t c : e.rows[e.rem[i]])
            if (e.cstate[c] == 1) col_rem[c].push_back(i);

    // ---- column scan: Horner for the HDPC sums and the pushes into b2 / output sums
    ir->phase_start[1] = (uint32_t)ir->nodes.size();
    std::vector<Acc> b2acc(n2), oacc(no), part(H);
    for (uint32_t i = 0; i < n2; ++i) b2acc[i].push(B, D(e.rem[i]));
    uint32_t t = NOVAL;
    std::vector<uint32_t> bh_direct;  // SCHED_4R: bh computed without a Horner scan
    if (passes & SCHED_4R) {
        // Peeling-order production, push-mode dependencies; no Horner scan.  bh_h = sum_j G[h][j] y_j
        // (G = MT * Gamma, RQ/params.go:116-133) is accumulated bit by bit: S[h][b] = XOR of the y_j
        // with bit b of G[h][j] set, bh_h = sum_b alpha^b S[h][b] (7 xtimes per h at the end).  Every
        // 8 consecutively produced y values form two groups of 4 whose subset XORs (11 per group) are
        // built once; each of the 8H bit rows then takes one XOR3 (its group-A subset, its group-B
        // subset).  ~12.75 VALU per y and no y waits for a scan: the live set drops by the scan's
        // buffer (hundreds of values) for the cost of ~2 Horner passes.
        std::vector<std::vector<uint32_t>> dependents(npiv);
        for (uint32_t k = 0; k < npiv; ++k)
            for (uint32_t j : e.deps[k]) dependents[j].push_back(k);
        std::vector<Acc> yacc(npiv);
        // next event (push or consumption) of every accumulator after production k, so a push whose
        // accumulator is not touched again within `pend_win` productions XORs at once
        const uint32_t pend_win = (passes & 0xFFFFu) ? (passes & 0xFFFFu) : 0xFFFFu;
        const uint32_t n_acc = npiv + n2 + no;
        std::vector<std::vector<uint32_t>> ev(n_acc);
        for (uint32_t k = 0; k < npiv; ++k) {
            for (uint32_t d : dependents[k]) ev[d].push_back(k);
            const uint32_t c = e.piv_col[k];
            for (uint32_t i : col_rem[c]) ev[npiv + i].push_back(k);
            for (uint32_t o : col_outs[c]) ev[npiv + n2 + o].push_back(k);
        }
        for (uint32_t d = 0; d < npiv; ++d) ev[d].push_back(d);
        std::vector<uint32_t> evp(n_acc, 0);
        auto may_pend = [&](uint32_t a, uint32_t k) {
            auto& v = ev[a];
            uint32_t& q = evp[a];
            while (q < v.size() && v[q] <= k) ++q;
            return q < v.size() && v[q] - k <= pend_win;
        };
        // bit-row accumulators: two subset operands per chunk make one XOR3; a row that gets one
        // operand keeps it pending for the next chunk's (Acc) instead of an XOR2 now
        std::vector<Acc> S8((size_t)H * 8);
        std::vector<uint32_t> chunk;  // pivot indices of produced y (column < KS)
        // SCHED_HA(n): the first n HDPC rows are tagged 4 (pair programs: wave A accumulates them, with
        // its own copies of the subset sums, so the two waves' VALU work balances), the others 1
        const uint32_t hA = std::min<uint32_t>(H, (passes >> SCHED_HA_SHIFT) & 0xFFu);
        auto flush = [&]() {
            if (chunk.empty()) return;
            const size_t ng = (chunk.size() + 3) / 4;
            std::vector<std::array<uint32_t, 16>> sub_all[2];
            sub_all[0].resize(ng);
            sub_all[1].resize(ng);
            for (size_t g = 0; g < ng; ++g) { sub_all[0][g].fill(NOVAL); sub_all[1][g].fill(NOVAL); }
            std::vector<std::array<uint32_t, 16>>* subp = &sub_all[0];
            auto subset = [&](size_t g, uint32_t m) -> uint32_t {  // XOR of group g's members in mask m
                auto& sub = *subp;
                auto& s = sub[g];
                if (s[m] != NOVAL) return s[m];
                std::vector<uint32_t> terms;
                for (uint32_t q = 0; q < 4; ++q)
                    if (m & (1u << q)) terms.push_back(y[chunk[g * 4 + q]]);
                if (terms.size() <= 1) { s[m] = terms.empty() ? NOVAL : terms[0]; return s[m]; }
                if (terms.size() == 4) {  // (pair) ^ y2 ^ y3 with the pair built once
                    const uint32_t m01 = m & 3u;
                    std::vector<uint32_t> v{sub[g][m01] != NOVAL ? sub[g][m01] : B.xsum({terms[0], terms[1]}), terms[2], terms[3]};
                    sub[g][m01] = v[0];
                    s[m] = B.xsum(v);
                    return s[m];
                }
                s[m] = B.xsum(terms);
                return s[m];
            };
            for (uint32_t h = 0; h < H; ++h) {
                B.grp = h < hA ? 4 : 1;
                subp = &sub_all[h < hA ? 1 : 0];
                for (uint32_t b = 0; b < 8; ++b)
                    for (size_t g = 0; g < ng; ++g) {
                        uint32_t m = 0;
                        for (uint32_t q = 0; q < 4 && g * 4 + q < chunk.size(); ++q) {
                            const uint32_t c = e.piv_col[chunk[g * 4 + q]];
                            if ((e.G[(size_t)h * KS + c] >> b) & 1) m |= 1u << q;
                        }
                        if (m) S8[h * 8 + b].push(B, subset(g, m));
                    }
            }
            chunk.clear();
            B.grp = 0;
        };
        for (uint32_t k = 0; k < npiv; ++k) {
            std::vector<uint32_t> tt{D(e.piv_row[k])};
            yacc[k].append_to(tt);
            y[k] = B.xsum(tt);
            ystate[k] = 2;
            for (uint32_t d : dependents[k]) yacc[d].push(B, y[k], may_pend(d, k));
            const uint32_t c = e.piv_col[k];
            B.grp = 2;
            for (uint32_t i : col_rem[c]) b2acc[i].push(B, y[k], may_pend(npiv + i, k));
            for (uint32_t o : col_outs[c]) oacc[o].push(B, y[k], may_pend(npiv + n2 + o, k));
            B.grp = 0;
            ir->st.push_dep += (uint32_t)dependents[k].size();
            ir->st.push_rem += (uint32_t)col_rem[c].size();
            ir->st.push_out += (uint32_t)col_outs[c].size();
            if (c < KS && y[k] != NOVAL) {
                chunk.push_back(k);
                if (chunk.size() == 8) flush();
            }
        }
        flush();
        bh_direct.assign(H, NOVAL);
        for (uint32_t h = 0; h < H; ++h) {
            B.grp = h < hA ? 4 : 1;
            uint32_t acc = NOVAL;
            for (int b = 7; b >= 0; --b) acc = B.xt(acc, S8[h * 8 + b].get(B));
            bh_direct[h] = acc;
        }
        B.grp = 0;
    } else if (passes & SCHED_RS) {
        // Peeling-order production, push-mode dependencies; the Horner chain absorbs the produced y
        // values by replacement selection: at most `hbuf` of them wait, and whenever the buffer is
        // over budget the chain advances to the smallest buffered column beyond its cursor.  When no
        // buffered column lies ahead, the chain parks (its state waits at its cursor) and a new run
        // starts at the smallest buffered column; a run that reaches a parked cursor merges with it.
        // The scan is linear, so the runs' pushes and end values add up to the single scan's; a buffer
        // of ~0.37 npiv gives one run (~KS xtimes) where fixed peeling-order passes need two.
        const uint32_t hbuf = passes & 0xFFFFu;
        std::vector<std::vector<uint32_t>> dependents(npiv);
        for (uint32_t k = 0; k < npiv; ++k)
            for (uint32_t j : e.deps[k]) dependents[j].push_back(k);
        std::vector<Acc> yacc(npiv);
        std::set<uint32_t> buf;                     // buffered (produced, not absorbed) pivoted columns
        std::map<uint32_t, uint32_t> parked;        // cursor column -> parked chain state
        int64_t cur = -1;                           // active chain: last column visited
        uint32_t tp = NOVAL;
        auto step_to = [&](uint32_t c) {            // advance the active chain through column c
            uint32_t yj = NOVAL;
            auto it = buf.find(c);
            if (it != buf.end()) { yj = y[(uint32_t)e.col_order[c]]; buf.erase(it); }
            tp = B.xt(tp, yj);
            if (c + 1 < KS && tp != NOVAL) {
                part[e.ma[c]].push(B, tp);
                part[e.mb[c]].push(B, tp);
            }
            auto pk = parked.find(c);
            if (pk != parked.end()) {
                std::vector<uint32_t> v{tp, pk->second};
                tp = B.xsum(v);
                parked.erase(pk);
            }
            cur = c;
        };
        auto absorb_one = [&]() {
            auto it = buf.upper_bound((uint32_t)std::max<int64_t>(cur, -1));
            if (cur < 0) it = buf.begin();
            if (it == buf.end()) {          // nothing ahead: park this run, start the next one
                if (tp != NOVAL) {
                    auto pk = parked.find((uint32_t)cur);
                    if (pk == parked.end()) parked[(uint32_t)cur] = tp;
                    else { std::vector<uint32_t> v{tp, pk->second}; pk->second = B.xsum(v); }
                }
                tp = NOVAL;
                it = buf.begin();
            }
            const uint32_t target = *it;
            // a fresh run starts at its first column: the columns before carry a zero state
            if (tp == NOVAL) cur = (int64_t)target - 1;
            while ((uint32_t)(cur + 1) <= target) step_to((uint32_t)(cur + 1));
        };
        for (uint32_t k = 0; k < npiv; ++k) {
            std::vector<uint32_t> tt{D(e.piv_row[k])};
            yacc[k].append_to(tt);
            y[k] = B.xsum(tt);
            ystate[k] = 2;
            for (uint32_t d : dependents[k]) yacc[d].push(B, y[k]);
            const uint32_t c = e.piv_col[k];
            for (uint32_t i : col_rem[c]) b2acc[i].push(B, y[k]);
            for (uint32_t o : col_outs[c]) oacc[o].push(B, y[k]);
            if (c < KS && y[k] != NOVAL) buf.insert(c);
            while (buf.size() > hbuf) absorb_one();
        }
        while (!buf.empty()) absorb_one();
        // finish: the active chain and every parked one run to column KS - 1
        if (tp != NOVAL || !parked.empty()) {
            if (tp == NOVAL) { cur = (int64_t)parked.begin()->first; tp = parked.begin()->second; parked.erase(parked.begin()); }
            while (cur + 1 < (int64_t)KS) step_to((uint32_t)(cur + 1));
            t = tp;
        }
    } else if (passes) {  // peeling-order production, push-mode dependencies, P Horner passes
        std::vector<std::vector<uint32_t>> dependents(npiv);
        for (uint32_t k = 0; k < npiv; ++k)
            for (uint32_t j : e.deps[k]) dependents[j].push_back(k);
        std::vector<Acc> yacc(npiv);
        std::vector<uint32_t> tends;
        // Horner pass over the y values of peeling positions [lo, hi), advanced a few columns at a
        // time: with `interleave`, pass q runs woven into the production of group q + 1 (whose
        // source loads then overlap its VALU work) instead of after it
        struct PassGen { uint32_t lo = 0, hi = 0, j = 0, tp = NOVAL; bool on = false; } pg;
        auto advance = [&](uint32_t ncols) {
            for (uint32_t c = 0; c < ncols && pg.on; ++c, ++pg.j) {
                if (pg.j == KS) {
                    if (pg.tp != NOVAL) tends.push_back(pg.tp);
                    pg.on = false;
                    break;
                }
                const uint32_t j = pg.j;
                uint32_t yj = NOVAL;
                if (e.cstate[j] == 1) {
                    const uint32_t k = (uint32_t)e.col_order[j];
                    if (k >= pg.lo && k < pg.hi) yj = y[k];
                }
                pg.tp = B.xt(pg.tp, yj);
                if (j + 1 < KS && pg.tp != NOVAL) {
                    part[e.ma[j]].push(B, pg.tp);
                    part[e.mb[j]].push(B, pg.tp);
                }
            }
        };
        const bool weave = interleave_passes();
        uint32_t q = 1, lo = 0, credit = 0;
        for (uint32_t k = 0; k < npiv; ++k) {
            std::vector<uint32_t> tt{D(e.piv_row[k])};
            yacc[k].append_to(tt);
            y[k] = B.xsum(tt);
            ystate[k] = 2;
            for (uint32_t d : dependents[k]) yacc[d].push(B, y[k]);
            const uint32_t c = e.piv_col[k];
            for (uint32_t i : col_rem[c]) b2acc[i].push(B, y[k]);
            for (uint32_t o : col_outs[c]) oacc[o].push(B, y[k]);
            if (pg.on) {  // KS columns of the running pass spread over this group's productions
                credit += KS * passes;
                advance(credit / npiv);
                credit %= npiv;
            }
            if (k + 1 == (uint64_t)npiv * q / passes) {
                advance(KS + 1);  // finish the previous pass
                pg = PassGen{lo, k + 1, 0, NOVAL, true};
                lo = k + 1;
                credit = 0;
                if (!weave) advance(KS + 1);
                ++q;
            }
        }
        advance(KS + 1);
        t = B.xsum(tends);
    }
    for (uint32_t j = 0; j < KS && !passes; ++j) {
        const uint32_t yj = (e.cstate[j] == 1) ? getY((uint32_t)e.col_order[j]) : NOVAL;
        t = B.xt(t, yj);
        if (j + 1 < KS && t != NOVAL) {
            part[e.ma[j]].push(B, t);
            part[e.mb[j]].push(B, t);
        }
        if (yj != NOVAL) {
            for (uint32_t i : col_rem[j]) b2acc[i].push(B, yj);
            for (uint32_t o : col_outs[j]) oacc[o].push(B, yj);
        }
    }
    for (uint32_t c = KS; c < e.L && !passes; ++c) {  // pivoted columns past the HDPC range (none in practice)
        if (e.cstate[c] != 1) continue;
        const uint32_t yc = getY((uint32_t)e.col_order[c]);
        for (uint32_t i : col_rem[c]) b2acc[i].push(B, yc);
        for (uint32_t o : col_outs[c]) oacc[o].push(B, yc);
    }
    // bh_h = part_h ^ alpha^h * t_(KS-1)
    std::vector<uint32_t> bh(H), b2(n2);
    if (!bh_direct.empty()) {
        bh = bh_direct;
    } else {
        uint32_t s = t;
        for (uint32_t h = 0; h < H; ++h) {
            if (h) s = B.xt(s);
            std::vector<uint32_t> v{part[h].get(B), s};
            bh[h] = B.xsum(v);
        }
    }
    B.grp = 2;
    for (uint32_t i = 0; i < n2; ++i) b2[i] = b2acc[i].get(B);

    // ---- dense part: C_F[f] = sum_bit alpha^bit X_bit[f], X_bit[f] = bits of Zi[f]*bh ^ Q[f]*b2
    // ---- outputs: out_o = oacc_o ^ V1_o*b2 ^ V2_o*C_F
    ir->phase_start[2] = (uint32_t)ir->nodes.size();
    B.grp = 3;
    std::vector<uint32_t> CF(H, NOVAL);
    std::vector<uint32_t> outv(no, NOVAL);
    const uint32_t dg = dense_group();
    if (dg) {
        // Four Russians over the inputs (round 3): the 8H bit rows X_bit[f] and the output rows are
        // GF(2) combinations of the n2 + H values b2 ++ bh, then the outputs of the H values C_F.  The
        // inputs are cut into groups of dg; a group's subset XORs are built once (only the subsets
        // some row uses) and every row takes one subset per group, so a row costs one XOR3 per two
        // groups instead of one per two terms (~half its n2/2 terms).  The output rows' b2 part rides
        // along with the dense rows; their C_F part follows the Horner chains.  Same XOR sets as the
        // direct sums: bit-identical.
        struct Row { Acc acc; std::vector<uint32_t> idx; };  // input indices with a one
        auto run = [&](const std::vector<uint32_t>& in, std::vector<Row*>& rws) {
            const uint32_t ni = (uint32_t)in.size(), ng = (ni + dg - 1) / dg;
            std::vector<std::vector<uint32_t>> mask(rws.size(), std::vector<uint32_t>(ng, 0));
            for (size_t r = 0; r < rws.size(); ++r)
                for (uint32_t x : rws[r]->idx) mask[r][x / dg] ^= 1u << (x % dg);
            for (uint32_t g0 = 0; g0 < ng; ++g0) {
                std::vector<uint32_t> sub(1u << dg, NOVAL);
                std::vector<uint8_t> built(1u << dg, 0);
                std::function<uint32_t(uint32_t)> subset = [&](uint32_t m) -> uint32_t {
                    if (built[m]) return sub[m];
                    built[m] = 1;
                    std::vector<uint32_t> mem;
                    for (uint32_t q = 0; q < dg; ++q)
                        if (m >> q & 1) mem.push_back(g0 * dg + q < ni ? in[g0 * dg + q] : NOVAL);
                    uint32_t v;
                    if (mem.size() <= 2) {
                        v = B.xsum(mem);
                    } else {  // the subset without its two highest members, then XOR3 those in
                        uint32_t rest = m, hi2[2], k = 0;
                        for (int q = (int)dg - 1; q >= 0 && k < 2; --q)
                            if (rest >> q & 1) { hi2[k++] = (uint32_t)q; rest &= ~(1u << q); }
                        std::vector<uint32_t> t{subset(rest), g0 * dg + hi2[0] < ni ? in[g0 * dg + hi2[0]] : NOVAL,
                                                g0 * dg + hi2[1] < ni ? in[g0 * dg + hi2[1]] : NOVAL};
                        v = B.xsum(t);
                    }
                    sub[m] = v;
                    return v;
                };
                for (size_t r = 0; r < rws.size(); ++r)
                    if (mask[r][g0]) rws[r]->acc.push(B, subset(mask[r][g0]));
            }
        };
        std::vector<uint32_t> in1(b2);
        in1.insert(in1.end(), bh.begin(), bh.end());
        std::vector<Row> drow((size_t)H * 8), orow(no);
        std::vector<Row*> rws;
        for (uint32_t f = 0; f < H; ++f)
            for (uint32_t bt = 0; bt < 8; ++bt) {
                Row& r = drow[(size_t)f * 8 + bt];
                for (uint32_t h = 0; h < H; ++h)
                    if ((e.Zi[(size_t)f * H + h] >> bt) & 1) r.idx.push_back(n2 + h);
                for (uint32_t m = 0; m < n2; ++m)
                    if ((e.Q[(size_t)f * n2 + m] >> bt) & 1) r.idx.push_back(m);
                rws.push_back(&r);
            }
        for (uint32_t o = 0; o < no; ++o) {
            if (outs[o].source) continue;
            Row& r = orow[o];
            std::vector<uint32_t> t0;
            oacc[o].append_to(t0);
            for (uint32_t v : t0) r.acc.push(B, v);
            for (uint32_t m = 0; m < n2; ++m)
                if (bit(V1[o].data(), m)) r.idx.push_back(m);
            rws.push_back(&r);
        }
        run(in1, rws);
        for (uint32_t f = 0; f < H; ++f) {
            uint32_t acc = NOVAL;
            for (int bt = 7; bt >= 0; --bt) acc = B.xt(acc, drow[(size_t)f * 8 + bt].acc.get(B));
            CF[f] = acc;
        }
        ir->phase_start[3] = (uint32_t)ir->nodes.size();
        std::vector<Row*> rw2;
        for (uint32_t o = 0; o < no; ++o) {
            if (outs[o].source) continue;
            orow[o].idx.clear();
            for (uint32_t f = 0; f < H; ++f)
                if (bit(V2[o].data(), f)) orow[o].idx.push_back(f);
            rw2.push_back(&orow[o]);
        }
        run(CF, rw2);
        for (uint32_t o = 0; o < no; ++o)
            if (!outs[o].source) outv[o] = orow[o].acc.get(B);
    } else {
        for (uint32_t f = 0; f < H; ++f) {
            uint32_t acc = NOVAL;
            for (int bt = 7; bt >= 0; --bt) {
                std::vector<uint32_t> terms;
                for (uint32_t h = 0; h < H; ++h)
                    if ((e.Zi[(size_t)f * H + h] >> bt) & 1) terms.push_back(bh[h]);
                for (uint32_t m = 0; m < n2; ++m)
                    if ((e.Q[(size_t)f * n2 + m] >> bt) & 1) terms.push_back(b2[m]);
                const uint32_t x = B.xsum(terms);
                acc = B.xt(acc, x);
            }
            CF[f] = acc;
        }
        ir->phase_start[3] = (uint32_t)ir->nodes.size();
        for (uint32_t o = 0; o < no; ++o) {
            if (outs[o].source) continue;
            std::vector<uint32_t> terms;
            oacc[o].append_to(terms);
            for (uint32_t m = 0; m < n2; ++m)
                if (bit(V1[o].data(), m)) terms.push_back(b2[m]);
            for (uint32_t f = 0; f < H; ++f)
                if (bit(V2[o].data(), f)) terms.push_back(CF[f]);
            outv[o] = B.xsum(terms);
        }
    }
    for (uint32_t o = 0; o < no; ++o) {
        uint32_t v = outv[o];
        if (outs[o].source) v = outs[o].row < K ? B.add(IR_LOAD, NOVAL, NOVAL, NOVAL, outs[o].row) : NOVAL;
        if (v == NOVAL) v = B.add(IR_ZERO);
        B.add(IR_STORE, v, NOVAL, NOVAL, o);
    }
    B.grp = 0;
    // dead-code elimination: keep only what the stores need (e.g. outputs that are all source rows)
    {
        std::vector<uint8_t> live(ir->nodes.size(), 0);
        for (size_t i = ir->nodes.size(); i-- > 0;) {
            const IrNode& n = ir->nodes[i];
            if (n.k == IR_STORE) live[i] = 1;
            if (!live[i]) continue;
            for (uint32_t x : {n.a, n.b, n.c})
                if (x != NOVAL) live[x] = 1;
        }
        std::vector<uint32_t> remap(ir->nodes.size(), NOVAL);
        std::vector<IrNode> kept;
        kept.reserve(ir->nodes.size());
        uint32_t ph = 0, new_ph[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < ir->nodes.size(); ++i) {
            while (ph < 4 && ir->phase_start[ph] == i) new_ph[ph++] = (uint32_t)kept.size();
            if (!live[i]) continue;
            IrNode n = ir->nodes[i];
            for (uint32_t* x : {&n.a, &n.b, &n.c})
                if (*x != NOVAL) *x = remap[*x];
            remap[i] = (uint32_t)kept.size();
            kept.push_back(n);
        }
        while (ph < 4) new_ph[ph++] = (uint32_t)kept.size();
        ir->nodes.swap(kept);
        std::memcpy(ir->phase_start, new_ph, sizeof new_ph);
    }
    auto& st = ir->st;
    for (const IrNode& n : ir->nodes) {
        switch (n.k) {
            case IR_LOAD: ++st.load; break;
            case IR_ZERO: ++st.zero; break;
            case IR_XOR2: ++st.xor2; break;
            case IR_XOR3: ++st.xor3; break;
            case IR_XT: ++st.xt; break;
            case IR_XTX: ++st.xtx; break;
            case IR_STORE: ++st.store; break;
        }
    }
    st.u = u; st.npiv = npiv; st.n2 = n2;
    return true;
}

inline uint32_t xtime4(uint32_t x) {
    const uint32_t hi = (x >> 7) & 0x01010101u;
    return ((x & 0x7F7F7F7Fu) << 1) ^ (hi * 0x1Du);
}

}  // namespace

bool build_colprog(const Params& p, const uint32_t* esi, uint32_t n_out, ColIR* ir, std::string* err, uint32_t passes) {
    std::vector<OutDesc> outs(n_out);
    uint32_t cols[64];
    for (uint32_t o = 0; o < n_out; ++o) {
        if (esi[o] < p.K) { outs[o].source = true; outs[o].row = esi[o]; continue; }
        const int n = lt_cols(p, esi[o] + p.Kp - p.K, cols);
        outs[o].cols.assign(cols, cols + n);
    }
    return build(p, outs, passes, ir, err);
}

bool build_colprog_C(const Params& p, ColIR* ir, std::string* err, uint32_t passes) {
    std::vector<OutDesc> outs(p.L);
    for (uint32_t c = 0; c < p.L; ++c) outs[c].cols = {c};
    return build(p, outs, passes, ir, err);
}

void eval_colprog(const ColIR& ir, const uint8_t* src, uint32_t T, uint8_t* out) {
    const uint32_t Td = T / 4;
    std::vector<uint32_t> v((size_t)ir.nodes.size() * Td, 0);
    auto V = [&](uint32_t i) { return &v[(size_t)i * Td]; };
    for (uint32_t i = 0; i < ir.nodes.size(); ++i) {
        const IrNode& n = ir.nodes[i];
        uint32_t* d = V(i);
        switch (n.k) {
            case IR_LOAD: std::memcpy(d, src + (size_t)n.imm * T, (size_t)Td * 4); break;
            case IR_ZERO: break;
            case IR_XOR2: for (uint32_t c = 0; c < Td; ++c) d[c] = V(n.a)[c] ^ V(n.b)[c]; break;
            case IR_XOR3: for (uint32_t c = 0; c < Td; ++c) d[c] = V(n.a)[c] ^ V(n.b)[c] ^ V(n.c)[c]; break;
            case IR_XT: for (uint32_t c = 0; c < Td; ++c) d[c] = xtime4(V(n.a)[c]); break;
            case IR_XTX: for (uint32_t c = 0; c < Td; ++c) d[c] = xtime4(V(n.a)[c]) ^ V(n.b)[c]; break;
            case IR_STORE: std::memcpy(out + (size_t)n.imm * T, V(n.a), (size_t)Td * 4); break;
        }
    }
}

}  // namespace rq
