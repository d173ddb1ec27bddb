// rq_plan.cpp -- per-K' encode schedule compiler (see rq_plan.hpp for the program shape).
//
// Constraint system (RQ/solver.go:25-65, RQ/params.go:116-160):
//   S LDPC rows (circulant B part, identity on B..B+S-1, two PI columns), rhs 0
//   K' LT rows (ISI 0..K'-1), rhs = padded source symbol
//   H HDPC rows [MT*Gamma | I_H], rhs 0 -- never materialised, handled by Horner chunks.
#include "rq_plan.hpp"

#include <algorithm>
#include <cstdio>

namespace rq {

const GF& gf() {
    static const GF g;
    return g;
}

namespace {

inline uint32_t src_word(uint32_t slot, uint32_t coef = 1) { return (slot & 0xFFFFu) | ((coef & 0xFFu) << 16); }

struct Builder {
    std::vector<Stmt> stmts;
    uint32_t phase = 0;
    void push(Stmt&& s) { s.phase = phase; stmts.push_back(std::move(s)); }
    void xor_(uint16_t dst, bool acc, const std::vector<uint32_t>& slots) {
        if (acc && slots.empty()) return;
        Stmt s;
        s.type = ST_XOR; s.acc = acc; s.dst = dst;
        for (uint32_t x : slots) s.src.push_back(src_word(x));
        push(std::move(s));
    }
    void muladd(uint16_t dst, uint16_t src, uint8_t c) {
        Stmt s;
        s.type = (c == 1) ? ST_XOR : ST_MUL; s.acc = true; s.dst = dst;
        s.src.push_back(src_word(src, c));
        push(std::move(s));
    }
    void xor_words(uint16_t dst, bool acc, const std::vector<uint32_t>& words) {
        if (acc && words.empty()) return;
        Stmt s;
        s.type = ST_XOR; s.acc = acc; s.dst = dst; s.src = words;
        push(std::move(s));
    }
    void mul_words(uint16_t dst, bool acc, const std::vector<uint32_t>& words) {
        if (acc && words.empty()) return;
        Stmt s;
        s.type = ST_MUL; s.acc = acc; s.dst = dst; s.src = words;
        push(std::move(s));
    }
    void scale(uint16_t dst, uint8_t c) {
        Stmt s;
        s.type = ST_SCALE; s.acc = true; s.dst = dst; s.extra = c;
        push(std::move(s));
    }
};

// Slots read / written by a statement (for the list scheduler).
void stmt_slots(const Stmt& s, uint32_t H, std::vector<uint32_t>* rd, std::vector<uint32_t>* wr) {
    rd->clear(); wr->clear();
    if (s.type == ST_HORNER) {
        for (size_t i = 0; i + s.extra < s.src.size(); ++i) {   // trailing tau words are not slots
            const uint32_t slot = s.src[i] & 0xFFFFu;
            if (slot != SLOT_NONE) rd->push_back(slot);
        }
        for (uint32_t h = 0; h < H; ++h) wr->push_back(s.dst + h);
        return;
    }
    for (uint32_t w : s.src)
        if (!(w & SRC_GLOBAL)) rd->push_back(w & 0xFFFFu);
    if (s.acc || s.type == ST_SCALE) rd->push_back(s.dst);
    wr->push_back(s.dst);
}

}  // namespace

bool compile_encode_plan(const Params& p, Plan* out, std::string* err, const PlanOptions& opt) {
    const uint32_t Q = opt.horner_chunks;
    const GF& g = gf();
    const uint32_t L = p.L, S = p.S, H = p.H, Kp = p.Kp, W = p.W, P = p.P, KS = Kp + S;
    const uint32_t NR = S + Kp;  // GF(2) rows: LDPC 0..S-1, LT S..S+K'-1
    out->p = p;

    // ---------------- sparse GF(2) rows ----------------
    std::vector<std::vector<uint32_t>> rows(NR);
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
    for (uint32_t i = 0; i < Kp; ++i) {
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

    // ---------------- peeling with inactivation (cf. RQ/inactivate.go:25-170) ----------------
    enum : uint8_t { ACTIVE = 0, PIVOTED = 1, INACTIVE = 2 };
    std::vector<uint8_t> cstate(L, ACTIVE);
    for (uint32_t c = W; c < L; ++c) cstate[c] = INACTIVE;  // PI columns start inactive
    std::vector<uint32_t> cnt(NR, 0);
    std::vector<uint8_t> rdone(NR, 0);
    for (uint32_t r = 0; r < NR; ++r)
        for (uint32_t c : rows[r]) cnt[r] += (cstate[c] == ACTIVE);
    std::vector<uint32_t> live_deg(L, 0);  // active rows (not done) per column
    for (uint32_t c = 0; c < L; ++c) live_deg[c] = (uint32_t)col_rows[c].size();
    // FIFO buckets by active count: rows released by a pivot are taken after the rows that were
    // already eligible (breadth-first peeling rounds keep the substitution DAG shallow).
    std::vector<std::vector<uint32_t>> bucket(64);
    std::vector<size_t> bhead(64, 0);
    for (uint32_t r = 0; r < NR; ++r) bucket[std::min<uint32_t>(cnt[r], 63)].push_back(r);
    std::vector<uint32_t> ucols;  // inactive columns in order: PI first, then inactivated
    for (uint32_t c = W; c < L; ++c) ucols.push_back(c);
    std::vector<uint32_t> piv_row, piv_col;
    std::vector<int32_t> col_order(L, -1);
    uint32_t inactivated = 0;

    auto drop_col = [&](uint32_t c, uint32_t except_row) {
        for (uint32_t r : col_rows[c]) {
            if (rdone[r] || r == except_row) continue;
            --cnt[r];
            bucket[std::min<uint32_t>(cnt[r], 63)].push_back(r);
        }
    };
    for (;;) {
        int32_t r = -1;
        for (uint32_t b = 1; b < 64 && r < 0; ++b) {
            auto& bk = bucket[b];
            while (bhead[b] < bk.size()) {
                const uint32_t x = bk[bhead[b]++];
                if (!rdone[x] && std::min<uint32_t>(cnt[x], 63) == b) { r = (int32_t)x; break; }
            }
        }
        if (r < 0) break;
        // pivot = active column with the most unfinished rows; the rest become inactive.
        uint32_t best = UINT32_MAX, best_deg = 0;
        for (uint32_t c : rows[r])
            if (cstate[c] == ACTIVE && (best == UINT32_MAX || live_deg[c] > best_deg)) { best = c; best_deg = live_deg[c]; }
        for (uint32_t c : rows[r]) {
            if (cstate[c] != ACTIVE || c == best) continue;
            cstate[c] = INACTIVE;
            ucols.push_back(c);
            ++inactivated;
            drop_col(c, UINT32_MAX);
        }
        cstate[best] = PIVOTED;
        col_order[best] = (int32_t)piv_col.size();
        piv_row.push_back((uint32_t)r);
        piv_col.push_back(best);
        rdone[r] = 1;
        drop_col(best, (uint32_t)r);
        for (uint32_t c : rows[r]) --live_deg[c];
    }
    // columns still active appear in no remaining row -> singular
    for (uint32_t c = 0; c < L; ++c)
        if (cstate[c] == ACTIVE) { cstate[c] = INACTIVE; ucols.push_back(c); ++inactivated; }

    const uint32_t u = (uint32_t)ucols.size();
    const uint32_t npiv = (uint32_t)piv_col.size();
    std::vector<uint32_t> rem;  // remaining GF(2) rows
    for (uint32_t r = 0; r < NR; ++r)
        if (!rdone[r]) rem.push_back(r);
    if (rem.size() + H != u) {
        if (err) *err = "plan: remaining rows != inactive columns";
        return false;
    }
    std::vector<int32_t> uidx(L, -1);
    for (uint32_t j = 0; j < u; ++j) uidx[ucols[j]] = (int32_t)j;

    // ---------------- slots ----------------
    // slot(c) = c for every column; remaining rows own the U-column slots; HDPC rows the last H.
    // Temporaries after L: Horner partials (Q*H), later reused by the dense solve (u slots).
    std::vector<uint16_t> row_slot(NR + H, SLOT_NONE);
    for (uint32_t k = 0; k < npiv; ++k) row_slot[piv_row[k]] = (uint16_t)piv_col[k];
    for (uint32_t i = 0; i < rem.size(); ++i) row_slot[rem[i]] = (uint16_t)ucols[i];
    for (uint32_t h = 0; h < H; ++h) row_slot[NR + h] = (uint16_t)ucols[rem.size() + h];
    const uint32_t tmp_base = L;
    const uint32_t nq = std::min<uint32_t>(Q, KS);
    out->n_slots = L + std::max<uint32_t>(nq * H, u);
    if (out->n_slots > 0xFFF0u) {
        if (err) *err = "plan: too many slots";
        return false;
    }
    out->load_slot.resize(Kp);
    for (uint32_t i = 0; i < Kp; ++i) out->load_slot[i] = row_slot[S + i];

    Builder bld;
    const uint32_t nw = (u + 63) / 64;
    std::vector<uint64_t> Wb((size_t)npiv * nw, 0);
    auto wrow = [&](uint32_t k) { return &Wb[(size_t)k * nw]; };
    // Term sets (XOR parity): slot term = pivot index j (< 2^24); global term = TG | isi.
    constexpr uint32_t TG = 1u << 31;
    auto symdiff = [](const std::vector<uint32_t>& a, const std::vector<uint32_t>& b) {
        std::vector<uint32_t> r;
        r.reserve(a.size() + b.size());
        size_t i = 0, j = 0;
        while (i < a.size() || j < b.size()) {
            if (j == b.size() || (i < a.size() && a[i] < b[j])) r.push_back(a[i++]);
            else if (i == a.size() || b[j] < a[i]) r.push_back(b[j++]);
            else { ++i; ++j; }
        }
        return r;
    };
    auto is_lt = [&](uint32_t k) { return piv_row[k] >= S; };
    auto src_of = [&](uint32_t t) { return (t & TG) ? t : src_word(piv_col[t]); };

    // ---------------- pass A: y = T^-1 D, in place, depth-capped by inlining ----------------
    bld.phase = 0;
    std::vector<std::vector<uint32_t>> deps(npiv), rowu(npiv);
    std::vector<std::vector<uint32_t>> fullA(npiv);  // y_k as terms incl. its own source row
    std::vector<uint32_t> depA(npiv, 0);
    for (uint32_t k = 0; k < npiv; ++k) {
        const uint32_t r = piv_row[k];
        uint64_t* wk = wrow(k);
        for (uint32_t c : rows[r]) {
            if (c == piv_col[k]) continue;
            if (cstate[c] == PIVOTED) {
                deps[k].push_back((uint32_t)col_order[c]);
                const uint64_t* wd = wrow((uint32_t)col_order[c]);
                for (uint32_t x = 0; x < nw; ++x) wk[x] ^= wd[x];
            } else {
                rowu[k].push_back(c);
                const uint32_t j = (uint32_t)uidx[c];
                wk[j >> 6] ^= 1ull << (j & 63);
            }
        }
        std::vector<uint32_t> terms(deps[k]);
        std::sort(terms.begin(), terms.end());
        for (;;) {
            uint32_t dmax = 0, jmax = 0;
            for (uint32_t t : terms)
                if (!(t & TG) && depA[t] + 1 > dmax) { dmax = depA[t] + 1; jmax = t; }
            if (dmax <= opt.depth_a) break;
            terms = symdiff(terms, std::vector<uint32_t>{jmax});
            terms = symdiff(terms, fullA[jmax]);
        }
        uint32_t d = 0;
        for (uint32_t t : terms)
            if (!(t & TG)) d = std::max(d, depA[t] + 1);
        depA[k] = d;
        fullA[k] = is_lt(k) ? symdiff(terms, std::vector<uint32_t>{TG | (r - S)}) : terms;
        std::vector<uint32_t> s;
        for (uint32_t t : terms) s.push_back(src_of(t));
        bld.xor_words((uint16_t)piv_col[k], true, s);
    }

    // ---------------- dense matrix Mu (u x u) and the remaining GF(2) rows ----------------
    bld.phase = 1;
    std::vector<uint8_t> Mu((size_t)u * u, 0);
    for (uint32_t i = 0; i < rem.size(); ++i) {
        const uint32_t r = rem[i];
        std::vector<uint64_t> acc(nw, 0);
        std::vector<uint32_t> s;
        for (uint32_t c : rows[r]) {
            if (cstate[c] == PIVOTED) {
                s.push_back(src_word(c));
                const uint64_t* wd = wrow((uint32_t)col_order[c]);
                for (uint32_t x = 0; x < nw; ++x) acc[x] ^= wd[x];
            } else {
                const uint32_t j = (uint32_t)uidx[c];
                acc[j >> 6] ^= 1ull << (j & 63);
            }
        }
        for (uint32_t j = 0; j < u; ++j) Mu[(size_t)i * u + j] = (acc[j >> 6] >> (j & 63)) & 1;
        bld.xor_words(row_slot[r], true, s);
    }

    // ---------------- HDPC: MT, G = MT*Gamma, Horner chunks ----------------
    std::vector<uint8_t> ma(KS), mb(KS);
    for (uint32_t j = 0; j + 1 < KS; ++j) {
        const uint32_t a = rand_(j + 1, 6, H);
        ma[j] = (uint8_t)a;
        mb[j] = (uint8_t)((a + rand_(j + 1, 7, H - 1) + 1) % H);
    }
    auto MT = [&](uint32_t h, uint32_t j) -> uint8_t {
        if (j == KS - 1) return g.pow_alpha(h);
        return (ma[j] == h || mb[j] == h) ? 1 : 0;
    };
    std::vector<uint8_t> G((size_t)H * KS);
    std::vector<uint8_t> F((size_t)H * (KS + 1), 0);  // F[h][e] = sum_{j>=e} MT[h][j] alpha^(j-e+1)
    for (uint32_t h = 0; h < H; ++h) {
        uint8_t acc = 0;
        for (int64_t j = (int64_t)KS - 1; j >= 0; --j) {
            acc = (uint8_t)(g.mul(acc, 2) ^ MT(h, (uint32_t)j));
            G[(size_t)h * KS + j] = acc;
        }
        uint8_t f = 0;
        for (int64_t e = (int64_t)KS - 1; e >= 0; --e) {
            f = g.mul(2, (uint8_t)(MT(h, (uint32_t)e) ^ f));
            F[(size_t)h * (KS + 1) + e] = f;
        }
    }
    for (uint32_t h = 0; h < H; ++h) {  // coefficients of the HDPC rows on U
        uint8_t* mrow = &Mu[(size_t)(rem.size() + h) * u];
        for (uint32_t j = 0; j < u; ++j) {
            const uint32_t c = ucols[j];
            uint8_t v = (c < KS) ? G[(size_t)h * KS + c] : 0;
            if (c == KS + h) v ^= 1;
            mrow[j] = v;
        }
        for (uint32_t k = 0; k < npiv; ++k) {
            const uint8_t gc = G[(size_t)h * KS + piv_col[k]];
            if (!gc) continue;
            const uint64_t* wk = wrow(k);
            for (uint32_t x = 0; x < nw; ++x) {
                uint64_t bits = wk[x];
                while (bits) {
                    const uint32_t j = x * 64 + (uint32_t)__builtin_ctzll(bits);
                    bits &= bits - 1;
                    mrow[j] ^= gc;
                }
            }
        }
    }
    bld.phase = 2;  // Horner chunks over columns 0..KS-1 (y of pivoted columns, zero otherwise)
    for (uint32_t q = 0; q < nq; ++q) {
        const uint32_t s0 = (uint32_t)((uint64_t)KS * q / nq), e0 = (uint32_t)((uint64_t)KS * (q + 1) / nq);
        Stmt st;
        st.type = ST_HORNER; st.acc = false; st.dst = (uint16_t)(tmp_base + q * H);
        for (uint32_t j = s0; j < e0; ++j) {
            // The last column (MT[h][KS-1] = alpha^h) scatters nothing (a == b cancels); its
            // alpha^h * t term is folded into the final chunk's tau below.
            const uint32_t slot = (cstate[j] == PIVOTED) ? j : SLOT_NONE;
            const bool last = j == KS - 1;
            st.src.push_back((slot & 0xFFFFu) | ((uint32_t)(last ? 0 : ma[j]) << 16) | ((uint32_t)(last ? 0 : mb[j]) << 21));
        }
        uint32_t word = 0;
        std::vector<uint32_t> tau;
        for (uint32_t h = 0; h < H; ++h) {
            const uint8_t th = (uint8_t)(F[(size_t)h * (KS + 1) + e0] ^ (e0 == KS ? g.pow_alpha(h) : 0));
            word |= (uint32_t)th << (8 * (h & 3));
            if ((h & 3) == 3 || h + 1 == H) { tau.push_back(word); word = 0; }
        }
        st.extra = (uint32_t)tau.size();
        for (uint32_t w : tau) st.src.push_back(w);  // trailing tau words (counted in extra)
        bld.push(std::move(st));
    }
    bld.phase = 3;
    for (uint32_t h = 0; h < H; ++h) {
        std::vector<uint32_t> parts;
        for (uint32_t q = 0; q < nq; ++q) parts.push_back(src_word(tmp_base + q * H + h));
        bld.xor_words(row_slot[NR + h], true, parts);
    }

    // ---------------- dense solve on U (replaces GaussianElimination, RQ/discmath/gauss.go:7-45) ----
    // Rows 0..n2-1 are GF(2) (slots dslot[i]), rows n2..u-1 the HDPC rows.  Pick pivot columns Pc
    // for the GF(2) block, E2 = Mu2[:,Pc]^-1 and R = E2*Mu2[:,Fc] over GF(2); then
    //   t   = E2 b2                      (XOR gathers, temps)
    //   bh' = bh ^ Mh[:,Pc] t            (mul-add gathers, in place)
    //   CF  = (Mh[:,Fc] ^ Mh[:,Pc] R)^-1 bh'   (H x H, temps)
    //   CP  = t ^ R CF                   (XOR, in place on temps)
    bld.phase = 4;
    const uint32_t n2 = (uint32_t)rem.size();
    std::vector<uint16_t> dslot(u);
    for (uint32_t i = 0; i < n2; ++i) dslot[i] = row_slot[rem[i]];
    for (uint32_t h = 0; h < H; ++h) dslot[n2 + h] = row_slot[NR + h];
    auto mu = [&](uint32_t r, uint32_t c) -> uint8_t& { return Mu[(size_t)r * u + c]; };
    // GF(2) elimination on [Mu2 | I] to find Pc and E2 (bit rows of length u + n2)
    const uint32_t bw = (u + n2 + 63) / 64;
    std::vector<uint64_t> aug((size_t)n2 * bw, 0);
    for (uint32_t i = 0; i < n2; ++i) {
        for (uint32_t j = 0; j < u; ++j)
            if (mu(i, j)) aug[(size_t)i * bw + (j >> 6)] |= 1ull << (j & 63);
        const uint32_t x = u + i;
        aug[(size_t)i * bw + (x >> 6)] |= 1ull << (x & 63);
    }
    auto abit = [&](uint32_t r, uint32_t x) { return (aug[(size_t)r * bw + (x >> 6)] >> (x & 63)) & 1; };
    std::vector<int32_t> pc_of_row(n2, -1);
    std::vector<uint8_t> is_pc(u, 0);
    for (uint32_t i = 0; i < n2; ++i) {
        int32_t jc = -1;
        for (uint32_t j = 0; j < u; ++j)
            if (!is_pc[j] && abit(i, j)) { jc = (int32_t)j; break; }
        if (jc < 0) { if (err) *err = "plan: singular GF(2) block"; return false; }
        pc_of_row[i] = jc;
        is_pc[jc] = 1;
        for (uint32_t q = 0; q < n2; ++q)
            if (q != i && abit(q, (uint32_t)jc))
                for (uint32_t x = 0; x < bw; ++x) aug[(size_t)q * bw + x] ^= aug[(size_t)i * bw + x];
    }
    std::vector<uint32_t> fcols;
    for (uint32_t j = 0; j < u; ++j)
        if (!is_pc[j]) fcols.push_back(j);
    if (fcols.size() != H) { if (err) *err = "plan: free column count != H"; return false; }
    const uint32_t tslot0 = tmp_base;          // t_i  (n2 slots)
    const uint32_t fslot0 = tmp_base + n2;     // C_F  (H slots)
    for (uint32_t i = 0; i < n2; ++i) {        // t_i = sum_j E2[i][j] b_j
        std::vector<uint32_t> s;
        for (uint32_t j = 0; j < n2; ++j)
            if (abit(i, u + j)) s.push_back(src_word(dslot[j]));
        bld.xor_words((uint16_t)(tslot0 + i), false, s);
    }
    // R[i][f] = aug[i][fcols[f]] (after reduction); Mh' and Z
    bld.phase = 5;
    std::vector<uint8_t> Z((size_t)H * H, 0);
    for (uint32_t h = 0; h < H; ++h) {
        const uint32_t hr = n2 + h;
        std::vector<uint32_t> s;
        for (uint32_t i = 0; i < n2; ++i) {
            const uint8_t c = mu(hr, (uint32_t)pc_of_row[i]);
            if (c) s.push_back(src_word(tslot0 + i, c));
        }
        for (uint32_t f = 0; f < H; ++f) {
            uint8_t z = mu(hr, fcols[f]);
            for (uint32_t i = 0; i < n2; ++i)
                if (abit(i, fcols[f])) z ^= mu(hr, (uint32_t)pc_of_row[i]);
            Z[(size_t)h * H + f] = z;
        }
        bld.mul_words(dslot[hr], true, s);
    }
    // Zinv by Gauss-Jordan over GF(256)
    std::vector<uint8_t> Zi((size_t)H * H, 0);
    for (uint32_t i = 0; i < H; ++i) Zi[(size_t)i * H + i] = 1;
    for (uint32_t c = 0; c < H; ++c) {
        uint32_t pr = H;
        for (uint32_t r = c; r < H; ++r)
            if (Z[(size_t)r * H + c]) { pr = r; break; }
        if (pr == H) { if (err) *err = "plan: singular HDPC block"; return false; }
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
    for (uint32_t f = 0; f < H; ++f) {         // C_F = Zinv bh'
        std::vector<uint32_t> s;
        for (uint32_t h = 0; h < H; ++h) {
            const uint8_t c = Zi[(size_t)f * H + h];
            if (c) s.push_back(src_word(dslot[n2 + h], c));
        }
        bld.mul_words((uint16_t)(fslot0 + f), false, s);
    }
    bld.phase = 6;
    for (uint32_t i = 0; i < n2; ++i) {        // C_P = t ^ R C_F
        std::vector<uint32_t> s;
        for (uint32_t f = 0; f < H; ++f)
            if (abit(i, fcols[f])) s.push_back(src_word(fslot0 + f));
        bld.xor_words((uint16_t)(tslot0 + i), true, s);
    }
    out->col_slot.assign(L, SLOT_NONE);
    for (uint32_t c = 0; c < L; ++c)
        if (cstate[c] == PIVOTED) out->col_slot[c] = (uint16_t)c;
    for (uint32_t i = 0; i < n2; ++i) out->col_slot[ucols[pc_of_row[i]]] = (uint16_t)(tslot0 + i);
    for (uint32_t f = 0; f < H; ++f) out->col_slot[ucols[fcols[f]]] = (uint16_t)(fslot0 + f);

    // ---------------- pass B: final C of pivoted columns ----------------
    // (i)  in place:  C_k = y_k ^ W_k C_U                       (depth 1 after the dense solve)
    // (ii) rebuild:   C_k = D_k ^ sum deps C_j ^ rowU C_U, with C_j inlined past the depth cap
    bld.phase = 7;
    constexpr uint32_t TU = 1u << 30;  // term for a U column (index into ucols)
    std::vector<std::vector<uint32_t>> fullB(npiv);
    std::vector<uint32_t> depB(npiv, 0);
    uint32_t n_inplace = 0, n_reload = 0;
    for (uint32_t k = 0; k < npiv; ++k) {
        std::vector<uint32_t> terms(deps[k]);
        for (uint32_t c : rowu[k]) terms.push_back(TU | (uint32_t)uidx[c]);
        std::sort(terms.begin(), terms.end());
        for (;;) {
            uint32_t dmax = 0, jmax = 0;
            for (uint32_t t : terms)
                if (!(t & (TG | TU)) && depB[t] + 1 > dmax) { dmax = depB[t] + 1; jmax = t; }
            if (dmax <= opt.depth_b) break;
            terms = symdiff(terms, std::vector<uint32_t>{jmax});
            terms = symdiff(terms, fullB[jmax]);
        }
        const bool lt = is_lt(k);
        if (lt) terms = symdiff(terms, std::vector<uint32_t>{TG | (piv_row[k] - S)});
        fullB[k] = terms;
        const uint64_t* wk = wrow(k);
        uint32_t wc = 0;
        for (uint32_t x = 0; x < nw; ++x) wc += (uint32_t)__builtin_popcountll(wk[x]);
        if (opt.passb_mode == 1 || wc <= terms.size()) {
            std::vector<uint32_t> s;
            for (uint32_t x = 0; x < nw; ++x) {
                uint64_t bits = wk[x];
                while (bits) {
                    const uint32_t j = x * 64 + (uint32_t)__builtin_ctzll(bits);
                    bits &= bits - 1;
                    s.push_back(src_word(out->col_slot[ucols[j]]));
                }
            }
            bld.xor_words((uint16_t)piv_col[k], true, s);
            depB[k] = 0;  // (i) rows hang directly off the dense solve
            ++n_inplace;
        } else {
            std::vector<uint32_t> s;
            uint32_t d = 0;
            for (uint32_t t : terms) {
                if (t & TG) s.push_back(t);
                else if (t & TU) s.push_back(src_word(out->col_slot[ucols[t & ~TU]]));
                else { s.push_back(src_word(piv_col[t])); d = std::max(d, depB[t] + 1); }
            }
            depB[k] = d;
            bld.xor_words((uint16_t)piv_col[k], false, s);
            ++n_reload;
        }
    }

    // ---------------- list scheduling into levels ----------------
    const uint32_t ns = (uint32_t)bld.stmts.size();
    std::vector<int32_t> last_w(out->n_slots, -1), last_r(out->n_slots, -1);
    std::vector<uint32_t> level(ns);
    std::vector<uint32_t> rd, wr;
    uint32_t nlev = 0;
    for (uint32_t i = 0; i < ns; ++i) {
        stmt_slots(bld.stmts[i], H, &rd, &wr);
        int32_t lv = 0;
        for (uint32_t x : rd) lv = std::max(lv, last_w[x] + 1);
        for (uint32_t x : wr) lv = std::max(lv, std::max(last_w[x], last_r[x]) + 1);
        level[i] = (uint32_t)lv;
        for (uint32_t x : rd) last_r[x] = std::max(last_r[x], lv);
        for (uint32_t x : wr) { last_w[x] = lv; last_r[x] = -1; }
        nlev = std::max(nlev, (uint32_t)lv + 1);
    }
    std::vector<uint32_t> order(ns);
    for (uint32_t i = 0; i < ns; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return level[a] < level[b]; });
    out->level_start.assign(nlev + 1, 0);
    for (uint32_t i = 0; i < ns; ++i) out->level_start[level[i] + 1]++;
    for (uint32_t l = 0; l < nlev; ++l) out->level_start[l + 1] += out->level_start[l];
    out->stmt_off.clear();
    out->words.clear();
    PlanStats& st = out->stats;
    st = PlanStats{};
    for (uint32_t oi = 0; oi < ns; ++oi) {
        const Stmt& s = bld.stmts[order[oi]];
        out->stmt_off.push_back((uint32_t)out->words.size());
        uint32_t nsrc = (uint32_t)s.src.size();
        if (s.type == ST_HORNER) nsrc -= s.extra;  // chunk length; tau words follow
        if (nsrc >= 4096) { if (err) *err = "plan: statement too long"; return false; }
        out->words.push_back((uint32_t)s.dst | (nsrc << 16) | (s.type << 28) | (s.acc ? ST_FLAG_ACC : 0u));
        if (s.type == ST_SCALE) out->words.push_back(s.extra);
        for (uint32_t w : s.src) out->words.push_back(w);
        if (s.type == ST_XOR) st.n_src_xor += nsrc;
        if (s.type == ST_MUL) st.n_src_mul += nsrc;
        if (s.type == ST_XOR)
            for (uint32_t w : s.src) st.n_reload += (w & SRC_GLOBAL) ? 1 : 0;
    }
    out->stmt_off.push_back((uint32_t)out->words.size());
    for (uint32_t i = 0; i < 8; ++i) st.phase_lo[i] = UINT32_MAX;
    for (uint32_t i = 0; i < ns; ++i) {
        const uint32_t ph = bld.stmts[i].phase;
        st.phase_lo[ph] = std::min(st.phase_lo[ph], level[i]);
        st.phase_hi[ph] = std::max(st.phase_hi[ph], level[i]);
        st.phase_n[ph]++;
    }
    st.n_stmts = ns;
    st.n_levels = nlev;
    st.u = u;
    st.inactivated = inactivated;
    st.n_pivots = npiv;
    st.n_slots = out->n_slots;
    st.horner_chunks = nq;
    st.passB_inplace = n_inplace;
    st.passB_reload = n_reload;
    for (uint32_t l = 0; l < nlev; ++l)
        st.max_level_width = std::max(st.max_level_width, out->level_start[l + 1] - out->level_start[l]);
    return true;
}

void encode_outputs(const Plan& plan, const uint32_t* isi, uint32_t n, std::vector<uint32_t>* words,
                    std::vector<uint32_t>* offs) {
    uint32_t cols[64];
    for (uint32_t i = 0; i < n; ++i) {
        const int nc = lt_cols(plan.p, isi[i], cols);
        // XOR semantics of encodeGen: a column listed twice cancels.
        std::sort(cols, cols + nc);
        uint32_t kept[64];
        int nk = 0;
        for (int j = 0; j < nc;) {
            int e = j;
            while (e < nc && cols[e] == cols[j]) ++e;
            if ((e - j) & 1) kept[nk++] = cols[j];
            j = e;
        }
        offs->push_back((uint32_t)words->size());
        words->push_back((uint32_t)nk);
        for (int j = 0; j < nk; ++j) words->push_back(plan.col_slot[kept[j]]);
    }
}

}  // namespace rq
