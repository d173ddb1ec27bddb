// rq_wave.cpp -- packs the level-scheduled plan into per-wave instruction streams
// (see WaveProgram in rq_plan.hpp).
//
// Stream layout per wave: a sequence of 64-word pages.  A page holds one or more *segments*;
// no segment crosses a page.  Segment = [op count] [ops...] [NEXT], NEXT bit0 = a workgroup
// barrier follows (end of a dependency level), bit1 = the next segment starts on the next page.
// The kernel keeps the current page and the next one in VGPRs (prefetched at the previous page
// switch) and reads words with v_readlane, so inside a segment descriptor reads never wait on
// memory.  Ops longer than a segment are split into continuation pieces executed by the same
// wave in order (LDS accesses of one wave are ordered, so no barrier is needed between pieces).
#include <algorithm>
#include <numeric>

#include "rq_plan.hpp"

namespace rq {
namespace {

constexpr uint32_t PAGE = 64;
constexpr uint32_t MAX_PIECE = PAGE - 2;  // op words that fit a segment with its count + NEXT

struct SDesc {  // decoded statement
    uint32_t type = 0, dst = 0, n = 0;
    bool acc = false;
    uint32_t g = 0xFFFFFFFFu;       // single global source row (isi) or none
    std::vector<uint32_t> src;      // slots (XOR/MUL) or column words (HORNER)
    std::vector<uint32_t> coef;     // MUL coefs / SCALE coef
    std::vector<uint32_t> tau;      // HORNER tau words
};

bool decode_stmt(const Plan& pl, uint32_t s, SDesc* d, std::string* err) {
    const uint32_t* w = pl.words.data() + pl.stmt_off[s];
    const uint32_t w0 = w[0];
    d->dst = w0 & 0xFFFFu;
    const uint32_t ns = (w0 >> 16) & 0xFFFu;
    d->type = (w0 >> 28) & 7u;
    d->acc = (w0 >> 31) != 0;
    const uint32_t H = pl.p.H;
    if (d->type == ST_SCALE) { d->coef.push_back(w[1]); d->n = 0; return true; }
    if (d->type == ST_HORNER) {
        for (uint32_t j = 0; j < ns; ++j) d->src.push_back(w[1 + j]);
        for (uint32_t j = 0; j < (H + 3) / 4; ++j) d->tau.push_back(w[1 + ns + j]);
        d->n = ns;
        return true;
    }
    for (uint32_t k = 0; k < ns; ++k) {
        const uint32_t sw = w[1 + k];
        if (sw & SRC_GLOBAL) {
            if (d->g != 0xFFFFFFFFu || d->type != ST_XOR) { if (err) *err = "wave: >1 global source"; return false; }
            d->g = sw & 0xFFFFFFu;
            continue;
        }
        d->src.push_back(sw & 0xFFFFu);
        d->coef.push_back((sw >> 16) & 0xFFu);
    }
    d->n = (uint32_t)d->src.size();
    return true;
}

// Emit the op pair (A, B) as one or more pieces of <= MAX_PIECE words.
void emit_pair(const SDesc& A, const SDesc* Bp, uint32_t H, uint32_t zero, uint32_t trash, uint32_t sd,
               std::vector<std::vector<uint32_t>>* pieces) {
    auto O = [sd](uint32_t slot) { return sd ? slot * sd : slot; };  // LDS dword offset (sd > 0)
    const SDesc nop;
    const SDesc& B = Bp ? *Bp : nop;
    const bool pair = Bp != nullptr;
    const uint32_t n = std::max(A.n, pair ? B.n : 0u);
    const uint32_t dstw = O(A.dst) | (O(pair ? B.dst : trash) << 16);
    const uint32_t nt = (H + 3) / 4;
    if (A.type == ST_SCALE) {
        pieces->push_back({A.type, dstw, A.coef[0] | ((pair ? B.coef[0] : 0u) << 8)});
        return;
    }
    if (A.type == ST_HORNER) {
        // columns padded at the front of the shorter chunk (t stays 0 there: scatters nothing)
        std::vector<uint32_t> cols;
        const uint32_t pad_col = 0xFFFFu;
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t ka = n - A.n, kb = n - (pair ? B.n : 0);
            auto col = [&](uint32_t e) {  // column word: slot field -> offset (NONE stays NONE)
                const uint32_t s = e & 0xFFFFu;
                return s == 0xFFFFu ? e : ((e & ~0xFFFFu) | O(s));
            };
            cols.push_back(k >= ka ? col(A.src[k - ka]) : pad_col);
            cols.push_back((pair && k >= kb) ? col(B.src[k - kb]) : pad_col);
        }
        const uint32_t per = (MAX_PIECE - 2 - 2 * nt) / 2;  // columns per piece
        for (uint32_t c0 = 0; c0 < n || c0 == 0; c0 += per) {
            const uint32_t c1 = std::min(n, c0 + per);
            const bool start = c0 == 0, finish = c1 == n;
            std::vector<uint32_t> op;
            op.push_back(A.type | (start ? 64u : 0u) | (finish ? 128u : 0u) | ((c1 - c0) << 16));
            op.push_back(dstw);
            op.insert(op.end(), cols.begin() + 2 * c0, cols.begin() + 2 * c1);
            if (finish) {
                for (uint32_t j = 0; j < nt; ++j) op.push_back(A.tau[j]);
                for (uint32_t j = 0; j < nt; ++j) op.push_back(pair ? B.tau[j] : 0u);
            }
            pieces->push_back(std::move(op));
            if (n == 0) break;
        }
        return;
    }
    // XOR / MUL
    const bool mul = A.type == ST_MUL;
    const bool hasG = A.g != 0xFFFFFFFFu || (pair && B.g != 0xFFFFFFFFu);
    const uint32_t wps = mul ? 2 : 1;
    uint32_t k0 = 0;
    bool first = true;
    do {
        const uint32_t room = MAX_PIECE - 2 - (first && hasG ? 2 : 0);
        const uint32_t k1 = std::min(n, k0 + room / wps);
        std::vector<uint32_t> op;
        const uint32_t accA = first ? (A.acc ? 8u : 0u) : 8u;
        const uint32_t accB = first ? ((pair && B.acc) ? 16u : 0u) : 16u;
        const bool g = first && hasG;
        op.push_back(A.type | accA | accB | (g ? 32u : 0u) | ((k1 - k0) << 16));
        op.push_back(dstw);
        if (g) { op.push_back(A.g); op.push_back(pair ? B.g : 0xFFFFFFFFu); }
        for (uint32_t k = k0; k < k1; ++k) {
            const uint32_t sa = O(k < A.n ? A.src[k] : zero);
            const uint32_t sb = O((pair && k < B.n) ? B.src[k] : zero);
            op.push_back(sa | (sb << 16));
            if (mul) {
                const uint32_t ca = k < A.n ? A.coef[k] : 0;
                const uint32_t cb = (pair && k < B.n) ? B.coef[k] : 0;
                op.push_back(ca | (cb << 8));
            }
        }
        pieces->push_back(std::move(op));
        k0 = k1;
        first = false;
    } while (k0 < n);
}

}  // namespace

bool build_wave_program(const Plan& pl, uint32_t n_waves, uint32_t sd, WaveProgram* out, std::string* err) {
    const uint32_t H = pl.p.H;
    const uint32_t zero = pl.n_slots, trash = pl.n_slots + 1;
    out->n_waves = n_waves;
    out->n_levels = (uint32_t)pl.level_start.size() - 1;
    out->zero_slot = zero;
    out->trash_slot = trash;
    out->n_slots = pl.n_slots + 1 + std::max<uint32_t>(H, 1);
    if (out->n_slots >= 0x8000u || (sd && (uint64_t)out->n_slots * sd >= 0xFFFFu)) {
        if (err) *err = "wave: slot image too large for 16-bit offsets";
        return false;
    }
    out->sd = sd;
    // per wave: list of segments (word vectors, each <= PAGE words incl. count and NEXT)
    std::vector<std::vector<std::vector<uint32_t>>> segs(n_waves);
    for (uint32_t lv = 0; lv < out->n_levels; ++lv) {
        std::vector<SDesc> st;
        for (uint32_t s = pl.level_start[lv]; s < pl.level_start[lv + 1]; ++s) {
            SDesc d;
            if (!decode_stmt(pl, s, &d, err)) return false;
            st.push_back(std::move(d));
        }
        std::stable_sort(st.begin(), st.end(), [](const SDesc& a, const SDesc& b) {
            return a.type != b.type ? a.type < b.type : a.n > b.n;
        });
        std::vector<std::vector<std::vector<uint32_t>>> groups;  // op pair -> its pieces
        std::vector<uint64_t> cost;
        for (size_t i = 0; i < st.size();) {
            const bool pair = i + 1 < st.size() && st[i + 1].type == st[i].type;
            std::vector<std::vector<uint32_t>> pieces;
            emit_pair(st[i], pair ? &st[i + 1] : nullptr, H, zero, trash, sd, &pieces);
            const uint32_t n = std::max(st[i].n, pair ? st[i + 1].n : 0u);
            cost.push_back(2 + (st[i].type == ST_HORNER ? 4 * n : n));
            groups.push_back(std::move(pieces));
            i += pair ? 2 : 1;
        }
        std::vector<uint32_t> order(groups.size());
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
        std::vector<uint64_t> load(n_waves, 0);
        std::vector<std::vector<uint32_t>> mine(n_waves);
        for (uint32_t o : order) {
            const uint32_t w = (uint32_t)(std::min_element(load.begin(), load.end()) - load.begin());
            load[w] += cost[o];
            mine[w].push_back(o);
        }
        for (uint32_t w = 0; w < n_waves; ++w) {
            std::vector<uint32_t> cur{0};  // count word
            auto close = [&](bool barrier) {
                cur.push_back(barrier ? 1u : 0u);  // NEXT (advance bit set during packing)
                segs[w].push_back(std::move(cur));
                cur.assign(1, 0);
            };
            for (uint32_t o : mine[w])
                for (auto& pc : groups[o]) {
                    if (cur.size() + pc.size() + 1 > PAGE) close(false);
                    cur.insert(cur.end(), pc.begin(), pc.end());
                    cur[0]++;
                }
            close(true);
        }
    }
    // pack segments into pages
    out->words.clear();
    out->wave_off.clear();
    out->max_stream = 0;
    for (uint32_t w = 0; w < n_waves; ++w) {
        std::vector<uint32_t> s;
        size_t prev_next = SIZE_MAX;  // index of the previous segment's NEXT word
        for (auto& sg : segs[w]) {
            const size_t used = s.size() % PAGE;
            if (used != 0 && used + sg.size() > PAGE) {
                s.resize(s.size() + (PAGE - used), 0);
                if (prev_next != SIZE_MAX) s[prev_next] |= 2u;
            }
            s.insert(s.end(), sg.begin(), sg.end());
            prev_next = s.size() - 1;
            if (s.size() % PAGE == 0) s[prev_next] |= 2u;  // page exactly full: next segment moves on
        }
        s.resize((s.size() + PAGE - 1) / PAGE * PAGE, 0);
        out->wave_off.push_back((uint32_t)out->words.size());
        out->words.insert(out->words.end(), s.begin(), s.end());
        out->max_stream = std::max<uint32_t>(out->max_stream, (uint32_t)s.size());
    }
    out->words.resize(out->words.size() + 2 * PAGE, 0);  // the kernel prefetches one page ahead
    return true;
}

}  // namespace rq
