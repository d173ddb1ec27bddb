// rq_wave.cpp -- packs the level-scheduled plan into per-wave instruction streams in the format
// of rq_wave_format.hpp.
//
// Per level, the level's statements are paired (two of the same kind side by side in the two
// halves of a wave; HORNER chunks run alone), split into pieces of at most WV_MAX_PIECE groups
// (a continuation piece re-reads its own destination as a source: the wave's LDS accesses are
// ordered, so no barrier is needed between pieces), assigned to waves longest-first onto the
// least-loaded wave, and closed per wave with an END(BARRIER) group.
#include <algorithm>
#include <array>
#include <numeric>

#include "rq_plan.hpp"
#include "rq_wave_format.hpp"

namespace rq {
namespace {

struct SDesc {  // decoded statement
    uint32_t type = 0, dst = 0;
    bool acc = false;
    uint32_t g = WV_NO_ISI;          // single global source row (isi) or none
    std::vector<uint32_t> src;       // slots (XOR/MUL) or column words (HORNER)
    std::vector<uint32_t> coef;      // MUL coefficients
    std::vector<uint32_t> tau;       // HORNER tau words
};

bool decode_stmt(const Plan& pl, uint32_t s, SDesc* d, std::string* err) {
    const uint32_t* w = pl.words.data() + pl.stmt_off[s];
    const uint32_t w0 = w[0];
    d->dst = w0 & 0xFFFFu;
    const uint32_t ns = (w0 >> 16) & 0xFFFu;
    d->type = (w0 >> 28) & 7u;
    d->acc = (w0 >> 31) != 0;
    const uint32_t H = pl.p.H;
    if (d->type == ST_SCALE) {  // dst = c * dst: a MUL of dst by c that does not accumulate
        d->type = ST_MUL;
        d->acc = false;
        d->src.push_back(d->dst);
        d->coef.push_back(w[1] & 0xFFu);
        return true;
    }
    if (d->type == ST_HORNER) {
        for (uint32_t j = 0; j < ns; ++j) d->src.push_back(w[1 + j]);
        for (uint32_t j = 0; j < (H + 3) / 4; ++j) d->tau.push_back(w[1 + ns + j]);
        return true;
    }
    for (uint32_t k = 0; k < ns; ++k) {
        const uint32_t sw = w[1 + k];
        if (sw & SRC_GLOBAL) {
            if (d->g != WV_NO_ISI || d->type != ST_XOR) { if (err) *err = "wave: >1 global source"; return false; }
            d->g = sw & 0xFFFFFFu;
            continue;
        }
        d->src.push_back(sw & 0xFFFFu);
        d->coef.push_back((sw >> 16) & 0xFFu);
    }
    return true;
}

struct Ctx {
    uint32_t H, sd, zero, trash;
    uint32_t off(uint32_t slot) const { return slot * sd * 4; }  // LDS byte offset of a slot row
};

using Group = std::array<uint32_t, WV_GROUP>;
using Piece = std::vector<Group>;

// Accumulation as a source: the (slot, coef) list a half reads, dst first when it accumulates.
void sources_of(const SDesc& s, std::vector<uint32_t>* slot, std::vector<uint32_t>* coef) {
    slot->clear(); coef->clear();
    if (s.acc) { slot->push_back(s.dst); coef->push_back(1); }
    for (size_t k = 0; k < s.src.size(); ++k) { slot->push_back(s.src[k]); coef->push_back(s.type == ST_MUL ? s.coef[k] : 1); }
}

// XOR / MUL op pair -> pieces.  B may be null (half B writes the trash slot).
void emit_pair(const Ctx& c, const SDesc& A, const SDesc* B, std::vector<Piece>* pieces) {
    const bool mul = A.type == ST_MUL;
    std::vector<uint32_t> sa, ca, sb, cb;
    sources_of(A, &sa, &ca);
    if (B) sources_of(*B, &sb, &cb);
    const uint32_t dA = A.dst, dB = B ? B->dst : c.trash;
    const uint32_t gA = A.g, gB = B ? B->g : WV_NO_ISI;
    const bool hasG = gA != WV_NO_ISI || gB != WV_NO_ISI;
    // per piece: XOR up to 4 * (MAX_PIECE - 1) sources, MUL up to (MAX_PIECE - 1) / 2
    const size_t cap = mul ? (WV_MAX_PIECE - 1) / 2 : 4 * (WV_MAX_PIECE - 1);
    size_t ia = 0, ib = 0;
    bool first = true;
    do {
        // continuation pieces accumulate onto the destination written by the previous piece
        std::vector<uint32_t> pa, pca, pb, pcb;
        if (!first) { pa.push_back(dA); pca.push_back(1); pb.push_back(dB); pcb.push_back(1); }
        while (pa.size() < cap && ia < sa.size()) { pa.push_back(sa[ia]); pca.push_back(ca[ia]); ++ia; }
        while (pb.size() < cap && ib < sb.size()) { pb.push_back(sb[ib]); pcb.push_back(cb[ib]); ++ib; }
        const uint32_t n = (uint32_t)std::max(pa.size(), pb.size());
        const uint32_t ng = mul ? 2 * n : std::max<uint32_t>(1, (n + 3) / 4);  // >= 1 payload group
        const bool g = first && hasG;
        Piece pc;
        Group h{};
        const uint32_t hdr = (mul ? OP_MUL : OP_XOR) | (g ? FLAG_G : 0u) | (ng << 16);
        h[0] = hdr; h[1] = c.off(dA); h[2] = g ? gA : WV_NO_ISI;
        h[4] = hdr; h[5] = c.off(dB); h[6] = g ? gB : WV_NO_ISI;
        pc.push_back(h);
        if (mul) {
            for (uint32_t k = 0; k < n; ++k) {
                Group g1{}, g2{};
                for (int half = 0; half < 2; ++half) {
                    const auto& ps = half ? pb : pa;
                    const auto& pcf = half ? pcb : pca;
                    // a missing source multiplies the zero slot (adds nothing)
                    const uint32_t slot = k < ps.size() ? ps[k] : c.zero;
                    uint32_t t[5];
                    gf_perm_tables((uint8_t)(k < ps.size() ? pcf[k] : 0u), t);
                    const int o = 4 * half;
                    g1[o] = c.off(slot); g1[o + 1] = t[0]; g1[o + 2] = t[1]; g1[o + 3] = t[2];
                    g2[o] = t[3]; g2[o + 1] = t[4];
                }
                pc.push_back(g1);
                pc.push_back(g2);
            }
        } else {
            for (uint32_t q = 0; q < ng; ++q) {
                Group gs{};
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t k = 4 * q + j;
                    gs[j] = c.off(k < pa.size() ? pa[k] : c.zero);
                    gs[4 + j] = c.off(k < pb.size() ? pb[k] : c.zero);
                }
                pc.push_back(gs);
            }
        }
        pieces->push_back(std::move(pc));
        first = false;
    } while (ia < sa.size() || ib < sb.size());
}

void emit_horner(const Ctx& c, const SDesc& A, std::vector<Piece>* pieces) {
    // columns padded at the FRONT to a multiple of 8: while t is still 0 a zero column adds nothing
    std::vector<uint32_t> cols;
    const uint32_t n = (uint32_t)A.src.size();
    const uint32_t npad = (8 - n % 8) % 8;
    for (uint32_t k = 0; k < npad; ++k) cols.push_back(c.off(c.zero));
    for (uint32_t e : A.src) {
        const uint32_t s = e & 0xFFFFu;
        const uint32_t a = (e >> 16) & 31u, b = (e >> 21) & 31u;
        cols.push_back(c.off(s == SLOT_NONE ? c.zero : s) | (a << 18) | (b << 22));
    }
    const uint32_t ngc = (uint32_t)cols.size() / 8;
    const uint32_t per = WV_MAX_PIECE - 2;  // header + column groups + (finish) tau group
    for (uint32_t g0 = 0; g0 < ngc || g0 == 0; g0 += per) {
        const uint32_t g1 = std::min(ngc, g0 + per);
        const bool start = g0 == 0, finish = g1 == ngc;
        Piece pc;
        Group h{};
        const uint32_t hdr = OP_HORNER | (start ? FLAG_HSTART : 0u) | (finish ? FLAG_HFINISH : 0u) | ((g1 - g0) << 16);
        h[0] = hdr; h[1] = c.off(A.dst); h[2] = WV_NO_ISI;
        h[4] = hdr; h[5] = c.off(c.trash); h[6] = WV_NO_ISI;
        pc.push_back(h);
        for (uint32_t q = g0; q < g1; ++q) {
            Group gc{};
            for (uint32_t j = 0; j < 8; ++j) gc[j] = cols[8 * q + j];
            pc.push_back(gc);
        }
        if (finish) {
            Group gt{};
            for (uint32_t j = 0; j < A.tau.size() && j < 4; ++j) gt[j] = gt[4 + j] = A.tau[j];
            pc.push_back(gt);
        }
        pieces->push_back(std::move(pc));
        if (ngc == 0) break;
    }
}

uint64_t piece_cost(const Piece& p) {  // rough issue cost for load balancing
    const uint32_t ty = p[0][0] & 7u, ng = (uint32_t)p.size() - 1;
    if (ty == OP_XOR) return 14 + 12 * (uint64_t)ng + ((p[0][0] & FLAG_G) ? 8 : 0);
    if (ty == OP_MUL) return 14 + 14 * (uint64_t)ng;
    return 14 + 80 * (uint64_t)ng;  // HORNER: 8 columns per group
}

}  // namespace

bool build_wave_program(const Plan& pl, uint32_t n_waves, uint32_t sd, WaveProgram* out, std::string* err) {
    if (sd == 0) { if (err) *err = "wave: strip width must be > 0"; return false; }
    const uint32_t H = pl.p.H;
    Ctx c;
    c.H = H; c.sd = sd; c.zero = pl.n_slots; c.trash = pl.n_slots + 1;
    out->n_waves = n_waves;
    out->n_levels = (uint32_t)pl.level_start.size() - 1;
    out->zero_slot = c.zero;
    out->trash_slot = c.trash;
    out->n_slots = pl.n_slots + 1 + std::max<uint32_t>(H, 1);  // + zero slot + H trash slots
    if ((uint64_t)out->n_slots * sd * 4 >= (1u << 18)) {
        if (err) *err = "wave: slot image too large for 18-bit byte offsets";
        return false;
    }
    out->sd = sd;
    std::vector<std::vector<Group>> stream(n_waves);  // per wave: groups (pages of WV_GPP)
    auto end_group = [](uint32_t flags) {
        Group e{};
        e[0] = e[4] = OP_END | flags;
        return e;
    };
    auto place = [&](std::vector<Group>& s, const Piece& pc) {  // append a piece, never across a page
        const size_t used = s.size() % WV_GPP;
        if (used + pc.size() + 1 > WV_GPP) {  // no room for the piece and a closing END
            s.push_back(end_group(FLAG_ADVANCE));
            while (s.size() % WV_GPP) s.push_back(Group{});
        }
        s.insert(s.end(), pc.begin(), pc.end());
    };
    for (uint32_t lv = 0; lv < out->n_levels; ++lv) {
        std::vector<SDesc> st;
        for (uint32_t s = pl.level_start[lv]; s < pl.level_start[lv + 1]; ++s) {
            SDesc d;
            if (!decode_stmt(pl, s, &d, err)) return false;
            st.push_back(std::move(d));
        }
        std::stable_sort(st.begin(), st.end(), [](const SDesc& a, const SDesc& b) {
            return a.type != b.type ? a.type < b.type : a.src.size() + a.acc > b.src.size() + b.acc;
        });
        std::vector<std::vector<Piece>> groups;  // op (pair) -> its pieces
        std::vector<uint64_t> cost;
        for (size_t i = 0; i < st.size();) {
            std::vector<Piece> pieces;
            size_t used = 1;
            if (st[i].type == ST_HORNER) {
                emit_horner(c, st[i], &pieces);
            } else {
                const bool pair = i + 1 < st.size() && st[i + 1].type == st[i].type;
                emit_pair(c, st[i], pair ? &st[i + 1] : nullptr, &pieces);
                used = pair ? 2 : 1;
            }
            uint64_t k = 0;
            for (const Piece& p : pieces) k += piece_cost(p);
            cost.push_back(k);
            groups.push_back(std::move(pieces));
            i += used;
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
            for (uint32_t o : mine[w])
                for (const Piece& pc : groups[o]) place(stream[w], pc);
            // close the level; an END in a page's last group also moves to the next page
            auto& s = stream[w];
            const bool last_in_page = s.size() % WV_GPP == WV_GPP - 1;
            s.push_back(end_group(FLAG_BARRIER | (last_in_page ? FLAG_ADVANCE : 0u)));
        }
    }
    out->words.clear();
    out->wave_off.clear();
    out->max_stream = 0;
    for (uint32_t w = 0; w < n_waves; ++w) {
        auto& s = stream[w];
        while (s.size() % WV_GPP) s.push_back(Group{});
        out->wave_off.push_back((uint32_t)out->words.size());
        for (const Group& g : s) out->words.insert(out->words.end(), g.begin(), g.end());
        out->max_stream = std::max<uint32_t>(out->max_stream, (uint32_t)(s.size() * WV_GROUP));
    }
    out->words.resize(out->words.size() + 3 * WV_PAGE, 0);  // the kernel stages pages ahead
    return true;
}

}  // namespace rq
