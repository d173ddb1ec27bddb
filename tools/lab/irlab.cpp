// IR live-set analysis (host-only experiment tool): builds the column program IR for (K, R repairs)
// and reports node counts, the live-value profile over program order, what the values live at the
// peak are waiting for, and the forward pass's live set in pull vs push form.
// g++ -O2 -std=c++17 -I rl-quic-raptor_amd/csrc tools/lab/irlab.cpp -o /tmp/irlab && /tmp/irlab 1024 76
#include "../../rl-quic-raptor_amd/csrc/rq_colprog.cpp"
#include <cstdio>
namespace rq { const GF& gf() { static const GF g; return g; } }
using namespace rq;
void classify(const ColIR& ir, uint32_t at);
int main(int argc, char** argv) {
    uint32_t K = argc > 1 ? atoi(argv[1]) : 1024, R = argc > 2 ? atoi(argv[2]) : 76;
    Params p; params_for_K(K, &p);
    std::vector<uint32_t> esi; for (uint32_t i = 0; i < R; ++i) esi.push_back(K + i);
    ColIR ir; std::string err;
    if (!build_colprog(p, esi.data(), R, &ir, &err)) { printf("err %s\n", err.c_str()); return 1; }
    const uint32_t n = ir.nodes.size();
    std::vector<uint32_t> last(n, 0);
    for (uint32_t i = 0; i < n; ++i) for (uint32_t x : {ir.nodes[i].a, ir.nodes[i].b, ir.nodes[i].c}) if (x != NOVAL) last[x] = i;
    uint32_t live = 0, peak = 0, peak_at = 0; std::vector<int> delta(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) if (ir.nodes[i].k != IR_STORE && last[i] > i) { delta[i]++; delta[last[i]]--; }
    std::vector<uint32_t> prof(n);
    for (uint32_t i = 0; i < n; ++i) { live += delta[i]; prof[i] = live; if (live > peak) { peak = live; peak_at = i; } }
    printf("K=%u nodes=%u loads=%u xor2=%u xor3=%u xt=%u xtx=%u u=%u npiv=%u n2=%u phases %u %u %u %u\n", K, n, ir.st.load, ir.st.xor2, ir.st.xor3, ir.st.xt, ir.st.xtx, ir.st.u, ir.st.npiv, ir.st.n2,
           ir.phase_start[0], ir.phase_start[1], ir.phase_start[2], ir.phase_start[3]);
    printf("peak live %u at node %u\n", peak, peak_at);
    for (uint32_t q = 0; q < 20; ++q) printf(" %u", prof[(size_t)n * q / 20]); printf("\n");
    void fwd_study(const Params&); fwd_study(p); classify(ir, peak_at); classify(ir, n/5); classify(ir, 3*n/5);
    // sum of lifetimes
    double sl = 0; for (uint32_t i = 0; i < n; ++i) if (last[i] > i) sl += last[i] - i; printf("mean live %.1f\n", sl / n);
}
// classify live values at a node
void classify(const ColIR& ir, uint32_t at) {
    const uint32_t n = ir.nodes.size();
    std::vector<std::vector<uint32_t>> uses(n);
    for (uint32_t i = 0; i < n; ++i) for (uint32_t x : {ir.nodes[i].a, ir.nodes[i].b, ir.nodes[i].c}) if (x != NOVAL) uses[x].push_back(i);
    int c_load = 0, c_hornonly = 0, c_horn_and_more = 0, c_nohorn = 0, c_acc = 0;
    double span_next = 0, span_last = 0; int cnt = 0;
    for (uint32_t v = 0; v < at; ++v) {
        if (ir.nodes[v].k == IR_STORE) continue;
        std::vector<uint32_t> rem; for (uint32_t u : uses[v]) if (u >= at) rem.push_back(u);
        if (rem.empty()) continue;
        cnt++; span_next += rem.front() - at; span_last += rem.back() - at;
        bool horn = false; int other = 0;
        for (uint32_t u : rem) { if (ir.nodes[u].k == IR_XTX && ir.nodes[u].b == v) horn = true; else other++; }
        if (ir.nodes[v].k == IR_LOAD) c_load++;
        else if (horn && !other) c_hornonly++;
        else if (horn) c_horn_and_more++;
        else if (rem.size() == 1) c_acc++;
        else c_nohorn++;
    }
    printf("at %u live %d: load %d, horner-only %d, horner+other %d, single-use %d, multi-use-nonhorner %d; mean next %.0f last %.0f\n",
        at, cnt, c_load, c_hornonly, c_horn_and_more, c_acc, c_nohorn, span_next/cnt, span_last/cnt);
}
// forward pass only, peeling order: pull vs push live sets
void fwd_study(const Params& p) {
    Elim e; std::string err; eliminate(p, &e, &err);
    const uint32_t n = e.piv_col.size();
    // pull: y_j live from j to last dependent
    std::vector<uint32_t> lastdep(n, 0);
    for (uint32_t k = 0; k < n; ++k) for (uint32_t j : e.deps[k]) lastdep[j] = std::max(lastdep[j], k);
    std::vector<int> d(n + 2, 0);
    for (uint32_t j = 0; j < n; ++j) if (lastdep[j] > j) { d[j]++; d[lastdep[j]]--; }
    int live = 0, peak = 0; for (uint32_t k = 0; k < n; ++k) { live += d[k]; peak = std::max(peak, live); }
    // push: accumulator of k live from first dep (min j) to k
    std::vector<int> d2(n + 2, 0);
    for (uint32_t k = 0; k < n; ++k) if (!e.deps[k].empty()) { uint32_t m = *std::min_element(e.deps[k].begin(), e.deps[k].end()); d2[m]++; d2[k]--; }
    int live2 = 0, peak2 = 0; for (uint32_t k = 0; k < n; ++k) { live2 += d2[k]; peak2 = std::max(peak2, live2); }
    // column order correlation: position in peeling vs column
    double edges = 0; for (auto& v : e.deps) edges += v.size();
    printf("fwd: npiv %u edges %.0f  pull peak %d  push peak %d\n", n, edges, peak, peak2);
}
