// rq_engine.cpp -- host runtime of librqhip.so: device contexts, per-K' plan cache, the
// batched device-resident encode/decode entry points, and the per-object Encoder/Decoder API
// that mirrors xssnick/raptorq as wrapped by go/fec/raptorq_wrap.go.
//
// There is no CPU fallback: every symbol the engine returns is computed by the HIP kernels in
// rq_kernels.hip; without a usable gfx950 device the calls fail with RQ_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rqhip.h"
#include "rq_colasm.hpp"
#include "rq_colprog.hpp"
#include "rq_device.hpp"
#include "rq_plan.hpp"

namespace rq {
namespace {

thread_local std::string g_err;
thread_local int g_device = -1;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(RQ_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// Growable device buffer (allocation happens outside any timed/captured region after warmup).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return RQ_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(n, 4096);
        if (hipMalloc(&p, want) != hipSuccess) return fail(RQ_ERR_DEVICE, "hipMalloc failed");
        cap = want;
        return RQ_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

// Waves per k_encode workgroup (16, or 8; rq_kernels.hip instantiates both).  RQHIP_WAVES
// overrides the default for experiments; it is read once per process.
uint32_t enc_waves() {
    static const uint32_t nw = [] {
        const char* e = std::getenv("RQHIP_WAVES");
        const uint32_t v = e ? (uint32_t)std::atoi(e) : 16u;
        return (v == 8u) ? 8u : 16u;
    }();
    return nw;
}

struct DevWave {  // the wave program for one strip width (slot fields are LDS dword offsets)
    WaveProgram wp;
    DevBuf wstream, wave_off;
};

struct DevPlan {
    Plan host;
    uint32_t n_slots = 0;  // slot image rows: plan slots + zero slot + H trash slots
    std::map<uint32_t, std::unique_ptr<DevWave>> waves;  // keyed by strip width sd
    DevBuf load_slot, col_slot;
    DevBuf cid;            // A^-1 restricted to source columns (decode), L x cid_stride bytes
    uint32_t cid_stride = 0;
    bool cid_ready = false;
};

// A compiled column program (rq_colprog.hpp / rq_colasm.hpp) loaded on one device.
struct ColKernel {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    Params p{};
    std::vector<uint32_t> esi;     // outputs (empty: all L intermediate symbols)
    uint32_t n_out = 0, n_slots = 0;
    MProg::Stats st{};
    uint32_t n_ins = 0;
    ~ColKernel() { if (mod) (void)hipModuleUnload(mod); }
};

struct DevCtx {
    int device = -1;
    std::mutex mu;
    bool tables = false;
    std::map<uint32_t, std::unique_ptr<DevPlan>> plans;  // keyed by K'
    std::map<std::string, std::unique_ptr<ColKernel>> colk;  // keyed by (K', K, outputs)
    DevBuf ws_idx, ws_sigma, ws_x, ws_xp, ws_status, ws_esi, ws_scratch;
};

std::mutex g_ctx_mu;
std::map<int, std::unique_ptr<DevCtx>> g_ctx;
std::mutex g_hplan_mu;
std::map<uint32_t, std::unique_ptr<Plan>> g_hplans;  // host-only plans (tests, stats)

int current_device(int* dev) {
    if (g_device < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RQ_ERR_DEVICE, "no HIP device available");
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) d = 0;
        g_device = d;
    }
    *dev = g_device;
    return RQ_OK;
}

int get_ctx(DevCtx** out) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(dev));
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto& c = g_ctx[dev];
    if (!c) {
        c.reset(new DevCtx());
        c->device = dev;
    }
    *out = c.get();
    return RQ_OK;
}

// Plan options; RQHIP_PASSB / RQHIP_DEPTH_B override the pass-B strategy for experiments.
const PlanOptions& plan_options() {
    static const PlanOptions o = [] {
        PlanOptions r;
        if (const char* e = std::getenv("RQHIP_PASSB")) r.passb_mode = (uint32_t)std::atoi(e);
        if (const char* e = std::getenv("RQHIP_DEPTH_B")) r.depth_b = (uint32_t)std::atoi(e);
        return r;
    }();
    return o;
}

int host_plan(uint32_t K, const Plan** out) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    std::lock_guard<std::mutex> lk(g_hplan_mu);
    auto& pl = g_hplans[p.Kp];
    if (!pl) {
        std::unique_ptr<Plan> np(new Plan());
        std::string err;
        if (!compile_encode_plan(p, np.get(), &err, plan_options())) return fail(RQ_ERR_PLAN, err);
        pl = std::move(np);
    }
    *out = pl.get();
    return RQ_OK;
}

template <class T>
int upload(DevBuf& b, const std::vector<T>& v) {
    int rc = b.ensure(v.size() * sizeof(T));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return RQ_OK;
}

// Caller holds ctx->mu.
int get_dev_plan(DevCtx* ctx, const Params& p, DevPlan** out) {
    if (!ctx->tables) {
        const int e = upload_tables();
        if (e) return fail(RQ_ERR_DEVICE, "upload_tables failed");
        ctx->tables = true;
    }
    auto& dp = ctx->plans[p.Kp];
    if (!dp) {
        const Plan* hp;
        int rc = host_plan(p.K, &hp);
        if (rc) return rc;
        std::unique_ptr<DevPlan> n(new DevPlan());
        n->host = *hp;
        n->n_slots = n->host.n_slots + 1 + std::max<uint32_t>(n->host.p.H, 1);
        if ((rc = upload(n->load_slot, n->host.load_slot))) return rc;
        if ((rc = upload(n->col_slot, n->host.col_slot))) return rc;
        dp = std::move(n);
    }
    *out = dp.get();
    return RQ_OK;
}

DevParams dev_params(const Params& p) {
    DevParams d;
    d.K = p.K; d.Kp = p.Kp; d.J = p.J; d.S = p.S; d.H = p.H; d.W = p.W; d.L = p.L; d.P = p.P; d.P1 = p.P1;
    return d;
}

int get_dev_wave(DevPlan* dp, uint32_t sd, DevWave** out) {
    auto& dw = dp->waves[sd];
    if (!dw) {
        std::unique_ptr<DevWave> n(new DevWave());
        std::string err;
        if (!build_wave_program(dp->host, enc_waves(), sd, &n->wp, &err)) return fail(RQ_ERR_PLAN, err);
        int rc;
        if ((rc = upload(n->wstream, n->wp.words))) return rc;
        if ((rc = upload(n->wave_off, n->wp.wave_off))) return rc;
        dw = std::move(n);
    }
    *out = dw.get();
    return RQ_OK;
}

// Strip geometry: the widest strip (<= 32 dwords) whose n_slots x sd image fits the LDS.
struct Geometry {
    uint32_t sd, n_strips, group;
};
int geometry(const DevPlan& dp, uint32_t T, uint32_t K, bool erasures, Geometry* g) {
    const uint32_t Td = T / 4;
    // - stream ring / tuple staging, erasure bitmap, 16-byte alignment of the ring
    const size_t ring = std::max<size_t>((size_t)enc_waves() * 2 * 64, 128 * 6) * 4;
    const size_t budget = 160 * 1024 - ring - 16 - (erasures ? ((K + 31) / 32) * 4 : 0);
    const size_t per_dword = (size_t)dp.n_slots * 4;
    // RQHIP_SD_MAX caps the strip width (narrower strips -> several workgroups per CU); experiments
    static const uint32_t sd_cap = [] {
        const char* e = std::getenv("RQHIP_SD_MAX");
        const uint32_t v = e ? (uint32_t)std::atoi(e) : 32u;
        return v ? std::min<uint32_t>(v, 32u) : 32u;
    }();
    uint32_t sd_max = (uint32_t)std::min<size_t>(sd_cap, budget / per_dword);
    if (sd_max == 0) return fail(RQ_ERR_UNSUPPORTED, "K' too large for the LDS-resident plan (n_slots=" +
                                                         std::to_string(dp.n_slots) + ")");
    g->n_strips = (Td + sd_max - 1) / sd_max;
    g->sd = (Td + g->n_strips - 1) / g->n_strips;
    g->group = 8;
    while (g->group < g->sd) g->group <<= 1;
    return RQ_OK;
}

EncArgs base_args(const DevPlan& dp, const DevWave& dw, const Params& p, uint32_t T, uint32_t sd) {
    EncArgs a;
    std::memset(&a, 0, sizeof a);
    a.p = dev_params(p);
    a.T = T;
    a.n_slots = dw.wp.n_slots;
    a.sd = sd;
    a.n_levels = dw.wp.n_levels;
    a.load_slot = dp.load_slot.as<uint16_t>();
    a.wstream = dw.wstream.as<uint32_t>();
    a.wave_off = dw.wave_off.as<uint32_t>();
    a.n_waves = dw.wp.n_waves;
    a.col_slot = dp.col_slot.as<uint16_t>();
    static const uint32_t dbg = [] {  // timing ablations only (tools/ablate.py)
        const char* s = std::getenv("RQHIP_DBG");
        return s ? (uint32_t)std::strtoul(s, nullptr, 0) : 0u;
    }();
    a.dbg = dbg;
    return a;
}

// Encode `n_blocks` blocks already on the device.  Caller holds ctx->mu.
int encode_locked(DevCtx* ctx, const Params& p, uint32_t T, uint32_t n_blocks, const void* src, uint64_t src_stride,
                  uint32_t n_esi, const uint32_t* d_esi, void* out, uint64_t out_stride, void* c_out,
                  uint64_t c_stride, void* stream) {
    DevPlan* dp;
    int rc = get_dev_plan(ctx, p, &dp);
    if (rc) return rc;
    Geometry g;
    if ((rc = geometry(*dp, T, p.K, false, &g))) return rc;
    DevWave* dw;
    if ((rc = get_dev_wave(dp, g.sd, &dw))) return rc;
    EncArgs a = base_args(*dp, *dw, p, T, g.sd);
    a.src = static_cast<const uint8_t*>(src);
    a.src_stride = src_stride;
    a.out_esi = d_esi;
    a.n_out = n_esi;
    a.out = static_cast<uint8_t*>(out);
    a.out_stride = out_stride;
    a.c_out = static_cast<uint8_t*>(c_out);
    a.c_stride = c_stride;
    static const char* stamp_file = std::getenv("RQHIP_STAMP_FILE");  // diagnostics only
    DevBuf stamps;
    if (stamp_file && stamps.ensure((size_t)a.n_levels * a.n_waves * 16) == RQ_OK) a.stamp = stamps.as<unsigned long long>();
    const int e = launch_encode(a, g.n_strips, n_blocks, g.group, stream);
    if (e) return fail(RQ_ERR_DEVICE, std::string("k_encode launch: ") + hipGetErrorString((hipError_t)e));
    if (a.stamp) {
        std::vector<unsigned long long> h((size_t)a.n_levels * a.n_waves * 2);
        if (hipStreamSynchronize((hipStream_t)stream) == hipSuccess &&
            hipMemcpy(h.data(), a.stamp, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE* f = std::fopen(stamp_file, "w")) {
                for (uint32_t l = 0; l < a.n_levels; ++l) {
                    std::fprintf(f, "%u", l);
                    for (uint32_t w = 0; w < a.n_waves; ++w)
                        std::fprintf(f, " %llu:%llu", h[((size_t)l * a.n_waves + w) * 2], h[((size_t)l * a.n_waves + w) * 2 + 1]);
                    std::fprintf(f, "\n");
                }
                std::fclose(f);
            }
        }
    }
    return RQ_OK;
}

// ---------------- column programs (the encode hot path) ----------------
// Compile (once per device and (K', K, outputs)) the straight-line gfx950 program for the given
// outputs: IR (rq_colprog.cpp) -> registers/scratch (rq_colasm.cpp) -> assembly -> code object
// (amd_comgr, in process) -> hipModuleLoadData.  Caller holds ctx->mu.
int get_col_kernel(DevCtx* ctx, const Params& p, const uint32_t* esi, uint32_t n_esi, bool all_C, ColKernel** out) {
    std::string key = std::to_string(p.Kp) + ":" + std::to_string(p.K) + (all_C ? ":C" : ":E");
    if (!all_C) {
        key.reserve(key.size() + n_esi * 6);
        for (uint32_t i = 0; i < n_esi; ++i) key += "," + std::to_string(esi[i]);
    }
    auto& slot = ctx->colk[key];
    if (!slot) {
        std::unique_ptr<ColKernel> k(new ColKernel());
        k->p = p;
        if (!all_C) k->esi.assign(esi, esi + n_esi);
        ColIR ir;
        std::string err;
        const bool ok = all_C ? build_colprog_C(p, &ir, &err) : build_colprog(p, esi, n_esi, &ir, &err);
        if (!ok) return fail(RQ_ERR_PLAN, err);
        AllocOpts o;
        MProg mp;
        if (!allocate_colprog(ir, o, &mp, &err)) return fail(RQ_ERR_PLAN, err);
        const std::string src = emit_colprog_asm(mp, "rq_colprog");
        std::vector<char> co;
        if (!comgr_assemble(src, &co, &err)) return fail(RQ_ERR_PLAN, err);
        HIP_TRY(hipModuleLoadData(&k->mod, co.data()));
        HIP_TRY(hipModuleGetFunction(&k->fn, k->mod, "rq_colprog"));
        k->n_out = ir.n_out;
        k->n_slots = mp.n_slots;
        k->st = mp.st;
        k->n_ins = (uint32_t)mp.ins.size();
        slot = std::move(k);
    }
    *out = slot.get();
    return RQ_OK;
}

// Run a column program over n_blocks device-resident blocks.  Caller holds ctx->mu.
int launch_col(DevCtx* ctx, ColKernel* k, uint32_t T, uint32_t n_blocks, const void* src, uint64_t src_stride,
               void* out, uint64_t out_stride, void* stream) {
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    const uint32_t Td = T / 4;
    // every buffer offset is 32-bit: split so that each launch spans < 4 GiB per buffer
    const uint64_t lim = 0xFFFFFFFFull - (uint64_t)std::max(k->p.K, k->n_out) * T;
    uint32_t per = n_blocks;
    while (per > 1 && ((uint64_t)per * src_stride > lim || (uint64_t)per * out_stride > lim)) per = (per + 1) / 2;
    if ((uint64_t)per * src_stride > lim || (uint64_t)per * out_stride > lim)
        return fail(RQ_ERR_UNSUPPORTED, "block stride beyond the 4 GiB buffer-offset range");
    const uint64_t max_cols = (uint64_t)per * Td;
    if (max_cols > 0x7FFFFFFFull) return fail(RQ_ERR_UNSUPPORTED, "batch too large");
    const uint32_t max_waves = (uint32_t)((max_cols + 63) / 64);
    const size_t spw = (size_t)std::max<uint32_t>(k->n_slots, 1) * 256;
    int rc;
    if ((rc = ctx->ws_scratch.ensure(spw * max_waves))) return rc;
    for (uint32_t b0 = 0; b0 < n_blocks; b0 += per) {
        const uint32_t nb = std::min(per, n_blocks - b0);
        ColKernArgs a;
        std::memset(&a, 0, sizeof a);
        a.src = (uint64_t)(uintptr_t)src + (uint64_t)b0 * src_stride;
        a.out = (uint64_t)(uintptr_t)out + (uint64_t)b0 * out_stride;
        a.scratch = (uint64_t)(uintptr_t)ctx->ws_scratch.p;
        a.src_stride = (uint32_t)src_stride;
        a.out_stride = (uint32_t)out_stride;
        a.T = T;
        a.n_cols = nb * Td;
        a.scr_per_wave = (uint32_t)spw;
        if (!divmagic(Td, a.n_cols, &a.magic, &a.shift)) return fail(RQ_ERR_UNSUPPORTED, "no division magic");
        size_t sz = sizeof a;
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        const uint32_t waves = (a.n_cols + 63) / 64;
        HIP_TRY(hipModuleLaunchKernel(k->fn, waves, 1, 1, 64, 1, 1, 0, (hipStream_t)stream, nullptr, cfg));
    }
    return RQ_OK;
}

// A^-1 restricted to the K' source columns: run the plan on the identity payload (T = K' bytes).
int ensure_cid(DevCtx* ctx, DevPlan* dp, void* stream) {
    if (dp->cid_ready) return RQ_OK;
    const Params& p0 = dp->host.p;
    Params p = p0;
    p.K = p.Kp;  // every source row present
    const uint32_t Tc = (p.Kp + 3) & ~3u;
    std::vector<uint8_t> id((size_t)p.Kp * Tc, 0);
    for (uint32_t i = 0; i < p.Kp; ++i) id[(size_t)i * Tc + i] = 1;
    DevBuf src;
    int rc = src.ensure(id.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(src.p, id.data(), id.size(), hipMemcpyHostToDevice));
    if ((rc = dp->cid.ensure((size_t)p.L * Tc))) return rc;
    if ((rc = encode_locked(ctx, p, Tc, 1, src.p, id.size(), 0, nullptr, nullptr, 0, dp->cid.p, 0, stream))) return rc;
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    dp->cid_stride = Tc;
    dp->cid_ready = true;
    return RQ_OK;
}

constexpr uint32_t MAX_E = 255;  // decode-solve limits (LDS-resident [M | I])

// Batched syndrome decode.  Caller holds ctx->mu.  Host arrays as in rq_decode_desc.
int decode_locked(DevCtx* ctx, const Params& p, uint32_t T, uint32_t n_blocks, void* data, uint64_t data_stride,
                  const uint32_t* n_erased, const uint32_t* erased, const uint32_t* n_repair,
                  const uint32_t* repair_esi, const void* repair, int32_t* status, void* stream) {
    DevPlan* dp;
    int rc = get_dev_plan(ctx, p, &dp);
    if (rc) return rc;
    if ((rc = ensure_cid(ctx, dp, stream))) return rc;
    // per-block bookkeeping (host, O(n_blocks))
    std::vector<uint32_t> blk_map, eoff(n_blocks + 1, 0), roff(n_blocks + 1, 0);
    size_t max_lds_solve = 0;
    uint32_t max_e = 0;
    for (uint32_t b = 0; b < n_blocks; ++b) {
        eoff[b + 1] = eoff[b] + n_erased[b];
        roff[b + 1] = roff[b] + n_repair[b];
        const uint32_t e = n_erased[b], nr = n_repair[b];
        if ((p.K - e) + nr < p.K) { status[b] = RQ_ERR_NOT_ENOUGH; continue; }
        if (e == 0) { status[b] = 1; continue; }
        const size_t need = (((size_t)nr * (e + nr) + 15) & ~size_t(15)) + (size_t)nr * 24;  // [M | I] + tuples
        if (e > MAX_E || nr > 255 || need > 150 * 1024) { status[b] = RQ_ERR_UNSUPPORTED; continue; }
        status[b] = -100;  // pending
        blk_map.push_back(b);
        max_lds_solve = std::max(max_lds_solve, need);
        max_e = std::max(max_e, e);
    }
    const uint32_t nw = (uint32_t)blk_map.size();
    if (nw == 0) return RQ_OK;
    const size_t n_er = eoff[n_blocks], n_rep = roff[n_blocks];
    // index workspace: blk_map | eoff | roff | erased | rep_esi | status
    std::vector<uint32_t> idx;
    idx.reserve(nw + 2 * (n_blocks + 1) + n_er + n_rep + n_blocks);
    const size_t o_map = 0;
    idx.insert(idx.end(), blk_map.begin(), blk_map.end());
    const size_t o_eoff = idx.size();
    idx.insert(idx.end(), eoff.begin(), eoff.end());
    const size_t o_roff = idx.size();
    idx.insert(idx.end(), roff.begin(), roff.end());
    const size_t o_er = idx.size();
    idx.insert(idx.end(), erased, erased + n_er);
    const size_t o_rep = idx.size();
    idx.insert(idx.end(), repair_esi, repair_esi + n_rep);
    const size_t o_st = idx.size();
    idx.resize(idx.size() + n_blocks, 0);
    if ((rc = ctx->ws_idx.ensure(idx.size() * 4))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->ws_idx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, (hipStream_t)stream));
    const uint32_t* di = ctx->ws_idx.as<uint32_t>();
    if ((rc = ctx->ws_sigma.ensure(std::max<size_t>(n_rep, 1) * T))) return rc;
    if ((rc = ctx->ws_x.ensure((size_t)nw * max_e * max_e))) return rc;
    if ((rc = ctx->ws_xp.ensure((size_t)nw * max_e * 2))) return rc;

    // 1) syndromes: sigma_j = r_j ^ G_j A^-1 D(S with erased rows zeroed)
    Geometry g;
    if ((rc = geometry(*dp, T, p.K, true, &g))) return rc;
    DevWave* dw;
    if ((rc = get_dev_wave(dp, g.sd, &dw))) return rc;
    EncArgs a = base_args(*dp, *dw, p, T, g.sd);
    a.src = static_cast<const uint8_t*>(data);
    a.src_stride = data_stride;
    a.blk_map = di + o_map;
    a.erased_off = di + o_eoff;
    a.erased = di + o_er;
    a.out_esi = di + o_rep;
    a.out_off = di + o_roff;
    a.out = ctx->ws_sigma.as<uint8_t>();
    a.xor_in = static_cast<const uint8_t*>(repair);
    int e = launch_encode(a, g.n_strips, nw, g.group, stream);
    if (e) return fail(RQ_ERR_DEVICE, std::string("k_encode(decode) launch: ") + hipGetErrorString((hipError_t)e));
    // 2) per-block solve
    SolveArgs s;
    s.p = dev_params(p);
    s.blk_map = di + o_map;
    s.erased_off = di + o_eoff;
    s.erased = di + o_er;
    s.rep_off = di + o_roff;
    s.rep_esi = di + o_rep;
    s.cid = dp->cid.as<uint8_t>();
    s.cid_stride = dp->cid_stride;
    s.xmat = ctx->ws_x.as<uint8_t>();
    s.xpiv = ctx->ws_xp.as<uint16_t>();
    s.status = reinterpret_cast<int32_t*>(ctx->ws_idx.as<uint32_t>() + o_st);
    s.max_e = max_e;
    e = launch_solve(s, nw, (uint32_t)((max_lds_solve + 15) & ~size_t(15)), stream);
    if (e) return fail(RQ_ERR_DEVICE, std::string("k_solve launch: ") + hipGetErrorString((hipError_t)e));
    // 3) apply
    ApplyArgs ap;
    ap.blk_map = di + o_map;
    ap.erased_off = di + o_eoff;
    ap.erased = di + o_er;
    ap.rep_off = di + o_roff;
    ap.sigma = ctx->ws_sigma.as<uint8_t>();
    ap.xmat = s.xmat;
    ap.xpiv = s.xpiv;
    ap.status = s.status;
    ap.data = static_cast<uint8_t*>(data);
    ap.data_stride = data_stride;
    ap.T = T;
    ap.max_e = max_e;
    const uint32_t n_strips = (T / 4 + 63) / 64;
    const uint32_t lds = max_e * 64 * 4 + ((max_e * max_e + 15) & ~15u);
    e = launch_apply(ap, n_strips, nw, lds, stream);
    if (e) return fail(RQ_ERR_DEVICE, std::string("k_apply launch: ") + hipGetErrorString((hipError_t)e));
    std::vector<int32_t> st(n_blocks);
    HIP_TRY(hipMemcpyAsync(st.data(), ctx->ws_idx.as<uint32_t>() + o_st, n_blocks * 4, hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    for (uint32_t b : blk_map) status[b] = st[b];
    return RQ_OK;
}

}  // namespace
}  // namespace rq

using namespace rq;

// ====================================== C ABI ==============================================
struct rq_enc {
    Params p{};
    uint32_t T = 0, Tp = 0;
    std::vector<uint8_t> src;  // K x Tp, zero padded (GenSymbol for esi < K aliases this)
    DevBuf d_src, d_C, d_esi, d_out;
};

struct rq_dec {
    Params p{};
    uint64_t size = 0;
    uint32_t T = 0;
    std::vector<uint8_t> fast;       // K x T
    std::vector<uint8_t> have;       // K flags
    uint32_t nfast = 0;
    std::map<uint32_t, std::vector<uint8_t>> slow;  // repair symbols by ESI
};

extern "C" {

const char* rq_strerror(int code) {
    switch (code) {
        case RQ_OK: return "ok";
        case RQ_ERR_SYMBOL_SIZE_ZERO: return "symbol size cannot be zero";
        case RQ_ERR_K_TOO_BIG: return "k is too big";
        case RQ_ERR_NOT_ENOUGH: return "not enough symbols to decode";
        case RQ_ERR_SYMBOL_SIZE: return "incorrect symbol size";
        case RQ_ERR_BAD_ARG: return "bad argument";
        case RQ_ERR_DEVICE: return "device error";
        case RQ_ERR_UNSUPPORTED: return "unsupported shape";
        case RQ_ERR_PLAN: return "plan compilation failed";
        default: return "unknown error";
    }
}

const char* rq_last_error(void) { return g_err.c_str(); }

int rq_params(uint64_t size, uint32_t T, uint32_t out[11]) {
    Params p;
    const int rc = calc_params(size, T, &p);
    if (rc) return fail(rc, rq_strerror(rc));
    std::memcpy(out, &p, sizeof p);
    return RQ_OK;
}

int rq_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rq_set_device(int device) {
    const int n = rq_device_count();
    if (device < 0 || device >= n) return fail(RQ_ERR_DEVICE, "bad device index");
    g_device = device;
    HIP_TRY(hipSetDevice(device));
    return RQ_OK;
}

int rq_plan_stats(uint32_t K, uint32_t stats[11]) {
    const Plan* pl;
    int rc = host_plan(K, &pl);
    if (rc) return rc;
    const PlanStats& s = pl->stats;
    const uint32_t v[11] = {s.n_stmts, s.n_levels, s.n_src_xor, s.n_src_mul, s.n_reload, s.u,
                            s.inactivated, s.n_pivots, s.n_slots, s.passB_inplace, s.passB_reload};
    std::memcpy(stats, v, sizeof v);
    return RQ_OK;
}

int rq_plan_export(uint32_t K, uint32_t sizes[5], uint32_t* level_start, uint32_t* stmt_off, uint32_t* words,
                   uint16_t* load_slot, uint16_t* col_slot) {
    const Plan* pl;
    int rc = host_plan(K, &pl);
    if (rc) return rc;
    sizes[0] = (uint32_t)pl->level_start.size();
    sizes[1] = (uint32_t)pl->stmt_off.size();
    sizes[2] = (uint32_t)pl->words.size();
    sizes[3] = pl->p.Kp;
    sizes[4] = pl->p.L;
    if (level_start) std::memcpy(level_start, pl->level_start.data(), pl->level_start.size() * 4);
    if (stmt_off) std::memcpy(stmt_off, pl->stmt_off.data(), pl->stmt_off.size() * 4);
    if (words) std::memcpy(words, pl->words.data(), pl->words.size() * 4);
    if (load_slot) std::memcpy(load_slot, pl->load_slot.data(), pl->load_slot.size() * 2);
    if (col_slot) std::memcpy(col_slot, pl->col_slot.data(), pl->col_slot.size() * 2);
    return RQ_OK;
}

int rq_wave_export(uint32_t K, uint32_t sd, uint32_t sizes[4], uint32_t* words, uint32_t* wave_off) {
    const Plan* pl;
    int rc = host_plan(K, &pl);
    if (rc) return rc;
    WaveProgram wp;
    std::string err;
    if (!build_wave_program(*pl, enc_waves(), sd, &wp, &err)) return fail(RQ_ERR_PLAN, err);
    sizes[0] = (uint32_t)wp.words.size();
    sizes[1] = wp.n_waves;
    sizes[2] = wp.n_levels;
    sizes[3] = wp.n_slots;
    if (words) std::memcpy(words, wp.words.data(), wp.words.size() * 4);
    if (wave_off) std::memcpy(wave_off, wp.wave_off.data(), wp.wave_off.size() * 4);
    return RQ_OK;
}

int rq_debug_colprog_eval(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                          uint8_t* out, uint32_t stats[12]) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    ColIR ir;
    std::string err;
    const bool ok = esi ? build_colprog(p, esi, n_out, &ir, &err) : build_colprog_C(p, &ir, &err);
    if (!ok) return fail(RQ_ERR_PLAN, err);
    if (src && out) eval_colprog(ir, src, T, out);
    if (stats) {
        const auto& s = ir.st;
        const uint32_t v[12] = {(uint32_t)ir.nodes.size(), s.xor2, s.xor3, s.xt, s.xtx, s.load, s.store, s.zero,
                                s.u, s.npiv, s.n2, ir.n_out};
        std::memcpy(stats, v, sizeof v);
    }
    return RQ_OK;
}

int rq_debug_colprog_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                             uint8_t* out, const uint32_t opts[5], uint32_t stats[16], char* asm_buf, size_t asm_cap,
                             size_t* asm_len) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    ColIR ir;
    std::string err;
    const bool ok = esi ? build_colprog(p, esi, n_out, &ir, &err) : build_colprog_C(p, &ir, &err);
    if (!ok) return fail(RQ_ERR_PLAN, err);
    AllocOpts o;
    if (opts) {
        if (opts[0]) o.n_vgpr = std::min<uint32_t>(opts[0], V_ALLOC);
        if (opts[1]) o.n_agpr = std::min<uint32_t>(opts[1], 256);
        if (opts[2]) o.la_load = opts[2];
        if (opts[3]) o.la_reload = opts[3];
        if (opts[4]) o.max_vmem = std::min<uint32_t>(opts[4], 60);
    }
    MProg mp;
    if (!allocate_colprog(ir, o, &mp, &err)) return fail(RQ_ERR_PLAN, err);
    if (src && out && !emulate_colprog(mp, src, T, out, &err)) return fail(RQ_ERR_PLAN, err);
    if (stats) {
        const auto& s = mp.st;
        const uint32_t v[16] = {(uint32_t)mp.ins.size(), s.valu, s.ldsrc, s.stout, s.spst, s.spld, s.accw, s.accr,
                                s.wait, s.nop, s.sync_reload, mp.n_slots, (uint32_t)ir.nodes.size(), ir.st.xt + ir.st.xtx, 0, 0};
        std::memcpy(stats, v, sizeof v);
    }
    if (asm_len) {
        const std::string a = emit_colprog_asm(mp, "rq_colprog");
        *asm_len = a.size();
        if (asm_buf && asm_cap >= a.size()) std::memcpy(asm_buf, a.data(), a.size());
    }
    return RQ_OK;
}

int rq_debug_gf_selftest(uint32_t* bad_xtime, uint32_t* bad_mul) {
    if (!bad_xtime || !bad_mul) return fail(RQ_ERR_BAD_ARG, "null output");
    DevCtx* ctx;
    int rc;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    const uint32_t n = 1024;
    std::vector<uint32_t> x(n), tabs(256 * 5), out((size_t)n * 257);
    uint32_t s = 0x12345678u;
    for (uint32_t i = 0; i < n; ++i) { s = s * 1664525u + 1013904223u; x[i] = i < 256 ? i * 0x01010101u : s; }
    for (uint32_t c = 0; c < 256; ++c) gf_perm_tables((uint8_t)c, &tabs[c * 5]);
    DevBuf dx, dt, dout;
    if ((rc = upload(dx, x)) || (rc = upload(dt, tabs)) || (rc = dout.ensure(out.size() * 4))) return rc;
    HIP_TRY((hipError_t)launch_gf_selftest(dx.as<uint32_t>(), n, dt.as<uint32_t>(), dout.as<uint32_t>()));
    HIP_TRY(hipMemcpy(out.data(), dout.p, out.size() * 4, hipMemcpyDeviceToHost));
    const GF& g = gf();
    auto mul4 = [&](uint32_t v, uint8_t c) {
        uint32_t r = 0;
        for (int b = 0; b < 4; ++b) r |= (uint32_t)g.mul((uint8_t)(v >> (8 * b)), c) << (8 * b);
        return r;
    };
    *bad_xtime = 0;
    *bad_mul = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (out[i] != mul4(x[i], 2)) ++*bad_xtime;
        for (uint32_t c = 0; c < 256; ++c)
            if (out[n + (size_t)c * n + i] != mul4(x[i], (uint8_t)c)) ++*bad_mul;
    }
    return RQ_OK;
}

int rq_debug_run_wave_program(uint32_t K, uint32_t T, const uint32_t* words, uint32_t n_words,
                              const uint32_t* wave_off, uint32_t n_levels, uint32_t n_blocks, uint32_t iters,
                              float* ms) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    DevCtx* ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevPlan* dp;
    if ((rc = get_dev_plan(ctx, p, &dp))) return rc;
    Geometry g;
    if ((rc = geometry(*dp, T, p.K, false, &g))) return rc;
    DevWave* dwv;
    if ((rc = get_dev_wave(dp, g.sd, &dwv))) return rc;
    EncArgs a = base_args(*dp, *dwv, p, T, g.sd);
    DevBuf w, wo, src;
    std::vector<uint32_t> wv(words, words + n_words);
    wv.resize(wv.size() + 256, 0);
    std::vector<uint32_t> ov(wave_off, wave_off + enc_waves());
    if ((rc = upload(w, wv)) || (rc = upload(wo, ov)) || (rc = src.ensure((size_t)n_blocks * K * T))) return rc;
    HIP_TRY(hipMemset(src.p, 0, (size_t)n_blocks * K * T));
    a.wstream = w.as<uint32_t>();
    a.wave_off = wo.as<uint32_t>();
    a.n_levels = n_levels;
    a.src = src.as<uint8_t>();
    a.src_stride = (uint64_t)K * T;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    launch_encode(a, g.n_strips, n_blocks, g.group, nullptr);
    HIP_TRY(hipEventRecord(e0, nullptr));
    for (uint32_t i = 0; i < iters; ++i) launch_encode(a, g.n_strips, n_blocks, g.group, nullptr);
    HIP_TRY(hipEventRecord(e1, nullptr));
    HIP_TRY(hipEventSynchronize(e1));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, e0, e1));
    *ms = t / (float)iters;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return RQ_OK;
}

int rq_encode_batch(const rq_encode_desc* d) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->T % 4 || d->K == 0 || (!d->src && d->n_blocks)) return fail(RQ_ERR_BAD_ARG, "bad encode descriptor (T % 4, K, src)");
    if (d->n_blocks == 0) return RQ_OK;
    if (d->n_esi && (!d->esi || !d->out)) return fail(RQ_ERR_BAD_ARG, "n_esi without esi/out");
    for (uint32_t i = 0; i < d->n_esi; ++i)
        if (d->esi[i] < d->K) return fail(RQ_ERR_BAD_ARG, "batch ESIs must be repair ids (>= K)");
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    DevCtx* ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!d->c_out) {
        if (!d->n_esi) return RQ_OK;
        ColKernel* k;
        if ((rc = get_col_kernel(ctx, p, d->esi, d->n_esi, false, &k))) return rc;
        return launch_col(ctx, k, d->T, d->n_blocks, d->src, d->src_stride, d->out, d->out_stride, d->stream);
    }
    const uint32_t* d_esi = nullptr;
    if (d->n_esi) {
        if ((rc = ctx->ws_esi.ensure(d->n_esi * 4))) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->ws_esi.p, d->esi, d->n_esi * 4, hipMemcpyHostToDevice, (hipStream_t)d->stream));
        d_esi = ctx->ws_esi.as<uint32_t>();
    }
    return encode_locked(ctx, p, d->T, d->n_blocks, d->src, d->src_stride, d->n_esi, d_esi, d->out, d->out_stride,
                         d->c_out, d->c_stride, d->stream);
}

int rq_decode_batch(const rq_decode_desc* d) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->T % 4 || d->K == 0) return fail(RQ_ERR_BAD_ARG, "bad decode descriptor (T % 4, K)");
    if (d->n_blocks == 0) return RQ_OK;
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    DevCtx* ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return decode_locked(ctx, p, d->T, d->n_blocks, d->data, d->data_stride, d->n_erased, d->erased, d->n_repair,
                         d->repair_esi, d->repair, d->status, d->stream);
}

// ---------------- per-object encoder (CreateEncoder / GenSymbol) ----------------
rq_enc* rq_encoder_create(const uint8_t* data, size_t len, uint32_t T, int* err) {
    int dummy;
    if (!err) err = &dummy;
    Params p;
    int rc = calc_params(len, T, &p);
    if (rc) { *err = fail(rc, rc == RQ_ERR_SYMBOL_SIZE_ZERO ? "failed to calc params: symbol size cannot be zero"
                                                           : "failed to calc params: k is too big"); return nullptr; }
    std::unique_ptr<rq_enc> e(new rq_enc());
    e->p = p;
    e->T = T;
    e->Tp = (T + 3) & ~3u;
    e->src.assign((size_t)p.K * e->Tp, 0);
    for (uint32_t i = 0; i < p.K; ++i) {
        const size_t off = (size_t)i * T;
        const size_t n = off >= len ? 0 : std::min<size_t>(T, len - off);
        if (n) std::memcpy(&e->src[(size_t)i * e->Tp], data + off, n);
    }
    DevCtx* ctx;
    if ((rc = get_ctx(&ctx))) { *err = rc; return nullptr; }
    std::lock_guard<std::mutex> lk(ctx->mu);
    if ((rc = e->d_src.ensure(e->src.size())) || (rc = e->d_C.ensure((size_t)p.L * e->Tp))) { *err = rc; return nullptr; }
    if (hipMemcpy(e->d_src.p, e->src.data(), e->src.size(), hipMemcpyHostToDevice) != hipSuccess) {
        *err = fail(RQ_ERR_DEVICE, "hipMemcpy H2D failed");
        return nullptr;
    }
    rc = encode_locked(ctx, p, e->Tp, 1, e->d_src.p, e->src.size(), 0, nullptr, nullptr, 0, e->d_C.p, 0, nullptr);
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = fail(RQ_ERR_DEVICE, "encode failed");
    if (rc) { *err = rc; return nullptr; }
    *err = RQ_OK;
    return e.release();
}

uint32_t rq_encoder_k(const rq_enc* e) { return e ? e->p.K : 0; }
uint32_t rq_encoder_symbol_size(const rq_enc* e) { return e ? e->T : 0; }

int rq_encoder_symbols(rq_enc* e, uint32_t first, uint32_t count, uint8_t* out) {
    if (!e || (!out && count)) return fail(RQ_ERR_BAD_ARG, "null encoder/out");
    const uint32_t K = e->p.K, T = e->T;
    std::vector<uint32_t> rep;
    for (uint32_t i = 0; i < count; ++i) {
        const uint64_t esi = (uint64_t)first + i;
        if (esi < K) std::memcpy(out + (size_t)i * T, &e->src[(size_t)esi * e->Tp], T);
        else rep.push_back((uint32_t)esi);
    }
    if (rep.empty()) return RQ_OK;
    DevCtx* ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if ((rc = e->d_esi.ensure(rep.size() * 4)) || (rc = e->d_out.ensure(rep.size() * e->Tp))) return rc;
    HIP_TRY(hipMemcpy(e->d_esi.p, rep.data(), rep.size() * 4, hipMemcpyHostToDevice));
    const int le = launch_gather(dev_params(e->p), e->d_C.as<uint8_t>(), e->Tp, e->d_esi.as<uint32_t>(),
                                 (uint32_t)rep.size(), e->d_out.as<uint8_t>(), nullptr);
    if (le) return fail(RQ_ERR_DEVICE, "k_gather launch failed");
    std::vector<uint8_t> buf(rep.size() * e->Tp);
    HIP_TRY(hipMemcpy(buf.data(), e->d_out.p, buf.size(), hipMemcpyDeviceToHost));
    size_t r = 0;
    for (uint32_t i = 0; i < count; ++i) {
        const uint64_t esi = (uint64_t)first + i;
        if (esi >= K) std::memcpy(out + (size_t)i * T, &buf[(r++) * e->Tp], T);
    }
    return RQ_OK;
}

int rq_encoder_symbol(rq_enc* e, uint32_t esi, uint8_t* out) { return rq_encoder_symbols(e, esi, 1, out); }

void rq_encoder_free(rq_enc* e) { delete e; }

// ---------------- per-object decoder (CreateDecoder / AddSymbol / Decode) ----------------
rq_dec* rq_decoder_create(uint64_t data_size, uint32_t T, int* err) {
    int dummy;
    if (!err) err = &dummy;
    Params p;
    const int rc = calc_params(data_size, T, &p);
    if (rc) { *err = fail(rc, rc == RQ_ERR_SYMBOL_SIZE_ZERO ? "failed to calc params: symbol size cannot be zero"
                                                           : "failed to calc params: k is too big"); return nullptr; }
    rq_dec* d = new rq_dec();
    d->p = p;
    d->size = data_size;
    d->T = T;
    d->fast.assign((size_t)p.K * T, 0);
    d->have.assign(p.K, 0);
    *err = RQ_OK;
    return d;
}

uint32_t rq_decoder_k(const rq_dec* d) { return d ? d->p.K : 0; }

int rq_decoder_add(rq_dec* d, uint32_t esi, const uint8_t* sym, size_t len, int* can_try) {
    if (!d) return fail(RQ_ERR_BAD_ARG, "null decoder");
    if (len != d->T) {
        char buf[96];
        std::snprintf(buf, sizeof buf, "incorrect symbol size %zu, should be %u", len, d->T);
        return fail(RQ_ERR_SYMBOL_SIZE, buf);
    }
    if (esi < d->p.K) {
        if (!d->have[esi]) {
            d->have[esi] = 1;
            std::memcpy(&d->fast[(size_t)esi * d->T], sym, d->T);
            d->nfast++;
        }
    } else if (!d->slow.count(esi)) {
        d->slow.emplace(esi, std::vector<uint8_t>(sym, sym + d->T));
    }
    if (can_try) *can_try = d->p.K <= d->nfast + (uint32_t)d->slow.size();
    return RQ_OK;
}

int rq_decoder_decode(rq_dec* d, uint8_t* out, int* ok) {
    if (!d || !ok) return fail(RQ_ERR_BAD_ARG, "null decoder/ok");
    const uint32_t K = d->p.K, T = d->T;
    *ok = 0;
    if (K > d->nfast + (uint32_t)d->slow.size()) return fail(RQ_ERR_NOT_ENOUGH, "not enough symbols to decode");
    if (d->nfast < K) {
        const uint32_t Tp = (T + 3) & ~3u;
        std::vector<uint32_t> erased, resi;
        for (uint32_t i = 0; i < K; ++i)
            if (!d->have[i]) erased.push_back(i);
        std::vector<uint8_t> data((size_t)K * Tp, 0), rep((size_t)d->slow.size() * Tp, 0);
        for (uint32_t i = 0; i < K; ++i)
            if (d->have[i]) std::memcpy(&data[(size_t)i * Tp], &d->fast[(size_t)i * T], T);
        size_t r = 0;
        for (auto& kv : d->slow) {
            resi.push_back(kv.first);
            std::memcpy(&rep[(r++) * Tp], kv.second.data(), T);
        }
        DevCtx* ctx;
        int rc = get_ctx(&ctx);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(ctx->mu);
        DevBuf dd, dr;
        if ((rc = dd.ensure(data.size())) || (rc = dr.ensure(std::max<size_t>(rep.size(), 4)))) return rc;
        HIP_TRY(hipMemcpy(dd.p, data.data(), data.size(), hipMemcpyHostToDevice));
        if (!rep.empty()) HIP_TRY(hipMemcpy(dr.p, rep.data(), rep.size(), hipMemcpyHostToDevice));
        const uint32_t ne = (uint32_t)erased.size(), nr = (uint32_t)resi.size();
        int32_t st = 0;
        rc = decode_locked(ctx, d->p, Tp, 1, dd.p, data.size(), &ne, erased.data(), &nr, resi.data(), dr.p, &st, nullptr);
        if (rc) return rc;
        if (st == RQ_ERR_UNSUPPORTED) return fail(RQ_ERR_UNSUPPORTED, "erasure pattern beyond the device solver limits");
        if (st != 1) return RQ_OK;  // rank-deficient: (false, nil, nil)
        HIP_TRY(hipMemcpy(data.data(), dd.p, data.size(), hipMemcpyDeviceToHost));
        for (uint32_t i : erased) std::memcpy(&d->fast[(size_t)i * T], &data[(size_t)i * Tp], T);
        // The library fills the missing rows into its own buffer as well (RQ/decoder.go:126-130).
        for (uint32_t i : erased) { d->have[i] = 1; d->nfast++; }
    }
    std::memcpy(out, d->fast.data(), d->size);
    *ok = 1;
    return RQ_OK;
}

void rq_decoder_free(rq_dec* d) { delete d; }

}  // extern "C"
