// rq_engine.cpp -- host runtime of librqhip.so: device contexts, the cache of compiled column
// programs, the batched device-resident encode/decode entry points, and the per-object
// Encoder/Decoder API that mirrors xssnick/raptorq as wrapped by go/fec/raptorq_wrap.go.
//
// There is no CPU fallback: every symbol the engine returns is computed on the GPU, by a
// generated gfx950 code object (rq_colprog / rq_colasm) or by the kernels in rq_kernels.hip;
// without a usable gfx950 device the calls fail with RQ_ERR_DEVICE.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wc++20-extensions"
#include <hip/hip_ext.h>  // hipExtModuleLaunchKernel (rq_launch_timing)
#pragma clang diagnostic pop
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <unordered_set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rqhip.h"
#include "../../include/rqhip_debug.h"
#include "rq_applygi.hpp"
#include "rq_gistream.hpp"
#include "rq_colasm.hpp"
#include "rq_colprog.hpp"
#include "rq_device.hpp"

namespace rq {

const GF& gf() {
    static const GF g;
    return g;
}

namespace {

thread_local std::string g_err;
thread_local int g_device = -1;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// Device row pitch for a T-byte symbol staged by the library: a multiple of 4 bytes (one dword per
// lane) and at least 8 (the column program's block/column split needs T/4 >= 2).
inline uint32_t pad_row(uint32_t T) { return T <= 8 ? 8u : (T + 3) & ~3u; }

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(RQ_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// Growable device buffer (allocation happens outside any timed region after warmup).  Growth is
// geometric: a reallocation frees the old buffer, and hipFree waits for the whole device, so a
// stream of varying sizes (chunks, shapes) should settle after a few calls.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return RQ_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        const size_t want = std::max<size_t>({n, cap + cap / 2, 4096});
        cap = 0;
        if (hipMalloc(&p, want) != hipSuccess) return fail(RQ_ERR_DEVICE, "hipMalloc failed");
        cap = want;
        return RQ_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

// A compiled column program loaded on one device.
struct ColKernel {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    Params p{};
    std::vector<uint32_t> esi;     // outputs (empty: all L intermediate symbols)
    uint32_t n_out = 0, n_slots = 0, n_ins = 0;
    uint32_t waves_per_cu = 4;     // residency of the code object (registers, LDS)
    uint32_t wg_waves = 1;         // waves per workgroup (MProg::wg_waves)
    bool pair = false;             // two-wave program (emit_pair_asm): one item per workgroup iteration
    bool fetch_ok = false;         // its workgroups past the grid can carry a decode's descriptor fetch
    std::vector<uint32_t> dma4_rows;  // four-row staging: every group's rows (needs 16-B aligned rows)
    MProg::Stats st{};
    uint64_t last_use = 0;         // LRU clock of the per-device cache
    DevBuf mrep;                   // decode: outputs on the identity payload
    uint32_t mrep_stride = 0;
    std::vector<uint32_t> src_rows;                 // source row of each buffer load, in issue order
    uint32_t row_end = 1;                           // 1 + the largest source row any load reads
    std::map<uint32_t, std::unique_ptr<DevBuf>> row_off;  // T -> src_rows * T (the kernel's soffsets)
    ~ColKernel() { if (mod) (void)hipModuleUnload(mod); }
};

// Pinned host staging (descriptor uploads and status downloads run as true async copies).
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return RQ_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        const size_t want = std::max<size_t>({n, cap + cap / 2, 1 << 16});  // geometric, as DevBuf
        cap = 0;
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return fail(RQ_ERR_DEVICE, "hipHostMalloc failed");
        cap = want;
        return RQ_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    ~HostBuf() { if (p) (void)hipHostFree(p); }
};

// Per-stream workspaces: kernels of calls on different streams may run concurrently, so every
// stream gets its own scratch / index / syndrome buffers (calls on one stream are ordered).
// Flags of the engine's own device-side events (`last`, the side-stream `cpy`): nobody on the host reads
// memory after them, so the marker needs no system-scope release (RQHIP_EV_NOFENCE=1 in experiments
// builds; measured in profiles/r04e).
unsigned internal_event_flags() {
    static const unsigned f = [] {
        const char* e = knob("RQHIP_EV_NOFENCE");
        return hipEventDisableTiming | (e && e[0] == '1' ? hipEventDisableSystemFence : 0u);
    }();
    return f;
}

struct Workspace {
    DevBuf r0, xb, xp, gws, scratch;
    DevBuf gi;                      // the register-table apply's index stream (k_xbits)
    DevBuf pk;                      // host-memory decode: recovered rows, packed for the D2H
    HostBuf h_status, h_pack;
    // decode descriptors, double-buffered so that rq_decode_batch_async can return before its upload
    // ran: call n uses set n % 2; the host refills a set's pinned staging only after that set's
    // previous upload completed (`up`); the device copy is rewritten in stream order, and grown
    // only after a stream synchronisation
    DevBuf idx[2];
    HostBuf h_idx[2];
    hipEvent_t up[2] = {nullptr, nullptr};
    DevBuf dstatus;                 // zero-copy descriptors: the solver/apply statuses stay on the device
    // side-stream descriptor upload (the default): set n's H2D copy runs on `cs` beside the syndrome
    // program; the caller's stream waits for `cpy[n % 2]` before the solve
    hipStream_t cs = nullptr;
    hipEvent_t cpy[2] = {nullptr, nullptr};
    // solve beside the syndrome program (solve_beside()): `go` on the caller's stream before the
    // syndrome program, `solved` on `cs` after the solver kernels
    hipEvent_t go = nullptr, solved = nullptr;

    uint32_t flip = 0;
    uint64_t last_use = 0;          // LRU clock (DevCtx::wsp)
    // recorded on the caller's stream after every call's last command that touches this workspace:
    // an evicted or released workspace is freed once it has completed (DevCtx::reap), so eviction
    // never synchronises the device while the context lock is held
    hipEvent_t last = nullptr;
    // the event that currently marks this workspace's last use: `last`, or a decode call's up[set]
    // recorded after its downloads (one marker per call instead of two)
    hipEvent_t done = nullptr;
    int mark(void* stream) {
#ifdef RQHIP_EXPERIMENTS
        static const bool nomark = std::getenv("RQHIP_NOMARK") != nullptr;  // timing only: what the markers cost
        if (nomark) return RQ_OK;
#endif
        if (!last && hipEventCreateWithFlags(&last, internal_event_flags()) != hipSuccess) {
            last = nullptr;
            return fail(RQ_ERR_DEVICE, "hipEventCreate failed");
        }
        if (hipEventRecord(last, (hipStream_t)stream) != hipSuccess) return fail(RQ_ERR_DEVICE, "hipEventRecord failed");
        done = last;
        return RQ_OK;
    }
    bool idle() const { return !done || hipEventQuery(done) != hipErrorNotReady; }
    ~Workspace() {
        if (last) (void)hipEventDestroy(last);
        for (hipEvent_t& e : up)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t& e : cpy)
            if (e) (void)hipEventDestroy(e);
        if (go) (void)hipEventDestroy(go);
        if (solved) (void)hipEventDestroy(solved);
        if (cs) (void)hipStreamDestroy(cs);
    }
};

// Records a workspace's `last` event on every exit once armed: a call that fails after it
// queued work touching the workspace still leaves the marker behind that work, so DevCtx::reap never
// frees buffers a failed call's kernels may still read or write.  The success paths disarm it and call
// mark() themselves (its error is theirs to return).
struct MarkGuard {
    Workspace* w = nullptr;
    void* stream = nullptr;
    bool armed = false;
    ~MarkGuard() {
        if (armed && w) (void)w->mark(stream);
    }
};

// Host-memory batch API: device staging of one pipeline stage (one internal stream).
struct Stage {
    hipStream_t s = nullptr;
    DevBuf in, out;                 // encode: source chunk / repairs; decode: data chunk / repairs
};

struct DevCtx {
    int device = -1;
    uint32_t n_cu = 256;
    std::mutex mu;
    bool tables = false;
    std::map<std::string, std::unique_ptr<ColKernel>> colk;  // keyed by (K', K, outputs); LRU-bounded
    uint64_t tick = 0;
    std::map<void*, std::unique_ptr<Workspace>> ws;
    static constexpr uint32_t NST = 3;  // host-memory pipeline stages: uploads run two chunks ahead
    Stage stage[NST];
    hipEvent_t kdone[NST] = {};  // host-memory paths: a stage's kernels were queued up to here
    // ... and its upload: the next chunk's upload waits for it, so the uploads run one after another
    // at the link's full rate instead of sharing it (all chunks' uploads finished together, and the
    // first chunk's kernels waited for the last upload: profiles/r02ae)
    hipEvent_t updone[NST] = {};
    // rq_launch_timing: while on, every column-program launch records this pair list's next
    // start / stop events as part of its own dispatch (hipExtModuleLaunchKernel): the kernel's time
    // without any marker command between it and its neighbours in the stream
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    size_t tev_used = 0;
    hipStream_t obj_stream = nullptr;  // per-object API: its own stream, pinned staging, device buffer
    // the register-table apply kernels (rq_applygi.cpp), assembled on first use for `gi_shape`: slot 1
    // reads precomputed syndromes (GiShape::SX), slot 0 the received and r0 rows
    hipModule_t gi_mod[2] = {};
    hipFunction_t gi_fn[2] = {};
    GiShape gi_shape[2];
    HostBuf obj_h;
    DevBuf obj_d;
    // Per-stream workspaces are bounded: a caller that uses a fresh stream per window would otherwise
    // grow device memory without limit (each holds r0 / scratch / descriptors, ~130 MB at K=1024 x
    // 1024 blocks).  Beyond MAX_WS caller streams the least recently used one is released (after a
    // device synchronisation: its stream may still run kernels reading it); the library's own stage
    // streams are never evicted.  rq_stream_release() releases one explicitly.
    static constexpr size_t MAX_WS = 8;
    std::vector<std::unique_ptr<Workspace>> dead;  // evicted / released, freed once idle
    void reap() {
        for (size_t i = 0; i < dead.size();)
            if (dead[i]->idle()) { dead[i] = std::move(dead.back()); dead.pop_back(); }
            else ++i;
    }
    Workspace* wsp(void* stream) {
        if (!dead.empty()) reap();
        auto& w = ws[stream];
        if (!w) {
            w.reset(new Workspace());
            evict_ws(stream);
        }
        w->last_use = ++tick;
        return w.get();
    }
    bool internal(void* s) const {
        for (const Stage& st : stage)
            if (st.s && (void*)st.s == s) return true;
        return obj_stream && (void*)obj_stream == s;
    }
    void evict_ws(void* keep) {
        size_t n_caller = 0;
        for (auto& kv : ws) n_caller += !internal(kv.first);
        while (n_caller > MAX_WS) {
            auto victim = ws.end();
            for (auto it = ws.begin(); it != ws.end(); ++it)
                if (it->first != keep && !internal(it->first) &&
                    (victim == ws.end() || it->second->last_use < victim->second->last_use))
                    victim = it;
            if (victim == ws.end()) return;
            dead.push_back(std::move(victim->second));  // freed by reap() once its last call completed
            ws.erase(victim);
            --n_caller;
        }
    }
    ~DevCtx() {  // rq_shutdown only (contexts are never destroyed at exit)
        (void)hipSetDevice(device);
        (void)hipDeviceSynchronize();
        ws.clear();
        dead.clear();
        colk.clear();
        for (hipModule_t m : gi_mod)
            if (m) (void)hipModuleUnload(m);
        for (Stage& st : stage)
            if (st.s) (void)hipStreamDestroy(st.s);
        for (hipEvent_t e : kdone)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : updone)
            if (e) (void)hipEventDestroy(e);
        if (obj_stream) (void)hipStreamDestroy(obj_stream);
        for (auto& pr : tev) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    }
    void release_ws(void* stream) {
        auto it = ws.find(stream);
        if (it == ws.end()) return;
        dead.push_back(std::move(it->second));
        ws.erase(it);
        reap();
    }
};

// Device contexts are created on first use and deliberately never destroyed by static destructors:
// at process exit the HIP runtime (or a profiler's tool library) may already be torn down, and a
// hipFree / hipModuleUnload from __cxa_finalize then faults (profiles/r02az: SIGSEGV in
// __cxa_finalize after rocprofv3's finalisation).  rq_shutdown() releases everything explicitly.
// Each library call holds its context through a CtxRef (a shared_ptr): rq_shutdown only takes the
// contexts out of the map, and a context is destroyed when the last call that fetched it returns, so
// a call racing rq_shutdown never touches freed memory.
std::mutex g_ctx_mu;
std::map<int, std::shared_ptr<DevCtx>>& g_ctx = *new std::map<int, std::shared_ptr<DevCtx>>();
struct CtxRef {
    std::shared_ptr<DevCtx> p;
    DevCtx* operator->() const { return p.get(); }
    operator DevCtx*() const { return p.get(); }
};

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

int get_ctx(CtxRef* out) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(dev));
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto& c = g_ctx[dev];
    if (!c) {
        c = std::make_shared<DevCtx>();
        c->device = dev;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            c->n_cu = (uint32_t)cus;
    }
    out->p = c;
    return RQ_OK;
}

template <class T>
int upload(DevBuf& b, const std::vector<T>& v, void* stream) {
    int rc = b.ensure(std::max<size_t>(v.size(), 1) * sizeof(T));
    if (rc) return rc;
    if (!v.empty()) HIP_TRY(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, (hipStream_t)stream));
    return RQ_OK;
}

DevParams dev_params(const Params& p) {
    DevParams d;
    d.K = p.K; d.Kp = p.Kp; d.J = p.J; d.S = p.S; d.H = p.H; d.W = p.W; d.L = p.L; d.P = p.P; d.P1 = p.P1;
    return d;
}

int ensure_tables(DevCtx* ctx) {
    if (ctx->tables) return RQ_OK;
    if (upload_tables()) return fail(RQ_ERR_DEVICE, "upload_tables failed");
    ctx->tables = true;
    return RQ_OK;
}

// Allocation options; RQHIP_ALLOC="v,a,la_load,la_reload,max_vmem,lds+1" overrides them for
// experiments (0 = keep the default; the sixth field is the LDS slot count plus one).
const AllocOpts& alloc_options() {
    static const AllocOpts o = [] {
        AllocOpts r;
        if (const char* e = knob("RQHIP_ALLOC")) {
            unsigned v[6] = {0, 0, 0, 0, 0, 0};
            std::sscanf(e, "%u,%u,%u,%u,%u,%u", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5]);
            if (v[5]) r.n_lds = std::min<uint32_t>(v[5] - 1, 512);
            if (v[0]) r.n_vgpr = std::min<uint32_t>(v[0], V_ALLOC);
            if (v[1]) r.n_agpr = std::min<uint32_t>(v[1], 256);
            if (v[2]) r.la_load = v[2];
            if (v[3]) r.la_reload = v[3];
            if (v[4]) r.max_vmem = std::min<uint32_t>(v[4], 60);
        }
        if (const char* h = knob("RQHIP_LDS_HORIZON")) r.lds_horizon = (uint32_t)std::atoi(h);
        if (const char* h = knob("RQHIP_LA_DMA")) r.la_dma = (uint32_t)std::atoi(h);
        if (const char* h = knob("RQHIP_SRC_BIAS")) r.src_bias = (uint32_t)std::atoi(h);
        if (const char* h = knob("RQHIP_SRC_LDS")) r.src_lds = (uint32_t)std::atoi(h);
        if (const char* h = knob("RQHIP_WAIT_AGE")) std::sscanf(h, "%u,%u", &r.wait_age, &r.lwait_age);
        if (const char* h = knob("RQHIP_LOAD_BATCH")) r.load_batch = (uint32_t)std::max(1, std::atoi(h));
        if (const char* h = knob("RQHIP_CIP")) std::sscanf(h, "%u,%u,%u,%u", &r.cip, &r.cip_batch, &r.cip_gap, &r.cip_agpr);
        if (const char* h = knob("RQHIP_LA_ADAPT")) std::sscanf(h, "%u,%u", &r.la_extra, &r.la_free);
        if (const char* h = knob("RQHIP_WG"))
            if (std::atoi(h) > 1) r.cip = 0;  // the prefetch is a single-wave-workgroup layout
        return r;
    }();
    return o;
}

// ---------------- on-disk cache of compiled column programs ----------------
// A column program is a pure function of (this library build, K', K, outputs, allocation options), so
// its code object and launch metadata are cached across processes under $RQHIP_CACHE_DIR (default
// $XDG_CACHE_HOME/rqhip or ~/.cache/rqhip; "0" disables).  The key hashes the library's own file
// bytes, so any rebuild starts a fresh cache.  Failures to read or write the cache only cost time.
uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

const std::string& cache_dir() {
    static const std::string d = [] {
        std::string r;
        if (const char* e = std::getenv("RQHIP_CACHE_DIR")) r = e;
        else if (const char* x = std::getenv("XDG_CACHE_HOME")) r = std::string(x) + "/rqhip";
        else if (const char* h = std::getenv("HOME")) r = std::string(h) + "/.cache/rqhip";
        if (r == "0") r.clear();
#ifdef RQHIP_EXPERIMENTS
        r.clear();  // experiment knobs change the generated code without changing the cache key
#endif
        return r;
    }();
    return d;
}

uint64_t library_hash() {
    static const uint64_t h = [] {
        Dl_info di;
        uint64_t x = 0;
        if (dladdr((const void*)&library_hash, &di) && di.dli_fname) {
            if (FILE* f = std::fopen(di.dli_fname, "rb")) {
                std::vector<char> buf(1 << 16);
                size_t n;
                x = 1469598103934665603ull;
                while ((n = std::fread(buf.data(), 1, buf.size(), f)) > 0) x = fnv1a(buf.data(), n, x);
                std::fclose(f);
            }
        }
        return x;
    }();
    return h;
}

struct CacheHdr {
    char magic[8];
    uint32_t n_out, n_slots, n_ins, waves_per_cu, name_len, n_rows, wg_waves, flags;  // flags bit 0: pair
    uint32_t n_dma4, row_end;  // four-row staging rows after the n_rows source-load rows; 1 + largest source row
    uint64_t co_len;
    MProg::Stats st;
    uint64_t body_hash;  // FNV-1a of the name, code object and row table (checked on load)
};
constexpr char CACHE_MAGIC[9] = "RQCO0009";

uint64_t cache_body_hash(const std::string& name, const std::vector<char>& co, const std::vector<uint32_t>& rows) {
    uint64_t h = fnv1a(name.data(), name.size());
    h = fnv1a(co.data(), co.size(), h);
    return fnv1a(rows.data(), rows.size() * 4, h);
}

bool cache_load(const std::string& path, CacheHdr* h, std::string* name, std::vector<char>* co,
                std::vector<uint32_t>* rows) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    bool ok = std::fread(h, sizeof *h, 1, f) == 1 && std::memcmp(h->magic, CACHE_MAGIC, 8) == 0 && h->name_len < 256 &&
              h->co_len < (1ull << 30) && h->n_rows < (1u << 24) && h->n_dma4 < (1u << 24);
    if (ok) {  // the source-load rows, then the four-row staging rows (cache_store writes both)
        const size_t nr = (size_t)h->n_rows + h->n_dma4;
        name->resize(h->name_len);
        co->resize(h->co_len);
        rows->resize(nr);
        ok = std::fread(&(*name)[0], 1, h->name_len, f) == h->name_len &&
             std::fread(co->data(), 1, h->co_len, f) == h->co_len &&
             std::fread(rows->data(), 4, nr, f) == nr;
    }
    std::fclose(f);
    // a torn or corrupted entry (the lengths can still look right) is dropped and rebuilt
    if (ok && cache_body_hash(*name, *co, *rows) != h->body_hash) ok = false;
    if (!ok) std::remove(path.c_str());
    return ok;
}

void cache_store(const std::string& path, const CacheHdr& h, const std::string& name, const std::vector<char>& co,
                 const std::vector<uint32_t>& rows) {
    ::mkdir(cache_dir().c_str(), 0755);
    // unique per process, thread and call: the per-device compiles of one process (run_sharded threads)
    // may miss on the same key at the same time
    static std::atomic<uint64_t> seq{0};
    const std::string tmp = path + ".tmp" + std::to_string(::getpid()) + "." +
                            std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id())) + "." +
                            std::to_string(seq++);
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(name.data(), 1, name.size(), f) == name.size() &&
                    std::fwrite(co.data(), 1, co.size(), f) == co.size() &&
                    std::fwrite(rows.data(), 4, rows.size(), f) == rows.size();
    std::fclose(f);
    if (ok) std::rename(tmp.c_str(), path.c_str());
    else std::remove(tmp.c_str());
}

// Waves per workgroup of a column program.  W = 4 at one wave per SIMD makes the four waves of a CU
// take four consecutive items, i.e. the four 256-B pieces of the same source rows (1 KiB): the
// memory-only pattern reads 4.87 -> 5.53 TB/s that way (tools/micro/sync_gen.py), but the full
// program measured the same for W = 1 / 2 / 4 (0.404-0.414 ms, profiles/r03e), so W = 1 stays the
// default; RQHIP_WG selects W in experiments builds (parity-tested at W = 4).
uint32_t colprog_wg_waves(uint32_t waves_per_cu, uint32_t lds_per_wave) {
    static const int forced = [] { const char* e = knob("RQHIP_WG"); return e ? std::atoi(e) : 0; }();
    uint32_t w = forced > 0 ? (uint32_t)forced : 1u;  // W = 4 measured neutral in the full program (r03e)
    while (w > 1 && (waves_per_cu % w || (uint64_t)lds_per_wave * w > 163840u)) w /= 2;
    return std::max<uint32_t>(1, w);
}

// Residency (waves per CU, from registers and LDS) of an allocated program; sets its waves per
// workgroup.  The engine and the debug entry points emit the same code.
uint32_t colprog_launch_shape(MProg* mp) {
    const uint32_t regs = colprog_regs(*mp), lds = (mp->lds_base + mp->n_lds_slots) * 256u;
    uint32_t w = 4 * std::max<uint32_t>(1, 512 / regs);
    if (lds) w = std::min<uint32_t>(w, 163840u / lds);
    const uint32_t wpc = std::max<uint32_t>(1, std::min<uint32_t>(w, 32));
    mp->wg_waves = colprog_wg_waves(wpc, lds);
    return wpc;
}

// ---------------- column programs (the encode hot path) ----------------
#ifdef RQHIP_EXPERIMENTS
// Two-wave (pair) column programs (rq_colasm.hpp compile_pair): wave A streams the source rows and runs
// the forward pass and pushes, wave B the HDPC bit accumulation, dense part and outputs, handed over
// through an LDS ring.  Taken for the bit-accumulation (SCHED_4R) programs, whose single wave is bound
// by its in-order issue behind the memory pipeline.  Experiments builds:
// RQHIP_PAIR=0/1 forces the choice; RQHIP_PAIR_CFG="lag,max_transfer,ring_max,quads,lookahead,hdpc_rows_on_A".
struct PairCfg {
    int mode = 0;  // -1 on where it compiles, 0 off, 1 forced (RQHIP_PAIR)
    uint32_t lag = 6, xfer = 16, ring = 192;
    uint32_t dma4 = 32, la_dma = 1200;  // wave A's four-row staging (quads, look-ahead); 16-B aligned rows only
    uint32_t ha = 0;  // HDPC rows whose bit accumulation wave A runs (SCHED_HA_SHIFT)
};
const PairCfg& pair_cfg() {
    static const PairCfg c = [] {
        PairCfg r;
        if (const char* e = knob("RQHIP_PAIR")) r.mode = std::atoi(e);
        if (const char* e = knob("RQHIP_PAIR_CFG")) {
            unsigned a = 0, b = 0, d = 0, q = 9999, la = 0, ha = 9999;
            std::sscanf(e, "%u,%u,%u,%u,%u,%u", &a, &b, &d, &q, &la, &ha);
            if (ha != 9999) r.ha = ha;
            if (a) r.lag = a;
            if (b) r.xfer = b;
            if (d) r.ring = d;
            if (q != 9999) r.dma4 = q;
            if (la) r.la_dma = la;
        }
        return r;
    }();
    return c;
}

// The program the engine runs for (K', outputs): the single-wave program of compile_colprog, or its
// pair split when that is chosen.  *use_pair says which; the debug entry points share this choice.
// Four-row staging in single-wave programs (16-B aligned rows, one-wave-per-SIMD programs): quads and
// look-ahead; RQHIP_DMA4="quads,lookahead" in experiments builds, off (0 quads) by default.
struct Dma4Cfg {
    uint32_t quads = 0, la = 1200;
};
const Dma4Cfg& dma4_cfg() {
    static const Dma4Cfg c = [] {
        Dma4Cfg r;
        if (const char* e = knob("RQHIP_DMA4")) {
            unsigned q = 0, la = 0;
            const int n = std::sscanf(e, "%u,%u", &q, &la);
            if (n >= 1) r.quads = q;
            if (n >= 2 && la) r.la = la;
        }
        return r;
    }();
    return c;
}
#endif  // RQHIP_EXPERIMENTS

// Whether a column program may differ with the caller's 16-B alignment (four-row staging, experiments).
bool staging_possible() {
#ifdef RQHIP_EXPERIMENTS
    return dma4_cfg().quads != 0 || pair_cfg().mode != 0;
#else
    return false;
#endif
}

bool compile_engine_program(const Params& p, const uint32_t* esi, uint32_t n_esi, const AllocOpts& ao,
                            bool search_waves, bool aligned16, ColIR* ir, MProg* mp, PairProg* pp, bool* use_pair,
                            std::string* err) {
    uint32_t passes = 0;
    *use_pair = false;
    if (!compile_colprog(p, esi, n_esi, ao, ir, mp, err, &passes, search_waves)) return false;
#ifndef RQHIP_EXPERIMENTS
    (void)aligned16; (void)pp;
    return true;
#else
    const Dma4Cfg& d4 = dma4_cfg();
    if (d4.quads && aligned16 && (passes & SCHED_4R) && mp->wg_waves <= 1) {
        MProg m4;
        std::string e2;
        if (compile_colprog_dma4(*ir, ao, d4.quads, d4.la, &m4, &e2) && m4.n_slots <= mp->n_slots) *mp = std::move(m4);
    }
    const PairCfg& c = pair_cfg();
    if (!esi || c.mode == 0 || !(passes & SCHED_4R)) return true;  // (mode 1 also needs the 4R schedule)
    std::string e2;
    AllocOpts pa = ao;
    pa.dma4 = aligned16 ? c.dma4 : 0;
    pa.la_dma = c.la_dma;
    ColIR irh;  // the first c.ha HDPC rows' bit accumulation on wave A (its own subset sums)
    if (c.ha && !build_colprog(p, esi, n_esi, &irh, &e2, passes | (c.ha << SCHED_HA_SHIFT))) {
        if (c.mode == 1) {
            if (err) *err = e2;
            return false;
        }
        return true;
    }
    if (!compile_pair(c.ha ? irh : *ir, pa, /*B: grp 1 and 3*/ 0xA, c.lag, c.xfer, c.ring, pp, &e2)) {
        if (c.mode == 1) {
            if (err) *err = e2;
            return false;
        }
        return true;
    }
    *use_pair = true;
    return true;
#endif
}

// Compile (once per device and (K', K, outputs)) the straight-line gfx950 program for the given
// outputs: IR (rq_colprog.cpp) -> registers/scratch (rq_colasm.cpp) -> assembly -> code object
// (amd_comgr, in process) -> hipModuleLoadData, or take the code object from the disk cache.
// Caller holds ctx->mu.
// aligned16: every launch of this program has T, the block stride and the base a multiple of 16 bytes
// (the four-row staging of pair programs reads 16-B chunks); a separate program otherwise.
int get_col_kernel(DevCtx* ctx, const Params& p, const uint32_t* esi, uint32_t n_esi, bool all_C, ColKernel** out,
                   bool aligned16 = false) {
    // the 16-B-aligned variant is a different program only where four-row staging could be chosen
    // (experiments builds with RQHIP_DMA4 / RQHIP_PAIR): elsewhere both alignments share one program
    const bool staged = staging_possible();
    std::string key = std::to_string(p.Kp) + ":" + std::to_string(p.K) + (all_C ? ":C" : ":E") + (aligned16 && staged ? "a" : "");
    if (!staged) aligned16 = false;
    if (!all_C) {
        key.reserve(key.size() + n_esi * 6);
        for (uint32_t i = 0; i < n_esi; ++i) key += "," + std::to_string(esi[i]);
    }
    constexpr size_t MAX_PROGRAMS = 48;  // loaded column programs per device (sparse decode unions)
    if (!ctx->colk.count(key) && ctx->colk.size() >= MAX_PROGRAMS) {
        auto victim = ctx->colk.begin();
        for (auto it = ctx->colk.begin(); it != ctx->colk.end(); ++it)
            if (it->second->last_use < victim->second->last_use) victim = it;
        (void)hipDeviceSynchronize();  // its kernels may still run on some stream: unload when idle
        ctx->colk.erase(victim);
    }
    auto& slot = ctx->colk[key];
    if (!slot) {
        std::unique_ptr<ColKernel> k(new ColKernel());
        k->p = p;
        if (!all_C) k->esi.assign(esi, esi + n_esi);
        const AllocOpts& ao = alloc_options();
        std::string path;
        if (!cache_dir().empty() && library_hash()) {
            uint64_t h = fnv1a(key.data(), key.size(), library_hash());
            h = fnv1a(&ao, sizeof ao, h);
            char hex[17];
            std::snprintf(hex, sizeof hex, "%016llx", (unsigned long long)h);
            path = cache_dir() + "/" + hex + ".co";
        }
        CacheHdr ch;
        std::string kname;
        std::vector<char> co;
        std::vector<uint32_t> rows;  // source-load rows, then the four-row groups' rows
        bool cached = !path.empty() && cache_load(path, &ch, &kname, &co, &rows);
        if (cached && (size_t)ch.n_rows + ch.n_dma4 == rows.size()) {
            k->src_rows.assign(rows.begin(), rows.begin() + ch.n_rows);
            k->dma4_rows.assign(rows.begin() + ch.n_rows, rows.end());
        } else if (cached) {
            cached = false;
        }
        if (cached && (hipModuleLoadData(&k->mod, co.data()) != hipSuccess ||
                       hipModuleGetFunction(&k->fn, k->mod, kname.c_str()) != hipSuccess)) {
            // a cached object the runtime refuses: drop the entry and build the program afresh
            (void)hipGetLastError();
            if (k->mod) (void)hipModuleUnload(k->mod);
            k->mod = nullptr;
            k->fn = nullptr;
            std::remove(path.c_str());
            cached = false;
        }
        if (!cached) {
            ColIR ir;
            std::string err;
            MProg mp;
            PairProg pp;
            bool pair = false;
            const bool search_waves = !knob("RQHIP_ALLOC");  // experiments: the given budget as is
            if (!compile_engine_program(p, all_C ? nullptr : esi, n_esi, ao, search_waves, aligned16, &ir, &mp, &pp, &pair,
                                        &err)) {
                ctx->colk.erase(key);
                return fail(RQ_ERR_PLAN, err);
            }
            // distinct symbol per program so kernel traces separate encode, decode and C programs
            kname = "rq_colprog_K" + std::to_string(p.K) + (all_C ? "_C" : "_n" + std::to_string(n_esi)) + (pair ? "_pair" : "");
            uint32_t wpc = 0;
            co.clear();
            if (pair) {
#ifdef RQHIP_EXPERIMENTS
                wpc = 4;  // two workgroups of two 512-register waves per CU (pair_lds_bytes <= 80 KiB)
                if (!comgr_assemble(emit_pair_asm(pp, kname), &co, &err)) { ctx->colk.erase(key); return fail(RQ_ERR_PLAN, err); }
#endif
            } else {
                wpc = colprog_launch_shape(&mp);
                if (!comgr_assemble(emit_colprog_asm(mp, kname), &co, &err)) { ctx->colk.erase(key); return fail(RQ_ERR_PLAN, err); }
            }
            const MProg& lead = pair ? pp.A : mp;  // the wave that loads the source rows
            std::memset(&ch, 0, sizeof ch);
            ch.waves_per_cu = wpc;
            std::memcpy(ch.magic, CACHE_MAGIC, 8);
            k->src_rows = colprog_src_rows(lead);
            k->dma4_rows = lead.dma4_rows;
            ch.n_rows = (uint32_t)k->src_rows.size();
            ch.n_dma4 = (uint32_t)k->dma4_rows.size();
            ch.row_end = colprog_row_end(lead);
            rows = k->src_rows;
            rows.insert(rows.end(), k->dma4_rows.begin(), k->dma4_rows.end());
            ch.n_out = ir.n_out;
            ch.n_slots = lead.n_slots;
            ch.n_ins = (uint32_t)(pair ? pp.A.ins.size() + pp.B.ins.size() : mp.ins.size());
            ch.wg_waves = pair ? 2 : mp.wg_waves;
            ch.flags = pair ? 1u : (mp.n_vgpr >= 24 ? 2u : 0u);  // 2: carries the descriptor fetch (rq_colasm.cpp)
            ch.name_len = (uint32_t)kname.size();
            ch.co_len = co.size();
            ch.st = lead.st;
            ch.body_hash = cache_body_hash(kname, co, rows);
            if (hipModuleLoadData(&k->mod, co.data()) != hipSuccess ||
                hipModuleGetFunction(&k->fn, k->mod, kname.c_str()) != hipSuccess) {
                ctx->colk.erase(key);
                return fail(RQ_ERR_DEVICE, "hipModuleLoadData/GetFunction failed for the column program");
            }
            if (!path.empty()) cache_store(path, ch, kname, co, rows);
        }
        k->n_out = ch.n_out;
        k->row_end = std::max<uint32_t>(ch.row_end, 1);
        k->n_slots = ch.n_slots;
        k->waves_per_cu = ch.waves_per_cu;
        k->wg_waves = std::max<uint32_t>(1, ch.wg_waves);
        k->pair = (ch.flags & 1u) != 0;
        k->fetch_ok = (ch.flags & 2u) != 0;
        k->st = ch.st;
        k->n_ins = ch.n_ins;
        slot = std::move(k);
    }
    slot->last_use = ++ctx->tick;
    *out = slot.get();
    return RQ_OK;
}

// XCD-aware wave order in column programs (RQHIP_XCD=0 disables it for experiments).
bool xcd_order() {
    static const bool on = [] {
        const char* e = knob("RQHIP_XCD");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Run a column program over n_blocks device-resident blocks.  Caller holds ctx->mu.
// A decode's descriptor fetch riding on its syndrome launch (ColKernArgs::cp_*): bytes (a multiple of
// kFetchQuantum, both buffers that large) from pinned host memory to the device.  `carried` reports
// whether the launch took it: only when its persistent grid leaves SIMDs free, so that the fetch runs
// beside the program instead of after it.
constexpr uint32_t kFetchQuantum = 16384;  // 4 KiB per wave and round trip, up to four waves per workgroup
struct DescFetch {
    const void* src = nullptr;  // the device's address of the pinned staging
    void* dst = nullptr;
    uint32_t bytes = 0;
    bool carried = false;
};

int launch_col(DevCtx* ctx, ColKernel* k, uint32_t T, uint32_t n_blocks, const void* src, uint64_t src_stride,
               void* out, uint64_t out_stride, void* stream, DescFetch* df = nullptr) {
    if (T < 8 || T % 4) return fail(RQ_ERR_BAD_ARG, "device-resident symbols: T must be a multiple of 4, at least 8");
    if (n_blocks == 0) return RQ_OK;
    if (!k->dma4_rows.empty() && (T % 16 || src_stride % 16 || (uintptr_t)src % 16))
        return fail(RQ_ERR_PLAN, "internal: a 16-B staged program launched on unaligned rows");
    const uint32_t Td = T / 4;
    // every buffer offset is 32-bit: split so that each launch spans < 4 GiB per buffer
    const uint64_t lim = 0xFFFFFFFFull - (uint64_t)std::max(k->p.K, k->n_out) * T;
    uint32_t per = n_blocks;
    while (per > 1 && ((uint64_t)per * src_stride > lim || (uint64_t)per * out_stride > lim)) per = (per + 1) / 2;
    if ((uint64_t)per * src_stride > lim || (uint64_t)per * out_stride > lim)
        return fail(RQ_ERR_UNSUPPORTED, "block stride beyond the 4 GiB buffer-offset range");
    if ((uint64_t)per * Td > 0x7FFFFFFFull) return fail(RQ_ERR_UNSUPPORTED, "batch too large");
    const uint32_t Wg = k->wg_waves;
    const uint32_t Wi = k->pair ? 1u : Wg;  // items per workgroup iteration (a pair's two waves share one)
    const uint32_t max_items = (uint32_t)(((uint64_t)per * Td + 63) / 64);
    const uint32_t max_iters = (max_items + Wi - 1) / Wi;  // workgroup iterations
    // persistent grid: at most the resident workgroup count (scratch is per grid wave; RQHIP_WAVES caps
    // the waves in experiments builds)
    static const uint32_t cap = [] { const char* e = knob("RQHIP_WAVES"); return e ? (uint32_t)std::atoi(e) : 0u; }();
    const uint32_t resident_w = cap ? std::min(cap, ctx->n_cu * k->waves_per_cu) : ctx->n_cu * k->waves_per_cu;
    const uint32_t resident = std::max<uint32_t>(1, resident_w / Wg);  // workgroups
    const uint32_t max_wg = std::min(max_iters, resident);
    const size_t spw = (size_t)std::max<uint32_t>(k->n_slots, 1) * 256;
    int rc;
    // A program with no global-scratch slot (K=1024 and below since round 3) touches no workspace: no
    // scratch buffer, and no `last` marker on the stream after it (each marker costs the stream a few
    // us between kernels, profiles/r04e).
    Workspace* w = nullptr;
    if (k->n_slots) {
        w = ctx->wsp(stream);
        if ((rc = w->scratch.ensure(spw * max_wg * Wi))) return rc;  // a pair's wave A alone uses scratch
    }
    MarkGuard mg{w, stream};
    auto& tab = k->row_off[T];
    if (!tab) {  // once per (program, T): the source loads' soffsets, padded to whole 16-entry groups
        std::unique_ptr<DevBuf> b(new DevBuf());
        std::vector<uint32_t> off((k->src_rows.size() + 15) / 16 * 16 + 16, 0);
        for (size_t j = 0; j < k->src_rows.size(); ++j) off[j] = k->src_rows[j] * T;
        for (uint32_t r : k->dma4_rows) off.push_back(r * T);  // colprog_row_table's layout
        if ((rc = b->ensure(off.size() * 4))) { k->row_off.erase(T); return rc; }
        if (hipMemcpy(b->p, off.data(), off.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            k->row_off.erase(T);
            return fail(RQ_ERR_DEVICE, "row-offset table upload failed");
        }
        tab = std::move(b);
    }
    for (uint32_t b0 = 0; b0 < n_blocks; b0 += per) {
        const uint32_t nb = std::min(per, n_blocks - b0);
        ColKernArgs a;
        std::memset(&a, 0, sizeof a);
        a.src = (uint64_t)(uintptr_t)src + (uint64_t)b0 * src_stride;
        a.out = (uint64_t)(uintptr_t)out + (uint64_t)b0 * out_stride;
        a.scratch = w ? (uint64_t)(uintptr_t)w->scratch.p : 0;
        a.src_stride = (uint32_t)src_stride;
        // the source resource's size: the launch's rows, so a wrong offset reads 0 instead of faulting
        a.src_bytes = (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, (uint64_t)(nb - 1) * src_stride + (uint64_t)k->row_end * T);
        a.out_stride = (uint32_t)out_stride;
        a.T = T;
        a.n_cols = nb * Td;
        a.scr_per_wave = (uint32_t)spw;
        a.row_off = (uint64_t)(uintptr_t)tab->p;
        if (!divmagic(Td, a.n_cols, &a.magic, &a.shift)) return fail(RQ_ERR_UNSUPPORTED, "no division magic");
        size_t sz = sizeof a;
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        const uint32_t items = (a.n_cols + 63) / 64, iters = (items + Wi - 1) / Wi;
        // Balanced rounds: as many workgroups as spread the iterations evenly over the rounds the
        // resident set needs (a multiple of 8 for the XCD remap), not the whole resident set with a
        // partial last round -- 1024 blocks K=1024 = 4 800 items: 960 waves x 5 instead of 704 x 5 +
        // 320 x 4, the busy waves then share HBM with fewer others (0.49 -> 0.47 ms, profiles/r02at).
        const uint32_t rounds = (iters + resident - 1) / resident;
        const uint32_t wgs = std::min(resident, ((iters + rounds - 1) / rounds + 7) / 8 * 8);
        a.n_items = iters;
        a.n_wg = wgs;
        // the descriptor fetch rides on the first launch when its grid leaves SIMDs free (64 at K=1024 x
        // 1 024 blocks): as many workgroups as free slots, up to one per 4 KiB x W round trip
        uint32_t n_cp = 0;
        const uint32_t free_wg = resident > wgs ? resident - wgs : 0u;
        const uint32_t per_trip = 4096u * Wg;
        if (df && df->bytes && b0 == 0 && free_wg && k->fetch_ok && df->bytes % per_trip == 0) {
            n_cp = std::min<uint32_t>(free_wg, (df->bytes + per_trip - 1) / per_trip);
            a.cp_src = (uint64_t)(uintptr_t)df->src;
            a.cp_dst = (uint64_t)(uintptr_t)df->dst;
            a.cp_bytes = df->bytes;
            const uint32_t trips = (df->bytes / per_trip + n_cp - 1) / n_cp;  // per workgroup
            a.cp_chunk = trips * per_trip;
            df->carried = true;
        }
#ifdef RQHIP_EXPERIMENTS
        // RQHIP_FETCH_LOG=1: the launch shape of a decode's syndrome launch (tests/test_gpu_experimental_programs.py
        // checks the fetch at W > 1 waves per workgroup, whose per-trip / chunk arithmetic W = 1 never exercises)
        static const bool fetch_log = knob("RQHIP_FETCH_LOG") != nullptr;
        if (fetch_log && df)
            std::fprintf(stderr, "[fetch] carried=%d W=%u wgs=%u resident=%u n_cp=%u bytes=%u chunk=%u\n", df->carried ? 1 : 0,
                         Wg, wgs, resident, n_cp, df->bytes, a.cp_chunk);
#endif
        if (xcd_order() && wgs % 8 == 0) {  // the remap needs the stride to keep g % 8 fixed
            a.xcd_q = iters / 8;
            a.xcd_n = a.xcd_q * 8;
        }
        if (ctx->timing) {  // measurement: the dispatch itself records the kernel's start / stop
            if (ctx->tev_used == ctx->tev.size()) {
                hipEvent_t e0, e1;
                HIP_TRY(hipEventCreate(&e0));
                if (hipEventCreate(&e1) != hipSuccess) {
                    (void)hipEventDestroy(e0);
                    return fail(RQ_ERR_DEVICE, "hipEventCreate failed");
                }
                ctx->tev.push_back({e0, e1});
            }
            const auto& pr = ctx->tev[ctx->tev_used++];
            mg.armed = w != nullptr;
            HIP_TRY(hipExtModuleLaunchKernel(k->fn, (wgs + n_cp) * 64 * Wg, 1, 1, 64 * Wg, 1, 1, 0, (hipStream_t)stream,
                                             nullptr, cfg, pr.first, pr.second, 0));
            continue;
        }
        mg.armed = w != nullptr;
        HIP_TRY(hipModuleLaunchKernel(k->fn, wgs + n_cp, 1, 1, 64 * Wg, 1, 1, 0, (hipStream_t)stream, nullptr, cfg));
    }
    mg.armed = false;
    return w ? w->mark(stream) : RQ_OK;
}

// Encode `n_blocks` device-resident blocks: outputs esi[0..n_esi) of every block.
int encode_locked(DevCtx* ctx, const Params& p, uint32_t T, uint32_t n_blocks, const void* src, uint64_t src_stride,
                  const uint32_t* esi, uint32_t n_esi, void* out, uint64_t out_stride, void* stream) {
    if (!n_esi || !n_blocks) return RQ_OK;
    ColKernel* k;
    const bool a16 = T % 16 == 0 && src_stride % 16 == 0 && (uintptr_t)src % 16 == 0;
    int rc = get_col_kernel(ctx, p, esi, n_esi, false, &k, a16);
    if (rc) return rc;
    return launch_col(ctx, k, T, n_blocks, src, src_stride, out, out_stride, stream);
}

// Decode output set (decode_pass): every candidate repair ESI the batch holds.  A dense range [K, K+R) (R a
// multiple of 4) when the received ESIs are not too sparse -- one compiled program then serves
// every erasure pattern of that range, and when the highest ESI received is the sender's last
// (N - 1, N - K a multiple of 4) it is the sender's own encode program -- otherwise the exact
// sorted set.
// Coefficients of every output over the source rows: the program on the identity payload.
int ensure_mrep(DevCtx* ctx, ColKernel* k, void* stream) {
    if (k->mrep_stride) return RQ_OK;
    const uint32_t K = k->p.K, Tid = (K + 15) & ~15u;  // 16-B rows: every program variant takes them
    std::vector<uint8_t> id((size_t)K * Tid, 0);
    for (uint32_t i = 0; i < K; ++i) id[(size_t)i * Tid + i] = 1;
    DevBuf src;
    int rc;
    if ((rc = src.ensure(id.size())) || (rc = k->mrep.ensure((size_t)k->n_out * Tid))) return rc;
    HIP_TRY(hipMemcpyAsync(src.p, id.data(), id.size(), hipMemcpyHostToDevice, (hipStream_t)stream));
    if ((rc = launch_col(ctx, k, Tid, 1, src.p, id.size(), k->mrep.p, (uint64_t)k->n_out * Tid, stream))) return rc;
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    k->mrep_stride = Tid;
    return RQ_OK;
}

// Optional decode output for host-memory batches: the recovered rows of `blocks` (the blocks that
// decoded, in the order they did; each block's erased rows in erased[] order), T bytes apart.
struct PackOut {
    std::vector<uint8_t> rows;
    std::vector<uint32_t> blocks;
};

// Synchronous decodes offer the solvers the first e + SUBSET_MARGIN received repairs of a block
// first: any e independent received rows determine x_E, so the subset changes no byte, and it keeps
// the column program's output set (and r0) small.  A block whose subset is rank-deficient while it
// received more repairs is solved again on all of them, so ok/fail matches the reference, which
// solves with every held symbol (RQ/decoder.go:93-121).
uint32_t g_subset_margin = 8;  // rq_debug_decode_margin lets the tests force the second pass

uint32_t lds_e_max() {
    static const uint32_t v = solve_lds_e_max();
    return v;
}

// How a decode pass ends: Sync waits and reads the statuses (and packed rows) back; Async leaves the
// statuses to land in the caller's pinned array; Deferred queues their download into the workspace
// and returns -- the caller syncs the stream and calls decode_collect.
enum class Fin { Sync, Async, Deferred };

// Statuses and packed recovered rows of a finished Sync / Deferred pass over blk_map (workspace w).
// With `sink`, each decoded block's rows go to sink(b, rows) straight from the pinned download
// instead of being copied into po.
using RowSink = std::function<void(uint32_t, const uint8_t*)>;
void decode_collect(const Workspace* w, const std::vector<uint32_t>& blk_map, const std::vector<uint32_t>& eoff,
                    uint32_t T, int32_t* status, PackOut* po, const RowSink* sink = nullptr) {
    const int32_t* st = static_cast<const int32_t*>(w->h_status.p);
    for (uint32_t b : blk_map) status[b] = st[b];
    if (!po && !sink) return;
    const uint8_t* rows = static_cast<const uint8_t*>(w->h_pack.p);
    size_t r = 0;
    for (uint32_t b : blk_map) {
        const size_t nb = (size_t)(eoff[b + 1] - eoff[b]) * T;
        if (status[b] == 1) {
            if (sink) {
                (*sink)(b, rows + r);
            } else {
                po->blocks.push_back(b);
                po->rows.insert(po->rows.end(), rows + r, rows + r + nb);
            }
        }
        r += nb;
    }
}

// Received repairs the first solver pass takes beyond e: k_solve_pm then carries e + 4 rows and as many
// identity columns instead of 64 (seven 16-byte quads per row at e ~ 51 instead of eight): 81.8 ->
// 77.0 us at 1 024 blocks (profiles/r03sm).  A block rank-deficient on those rows (~256^-5 for e ~ 51)
// goes to the general solver with every received repair.  Experiments builds: RQHIP_SOLVE_MARGIN
// (0 = the first 64).
uint32_t solve_row_margin() {
    static const uint32_t m = [] { const char* e = knob("RQHIP_SOLVE_MARGIN"); return e ? (uint32_t)std::atoi(e) : 4u; }();
    return m;
}

// Host side of one decode pass (bounded per call, nothing cached across calls -- a
// receiver sees a new erasure pattern per batch).  plan_decode: per-block offsets of X and of the
// general solver's workspace, the union of the candidate repair ESIs (a presence map, then a dense
// [K, K+R) range when the set is not too sparse), and the index-workspace layout.  fill_decode_idx:
// the descriptor words, written once, straight into the pinned staging the upload reads.  The vectors
// keep their capacity per thread between calls.
struct DecodePlan {
    uint32_t nw = 0, max_e = 0, max_lds_e = 0;
    bool need_general = false;  // some block may reach the general solver (e or candidates > 64)
    bool wide = false;          // some block has 64 < e <= 128
    uint64_t xo = 0, go = 0;    // X and general-workspace sizes (64-B units)
    size_t nz = 0;              // recovered rows to pack (host-memory decodes)
    uint32_t K = 0, mx = 0;
    bool mapped = false, dense_uni = false;
    std::vector<uint32_t> xoff, goff, uni, upos;
    std::vector<uint8_t> seen;
    // index workspace: blk_map | eoff | roff | cnt | erased | rep_uidx | status | xoff | goff
    // [| pack list (blk, row): host-memory decodes only]
    size_t o_map = 0, o_eoff = 0, o_roff = 0, o_cnt = 0, o_er = 0, o_ru = 0, o_st = 0, o_xo = 0, o_go = 0, o_zb = 0,
           o_zr = 0, n_idx = 0;
};

DecodePlan& decode_plan_scratch() {
    static thread_local DecodePlan pl;
    return pl;
}

// mx_hint: the largest candidate ESI when the caller knows it (every block offers all its received
// repairs: the argument check's maximum), else 0.
int plan_decode(const Params& p, uint32_t n_blocks, const std::vector<uint32_t>& eoff, const std::vector<uint32_t>& roff,
                const uint32_t* repair_esi, const std::vector<uint32_t>& cnt, const std::vector<uint32_t>& blk_map,
                bool pack, DecodePlan* pl, uint32_t mx_hint = 0) {
    const uint32_t nw = (uint32_t)blk_map.size();
    pl->nw = nw;
    pl->max_e = pl->max_lds_e = 0;
    pl->need_general = pl->wide = false;
    pl->xoff.resize(nw);
    pl->goff.resize(nw);
    uint64_t xo = 0, go = 0;
    uint32_t mx = 0;
    size_t n_cand = 0, nz = 0;
    const uint32_t lds_max = lds_e_max(), margin = solve_row_margin();
    for (uint32_t bi = 0; bi < nw; ++bi) {
        const uint32_t b = blk_map[bi], e = eoff[b + 1] - eoff[b];
        pl->max_e = std::max(pl->max_e, e);
        if (e <= lds_max) pl->max_lds_e = std::max(pl->max_lds_e, e);
        pl->need_general |= (e > 64 || cnt[b] > std::min<uint32_t>(64, e + margin));
        pl->wide |= (e > 64 && e <= 128);
        if (!mx_hint) {
            const uint32_t* x = repair_esi + roff[b];
            uint32_t m = 0;
            for (uint32_t i = 0; i < cnt[b]; ++i) m = std::max(m, x[i]);
            mx = std::max(mx, m);
        }
        n_cand += cnt[b];
        nz += e;
        pl->xoff[bi] = (uint32_t)xo;
        xo += ((uint64_t)e * x_stride(e) + 63) / 64;
        pl->goff[bi] = (uint32_t)go;
        if (e > lds_max) go += (solve_ws_bytes(e) + 63) / 64;
    }
    if (xo >= (1ull << 32) || go >= (1ull << 32)) return fail(RQ_ERR_UNSUPPORTED, "decode workspace beyond 256 GiB");
    pl->xo = xo;
    pl->go = go;
    if (mx_hint) mx = mx_hint;
    const uint32_t K = p.K;
    pl->K = K;
    pl->mx = mx;
    pl->mapped = n_cand && (uint64_t)mx - K < (1u << 22);
    auto& uni = pl->uni;
    uni.clear();
    // The rule below makes the union the dense range [K, K + span) when span <= 4 |union| + 64.  The
    // distinct candidates of the block that offers the most are a lower bound on |union|: when that
    // bound already satisfies the rule, the presence pass over every candidate is skipped (same union).
    bool dense_known = false;
    if (pl->mapped) {
        uint32_t bmax = blk_map[0];
        for (uint32_t b : blk_map)
            if (cnt[b] > cnt[bmax]) bmax = b;
        pl->seen.assign((size_t)(mx - K) + 1, 0);
        uint8_t* seen = pl->seen.data();
        uint32_t lb = 0;
        for (uint32_t i = 0; i < cnt[bmax]; ++i) {
            const uint32_t v = repair_esi[roff[bmax] + i] - K;
            lb += !seen[v];
            seen[v] = 1;
        }
        const uint64_t span = ((uint64_t)mx - K + 4) & ~(uint64_t)3;
        if (span <= 4ull * lb + 64) {
            uni.resize((size_t)span);
            for (uint32_t i = 0; i < span; ++i) uni[i] = K + i;
            dense_known = true;
        }
    }
    if (dense_known) {
    } else if (pl->mapped) {
        pl->seen.assign((size_t)(mx - K) + 1, 0);
        uint8_t* seen = pl->seen.data();
        for (uint32_t b : blk_map) {
            const uint32_t* x = repair_esi + roff[b];
            for (uint32_t i = 0; i < cnt[b]; ++i) seen[x[i] - K] = 1;
        }
        for (size_t i = 0; i < pl->seen.size(); ++i)
            if (seen[i]) uni.push_back(K + (uint32_t)i);
    } else {
        for (uint32_t b : blk_map) uni.insert(uni.end(), repair_esi + roff[b], repair_esi + roff[b] + cnt[b]);
        std::sort(uni.begin(), uni.end());
        uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
    }
    if (!uni.empty() && !dense_known) {
        const uint64_t span = ((uint64_t)uni.back() - K + 4) & ~(uint64_t)3;
        if (span <= 4 * uni.size() + 64) {
            uni.resize((size_t)span);
            for (uint32_t i = 0; i < span; ++i) uni[i] = K + i;
        }
    }
    // union index of every candidate repair: direct for a dense union, a table for a mapped one,
    // binary search otherwise
    pl->dense_uni = !uni.empty() && uni.back() - uni.front() + 1 == uni.size();
    if (!pl->dense_uni && pl->mapped) {
        pl->upos.assign((size_t)(mx - K) + 1, 0);
        for (uint32_t j = 0; j < uni.size(); ++j) pl->upos[uni[j] - K] = j;
    }
    const size_t n_er = eoff[n_blocks], n_rep = roff[n_blocks];
    if (!pack) nz = 0;
    pl->nz = nz;
    pl->o_map = 0;
    pl->o_eoff = pl->o_map + nw;
    pl->o_roff = pl->o_eoff + n_blocks + 1;
    pl->o_cnt = pl->o_roff + n_blocks + 1;
    pl->o_er = pl->o_cnt + n_blocks;
    pl->o_ru = pl->o_er + n_er;
    pl->o_st = pl->o_ru + n_rep;
    pl->o_xo = pl->o_st + n_blocks;
    pl->o_go = pl->o_xo + nw;
    pl->o_zb = pl->o_go + nw;
    pl->o_zr = pl->o_zb + nz;
    pl->n_idx = pl->o_zr + nz;
    return RQ_OK;
}

void fill_decode_idx(const DecodePlan& pl, uint32_t n_blocks, const std::vector<uint32_t>& eoff, const uint32_t* erased,
                     const std::vector<uint32_t>& roff, const uint32_t* repair_esi, const std::vector<uint32_t>& cnt,
                     const std::vector<uint32_t>& blk_map, const int32_t* status, uint32_t* I) {
    const uint32_t nw = pl.nw;
    const size_t n_er = eoff[n_blocks];
    std::memcpy(I + pl.o_map, blk_map.data(), nw * 4);
    std::memcpy(I + pl.o_eoff, eoff.data(), (n_blocks + 1) * 4);
    std::memcpy(I + pl.o_roff, roff.data(), (n_blocks + 1) * 4);
    std::memcpy(I + pl.o_cnt, cnt.data(), n_blocks * 4);
    if (n_er) std::memcpy(I + pl.o_er, erased, n_er * 4);
    // union indices of the mapped blocks' candidates (the kernels read no other block's entries)
    uint32_t* u = I + pl.o_ru;
    for (uint32_t b : blk_map) {
        const uint32_t* x = repair_esi + roff[b];
        uint32_t* ub = u + roff[b];
        const uint32_t n = cnt[b];
        if (pl.dense_uni) {
            const uint32_t f = pl.uni.front();
            for (uint32_t i = 0; i < n; ++i) ub[i] = x[i] - f;
        } else if (pl.mapped) {
            const uint32_t K = pl.K;
            for (uint32_t i = 0; i < n; ++i) ub[i] = pl.upos[x[i] - K];
        } else {
            for (uint32_t i = 0; i < n; ++i)
                ub[i] = (uint32_t)(std::lower_bound(pl.uni.begin(), pl.uni.end(), x[i]) - pl.uni.begin());
        }
    }
    // device status: host-decided values, ST_PENDING for the rest
    std::memcpy(I + pl.o_st, status, n_blocks * 4);
    std::memcpy(I + pl.o_xo, pl.xoff.data(), nw * 4);
    std::memcpy(I + pl.o_go, pl.goff.data(), nw * 4);
    if (pl.nz) {  // recovered rows packed densely for the download, in blk_map order
        uint32_t* zb = I + pl.o_zb;
        uint32_t* zr = I + pl.o_zr;
        for (uint32_t b : blk_map)
            for (uint32_t i = eoff[b]; i < eoff[b + 1]; ++i) {
                *zb++ = b;
                *zr++ = erased[i];
            }
    }
}

// One solve pass over the blocks of `blocks` (each pending; cnt[b] = candidate repairs offered).
// Caller holds ctx->mu.  Host arrays as in rq_decode_desc.
// Decode solve beside the syndrome program (decode_pass); RQHIP_SOLVE_BESIDE=0/1 in experiments builds.
bool solve_beside() {
    static const bool on = [] {
        const char* e = knob("RQHIP_SOLVE_BESIDE");
        return e ? e[0] == '1' : false;
    }();
    return on;
}

// The decode's apply: 1 = the register-table kernel (rq_applygi.cpp, k_xbits + the generated kernel),
// 0 = k_apply's v_perm byte tables.  rq_debug_apply_mode switches it (tests compare the two).
uint32_t g_apply_mode = 1;
// 1: the register-table apply reads syndromes precomputed beside the first solver (GiShape::SX; experiments
// library only, RQHIP_APPLY_SX=1 or rq_debug_apply_sx: measured not to pay).
uint32_t g_apply_sx = knob("RQHIP_APPLY_SX") && knob("RQHIP_APPLY_SX")[0] == '1' ? 1u : 0u;
// Stream bound of the register-table apply: e <= kGiMaxE and the whole stream of the solve
// list <= kGiMaxBytes.  Within it every byte offset the kernel forms (block base, slice records, their
// one-pair prefetch) stays far below 2^32 and the allocation stays small; config 3 (e ~ 60) needs 27 MB.
constexpr uint32_t kGiMaxE = 512;
constexpr uint64_t kGiMaxBytes = 512ull << 20;
bool gi_stream_fits(uint32_t max_e, uint32_t n_solve, const GiShape& sh) {
    if (max_e > kGiMaxE) return false;
    const GiLayout gl = gi_layout(max_e, sh);
    return (uint64_t)n_solve * gl.block * 4 + 4096 <= kGiMaxBytes;
}

// The register-table apply's shape: KC = 8 outputs per wave, groups of G = 5 syndromes, loads two groups
// ahead, one dword column per lane (120 VGPRs: four waves per SIMD); RQHIP_APPLY_GI="KC,G,PDG[,CPL]" in
// experiments builds.
const GiShape& apply_gi_shape() {
    static const GiShape sh = [] {
        GiShape g;
        if (const char* e = knob("RQHIP_APPLY_GI")) {
            unsigned kc = 0, gg = 0, pd = 0, cpl = 1, pk = 0;
            if (std::sscanf(e, "%u,%u,%u,%u,%u", &kc, &gg, &pd, &cpl, &pk) >= 3) {
                GiShape t;
                t.KC = kc; t.G = gg; t.PDG = pd; t.CPL = cpl; t.PACK = pk;
                if (gi_shape_ok(t)) g = t;
            }
        }
        if (const char* d = knob("RQHIP_APPLY_DIAG")) g.diag = (uint32_t)std::atoi(d);
        if (const char* d = knob("RQHIP_APPLY_STPOL")) g.stpol = (uint32_t)std::atoi(d) & 3u;
        return g;
    }();
    return sh;
}

// The apply kernel of this device, assembled (amd_comgr, in process) on first use.  Caller holds ctx->mu.
int get_gi_kernel(DevCtx* ctx, const GiShape& sh, hipFunction_t* fn) {
    const uint32_t slot = sh.SX ? 1 : 0;
    const GiShape& have = ctx->gi_shape[slot];
    if (ctx->gi_fn[slot] && have.KC == sh.KC && have.G == sh.G && have.PDG == sh.PDG && have.CPL == sh.CPL &&
        have.PACK == sh.PACK && have.diag == sh.diag && have.stpol == sh.stpol) {
        *fn = ctx->gi_fn[slot];
        return RQ_OK;
    }
    std::vector<char> co;
    std::string err;
    const std::string src = emit_apply_gi_asm(sh);
    if (!check_apply_gi_asm(src, sh, &err) || !comgr_assemble(src, &co, &err)) return fail(RQ_ERR_PLAN, err);
    hipModule_t mod = nullptr;
    hipFunction_t f = nullptr;
    if (hipModuleLoadData(&mod, co.data()) != hipSuccess ||
        hipModuleGetFunction(&f, mod, gi_kernel_name(sh).c_str()) != hipSuccess) {
        if (mod) (void)hipModuleUnload(mod);
        return fail(RQ_ERR_DEVICE, "apply kernel load failed");
    }
    if (ctx->gi_mod[slot]) (void)hipModuleUnload(ctx->gi_mod[slot]);  // a shape change (experiments): idle by then
    ctx->gi_mod[slot] = mod;
    ctx->gi_fn[slot] = f;
    ctx->gi_shape[slot] = sh;
    *fn = f;
    return RQ_OK;
}

int decode_pass(DevCtx* ctx, const Params& p, uint32_t T, uint32_t n_blocks, void* data, uint64_t data_stride,
                const std::vector<uint32_t>& eoff, const uint32_t* erased, const std::vector<uint32_t>& roff,
                const uint32_t* repair_esi, const std::vector<uint32_t>& cnt, const std::vector<uint32_t>& blk_map,
                const void* repair, int32_t* status, void* stream, PackOut* po, Fin fin, uint32_t mx_hint = 0,
                int32_t* status_dev = nullptr) {
    int rc;
    const bool async = fin == Fin::Async;
    DecodePlan& pl = decode_plan_scratch();
    const GiShape& gsh = apply_gi_shape();
    if ((rc = plan_decode(p, n_blocks, eoff, roff, repair_esi, cnt, blk_map, po != nullptr, &pl, mx_hint))) return rc;
    const uint32_t nw = pl.nw, max_e = pl.max_e, max_lds_e = pl.max_lds_e;
    // The register-table apply's stream is laid out for the batch's largest e (~1.6 e^2 dwords per block
    // and the kernel's slice offsets in 32 bits): it runs only while the whole stream stays within
    // gi_stream_fits' bound; a batch beyond it (one block with e in the thousands) takes k_apply, whose
    // working set is e x 64 bytes of X per block.
    const bool gi = g_apply_mode == 1 && gi_stream_fits(max_e, nw, gsh);
    // Precomputed syndromes (GiShape::SX, experiments library): the first solver launch's extra workgroups
    // XOR the received rows into the r0 rows beside the solves, and the apply loads one row per syndrome.
    // Needs the r0 rows final before the solver (not the solve beside the syndrome program), 16-byte rows
    // and a 16-byte aligned received-row buffer.  Apply -13 us, but the solve +5..27 us and the next
    // column-program launch +5..8 us (profiles/r06_sx): off, and absent from the release library.
    const bool want_sx = gi && g_apply_sx && T % 16 == 0 && (reinterpret_cast<uintptr_t>(repair) & 15) == 0;
    GiShape gsx = gsh;
    gsx.SX = 1;
    hipFunction_t gi_fn = nullptr, gi_fn_sx = nullptr;
    if (gi && (rc = get_gi_kernel(ctx, gsh, &gi_fn))) return rc;
    if (want_sx && (rc = get_gi_kernel(ctx, gsx, &gi_fn_sx))) return rc;
    const bool need_general = pl.need_general, wide = pl.wide;
    const uint64_t xo = pl.xo, go = pl.go;
    const size_t nz = pl.nz;
    const std::vector<uint32_t>& uni = pl.uni;
    ColKernel* k;
    const bool a16 = T % 16 == 0 && data_stride % 16 == 0 && (uintptr_t)data % 16 == 0;
    if ((rc = get_col_kernel(ctx, p, uni.data(), (uint32_t)uni.size(), false, &k, a16))) return rc;
    if ((rc = ensure_mrep(ctx, k, stream))) return rc;
    const size_t n_er = eoff[n_blocks];
    const size_t o_map = pl.o_map, o_eoff = pl.o_eoff, o_er = pl.o_er, o_ru = pl.o_ru, o_st = pl.o_st,
                 o_xo = pl.o_xo, o_go = pl.o_go, o_zb = pl.o_zb, o_zr = pl.o_zr, n_idx = pl.n_idx;
    const size_t o_roff = pl.o_roff, o_cnt = pl.o_cnt;
    auto fill_idx = [&](uint32_t* I) { fill_decode_idx(pl, n_blocks, eoff, erased, roff, repair_esi, cnt, blk_map, status, I); };
    // descriptors through pinned staging, without blocking this thread.  (An upload on a copy stream
    // of its own, joined by events, measured 0.25 ms slower per rq_decode_batch_async call, r02u.)
    Workspace* w = ctx->wsp(stream);
    const uint32_t set = w->flip++ & 1u;
    if (!w->up[0]) {
        for (int i = 0; i < 2; ++i) {  // only says the device finished reading the pinned staging:
            // no system-scope release (cache writeback) needed
            HIP_TRY(hipEventCreateWithFlags(&w->up[i], hipEventDisableTiming | hipEventDisableSystemFence));
        }
    }
    // The kernels read the descriptors straight from the pinned staging over PCIe (zero copy): no
    // H2D copy of ~0.5 MB sits in the stream between the caller's previous work and the solve (the
    // statuses alone go to the device); `up` then marks the end of the call's kernels.  Measured
    // 1-2 % faster per step than the in-stream copy (profiles/r02aa; RQHIP_DEC_ZC=0 restores it in
    // experiments builds).
    // Descriptor mode (RQHIP_DEC_ZC in experiments builds): 3 = fetched from the pinned staging by spare
    // workgroups of the syndrome launch (the default), 2 = side-stream upload, 1 = zero copy, 0 =
    // in-stream upload.  Measured at 1 024 blocks K=1024 (profiles/r03_solve2): zero copy leaves the
    // solve and the apply reading every descriptor over PCIe (solve 77 us, apply 188) against 58 / 176
    // us from device memory, but an in-stream upload costs more than that before the solve (decode
    // 0.663 against 0.647 ms); the side stream's copy runs beside the syndrome program but the caller's
    // stream then waits for it across queues (~6 us before the solve, profiles/r05n).  The fetch runs
    // beside the program as well, on the SIMDs its persistent grid leaves free, and needs no wait.
    static const int desc_mode = [] { const char* e = knob("RQHIP_DEC_ZC"); return e ? std::atoi(e) : 3; }();
    const bool zero_copy = desc_mode != 0;  // statuses in dstatus, `up` after the last kernel
    const bool fetch = desc_mode == 3 && !k->pair;  // (the two-wave programs carry no fetch)
    const bool side = desc_mode == 2 || (desc_mode == 3 && !fetch);
    const size_t idx_bytes = (n_idx * 4 + kFetchQuantum - 1) / kFetchQuantum * kFetchQuantum;  // fetch granularity
    if ((side || fetch) && !w->cs) {  // events first: a half-built pair is destroyed, never published
        // (the fetch falls back to the side-stream upload when the syndrome launch's grid is full)
        hipEvent_t ev[2] = {nullptr, nullptr};
        hipStream_t cs = nullptr;
        bool ok = hipEventCreateWithFlags(&ev[0], internal_event_flags()) == hipSuccess &&
                  hipEventCreateWithFlags(&ev[1], internal_event_flags()) == hipSuccess &&
                  hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) == hipSuccess;
        if (!ok) {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
            return fail(RQ_ERR_DEVICE, "side-stream setup failed");
        }
        w->cpy[0] = ev[0];
        w->cpy[1] = ev[1];
        w->cs = cs;
    }
    // the set's staging and (zero copy / side upload) its device copy were last read by call n - 2's
    // kernels, which precede `up[set]`
    HIP_TRY(hipEventSynchronize(w->up[set]));
    if ((rc = w->h_idx[set].ensure(idx_bytes)) || (rc = w->h_status.ensure((size_t)n_blocks * 4))) return rc;
    if (w->idx[set].cap < idx_bytes || w->dstatus.cap < (size_t)n_blocks * 4)
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // realloc: idle
    if ((rc = w->idx[set].ensure(idx_bytes))) return rc;
    fill_idx(w->h_idx[set].as<uint32_t>());
    const uint32_t* di;
    int32_t* dst_status;
    // An error return after the side copy is queued must still leave `up[set]` behind that copy (and
    // whatever this call queued after it): the call that reuses the set two calls later rewrites its
    // pinned staging once `up[set]` completes.
    struct UpGuard {
        Workspace* w = nullptr;
        hipStream_t s = nullptr;
        uint32_t set = 0;
        bool side = false;
        bool armed = false;
        ~UpGuard() {
            if (!armed) return;
            if (side) (void)hipStreamWaitEvent(s, w->cpy[set], 0);
            (void)hipEventRecord(w->up[set], s);
        }
    } up_guard{w, (hipStream_t)stream, set, side, false};
    DescFetch df;
    MarkGuard mark_guard{w, stream};
    if (side) {
        if ((rc = w->dstatus.ensure((size_t)n_blocks * 4))) return rc;
        mark_guard.armed = true;
        HIP_TRY(hipMemcpyAsync(w->idx[set].p, w->h_idx[set].p, n_idx * 4, hipMemcpyHostToDevice, w->cs));
        up_guard.armed = true;
        HIP_TRY(hipEventRecord(w->cpy[set], w->cs));
        di = w->idx[set].as<uint32_t>();
        dst_status = w->dstatus.as<int32_t>();  // the host-decided statuses: copied by the first solver
    } else if (fetch) {
        if ((rc = w->dstatus.ensure((size_t)n_blocks * 4))) return rc;
        void* hdev = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&hdev, w->h_idx[set].p, 0));
        df.src = hdev;
        df.dst = w->idx[set].p;
        df.bytes = (uint32_t)idx_bytes;
        mark_guard.armed = true;
        up_guard.armed = true;  // the syndrome launch reads the staging: `up[set]` after it on any return
        di = w->idx[set].as<uint32_t>();
        dst_status = w->dstatus.as<int32_t>();  // the host-decided statuses: copied by the first solver
    } else if (zero_copy) {
        if ((rc = w->dstatus.ensure((size_t)n_blocks * 4))) return rc;
        di = static_cast<const uint32_t*>(w->h_idx[set].p);
        dst_status = w->dstatus.as<int32_t>();  // the host-decided statuses: copied by the first solver
    } else {
        HIP_TRY(hipMemcpyAsync(w->idx[set].p, w->h_idx[set].p, n_idx * 4, hipMemcpyHostToDevice,
                               (hipStream_t)stream));
        HIP_TRY(hipEventRecord(w->up[set], (hipStream_t)stream));
        di = w->idx[set].as<uint32_t>();
        dst_status = reinterpret_cast<int32_t*>(w->idx[set].as<uint32_t>() + o_st);
    }
    if ((rc = w->r0.ensure((size_t)n_blocks * uni.size() * T))) return rc;
    mark_guard.armed = true;  // the kernels below read and write this workspace's buffers
    if ((rc = w->xb.ensure((size_t)xo * 64))) return rc;
    if ((rc = w->xp.ensure(std::max<size_t>(n_er, 1) * 2))) return rc;
    if (go && (rc = w->gws.ensure((size_t)go * 64))) return rc;
    // the apply's stream (fixed layout by the largest e) + slack: a slice's last group prefetches one
    // index pair past its records
    const GiLayout gl = gi_layout(max_e, gsh);
    if (gi && (rc = w->gi.ensure((size_t)nw * gl.block * 4 + 4096))) return rc;
    // The solve reads only the descriptors and M (the program's repair-coefficient matrix), not the
    // syndromes: it can run on the side stream beside the syndrome program, which leaves SIMDs and
    // LDS free (960 one-wave workgroups on 1 024 SIMDs at K=1024).  The side stream first waits for
    // this call's start on the caller's stream (`go`: the previous call's apply and downloads have
    // finished with X, the statuses and the workspace); the apply waits for `solved`.
    const bool beside = side && solve_beside();
    if (beside && !w->go) {
        hipEvent_t ev[2] = {nullptr, nullptr};
        if (hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
            return fail(RQ_ERR_DEVICE, "side-stream events failed");
        }
        w->go = ev[0];
        w->solved = ev[1];
    }
    if (beside) {
        HIP_TRY(hipEventRecord(w->go, (hipStream_t)stream));
        HIP_TRY(hipStreamWaitEvent(w->cs, w->go, 0));
    }

    // 1) r0 = the column program on every block, erased rows as they are (whatever bytes g_E they
    //    hold): the syndromes s = r ^ r0 = M (x_E ^ g_E), and k_apply starts each output from g_E
    PackArgs z;
    z.blk = di + o_zb; z.row = di + o_zr; z.data = static_cast<uint8_t*>(data); z.data_stride = data_stride;
    z.T = T; z.n = nz; z.pack = nullptr;
    // 2) per-block solve (after the side stream's descriptor upload): on the side stream, or after the
    //    syndrome program on the caller's
    // The caller's stream waits for the upload either before the syndrome program (RQHIP_DESC_WAIT=1 in
    // experiments builds: the upload has long finished by then, the wait is the queue's barrier packet)
    // or between it and the solve (the default).
    static const bool wait_early = [] { const char* e = knob("RQHIP_DESC_WAIT"); return e && e[0] == '1'; }();
    if (side && !beside && wait_early) HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, w->cpy[set], 0));
    if (!beside && (rc = launch_col(ctx, k, T, n_blocks, data, data_stride, w->r0.p, (uint64_t)uni.size() * T, stream,
                                    fetch ? &df : nullptr)))
        return rc;
    if (side && !beside && !wait_early) HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, w->cpy[set], 0));
    if (fetch && !df.carried) {  // no SIMD free beside the program: the upload on the side stream instead
        HIP_TRY(hipMemcpyAsync(w->idx[set].p, w->h_idx[set].p, n_idx * 4, hipMemcpyHostToDevice, w->cs));
        up_guard.side = true;
        HIP_TRY(hipEventRecord(w->cpy[set], w->cs));
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, w->cpy[set], 0));
    }
    SolveArgs s;
    s.blk_map = di + o_map;
    s.erased_off = di + o_eoff;
    s.erased = di + o_er;
    s.rep_off = di + o_roff;
    s.rep_cnt = di + o_cnt;
    s.rep_uidx = di + o_ru;
    s.mrep = k->mrep.as<uint8_t>();
    s.mrep_stride = k->mrep_stride;
    s.xcoef = w->xb.as<uint8_t>();
    s.xoff = di + o_xo;
    s.xpiv = w->xp.as<uint16_t>();
    s.status = dst_status;
    s.gws = w->gws.as<uint8_t>();
    s.goff = di + o_go;
    s.lds_e = lds_e_max();
    s.status_init = zero_copy ? reinterpret_cast<const int32_t*>(di + o_st) : nullptr;
    s.n_all = n_blocks;
    s.row_margin = solve_row_margin();
    s.n_map = nw;
    s.diag_steps = 0;
    s.diag = 0;
    // no block beyond the first solver's 64 rows: it finishes every block itself (launch_solve clears this
    // for the experiments variants)
    static const bool inl_off = [] { const char* e = knob("RQHIP_SOLVE_INLINE"); return e && e[0] == '0'; }();
    s.inline_general = max_e <= 64 && !inl_off ? 1u : 0u;
    // the register-table apply's index stream: written by the solvers (below), else k_xbits after them
    XbitsArgs xa{};
    if (gi) {
        xa.blk_map = s.blk_map;
        xa.status = s.status;
        xa.erased_off = s.erased_off;
        xa.erased = s.erased;
        xa.rep_off = s.rep_off;
        xa.rep_uidx = s.rep_uidx;
        xa.xcoef = s.xcoef;
        xa.xoff = s.xoff;
        xa.xpiv = s.xpiv;
        xa.recv = static_cast<const uint8_t*>(repair);
        xa.r0 = w->r0.as<uint8_t>();
        xa.data = static_cast<uint8_t*>(data);
        xa.data_stride = data_stride;
        xa.gi = w->gi.as<uint32_t>();
        xa.L = gl;
        xa.T = T;
        xa.n_union = (uint32_t)uni.size();
    }
    // The solvers write it for the shipped shape as they finish each block (k_solve_pq from its rows in
    // LDS, k_solve from the X it wrote); k_solve's grid doing all blocks after its own solves measured
    // 17.6 us against 4.7 + 8.5 us for k_solve and k_xbits apart (256 LDS-heavy workgroups, four blocks
    // each, one after another).
    const GiShape shipped;
    s.xb_on = gi && max_e && gsh.KC == shipped.KC && gsh.G == shipped.G && gsh.PDG == shipped.PDG &&
                      gsh.PACK == shipped.PACK ? 1u : 0u;
    s.xb = xa;
    // An async call whose status array the device can write (rq_decode_batch_async's pinned array) gets
    // its statuses from k_solve, the last solver launch, instead of a download after the apply (a copy
    // kernel and its gap, ~8 us per call).  Without the general solver the download stays.
    const bool status_by_solver = async && status_dev && need_general && !po;
    s.host_status = status_by_solver ? status_dev : nullptr;
    // two blocks per syndrome workgroup: two such workgroups per CU run beside the four solving ones
    static const uint32_t sx_cap = [] { const char* e = knob("RQHIP_SX_WGS"); return e ? (uint32_t)std::max(1, std::atoi(e)) : 512u; }();
    static const uint32_t sx_pol = [] { const char* e = knob("RQHIP_SX_POL"); return e ? (uint32_t)std::atoi(e) & 31u : 0u; }();
    s.sx_wgs = want_sx && !beside && nw && max_e ? std::min<uint32_t>(sx_cap, (nw + 1) / 2) : 0u;
    s.sx_pol = sx_pol;
    bool xbits_done = false, sx_done = false;
    if (launch_solve(s, nw, need_general, wide, max_lds_e, beside ? (void*)w->cs : stream, &xbits_done, &sx_done))
        return fail(RQ_ERR_DEVICE, "k_solve launch failed");
    if (sx_done) gi_fn = gi_fn_sx;  // the r0 rows hold the syndromes now
    if (beside) {
        HIP_TRY(hipEventRecord(w->solved, w->cs));
        if ((rc = launch_col(ctx, k, T, n_blocks, data, data_stride, w->r0.p, (uint64_t)uni.size() * T, stream)))
            return rc;
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, w->solved, 0));
    }
    // 3) apply: x_E = X * s
    ApplyArgs ap;
    ap.blk_map = di + o_map;
    ap.erased_off = di + o_eoff;
    ap.erased = di + o_er;
    ap.rep_off = di + o_roff;
    ap.rep_uidx = di + o_ru;
    ap.recv = static_cast<const uint8_t*>(repair);
    ap.r0 = w->r0.as<uint8_t>();
    ap.n_union = (uint32_t)uni.size();
    ap.xcoef = s.xcoef;
    ap.xoff = s.xoff;
    ap.xpiv = s.xpiv;
    ap.status = s.status;
    ap.data = static_cast<uint8_t*>(data);
    ap.data_stride = data_stride;
    ap.T = T;
    ap.max_e = max_e;
    // recovered-row store policy (RQHIP_APPLY_SC1=1 in experiments builds: written through, so the
    // kernel boundary after the apply has no dirty lines to write back)
    static const uint32_t apply_sc1 = [] { const char* e = knob("RQHIP_APPLY_SC1"); return e && e[0] == '1' ? 1u : 0u; }();
    ap.out_sc1 = apply_sc1;
    if (gi && nw && max_e) {
        if (!xbits_done && launch_xbits(xa, nw, gsh, stream)) return fail(RQ_ERR_DEVICE, "k_xbits launch failed");
        ApplyGiArgs ga{};
        ga.gi = xa.gi;
        ga.block_bytes = gl.block * 4;
        ga.of_bytes = gl.of * 4;
        ga.ix_bytes = gl.ix * 4;
        ga.ix_slice_bytes = gl.ix_slice * 4;
        ga.n_blocks = nw;
        ga.T = T;
        ga.strips = (T / 4 + 64 * gsh.CPL - 1) / (64 * gsh.CPL);  // waves per (block, slice)
        // one wave per workgroup: the strips of a (block, slice) as one workgroup (sharing the CU's scalar
        // cache, RQHIP_APPLY_WS=8 in experiments builds) measured 152 against 112 us
        static const uint32_t ws_cap = [] { const char* e = knob("RQHIP_APPLY_WS"); return e ? (uint32_t)std::max(1, std::atoi(e)) : 1u; }();
        ga.ws = std::min<uint32_t>(ga.strips, std::min<uint32_t>(ws_cap, 8));
        ga.nsg = (ga.strips + ga.ws - 1) / ga.ws;
        ga.sg_magic = (uint32_t)((0x80000000ull + ga.nsg - 1) / ga.nsg);
        size_t asz = sizeof ga;
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ga, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
        HIP_TRY(hipModuleLaunchKernel(gi_fn, 8, gl.nslm * ga.nsg, (nw + 7) / 8, 64 * ga.ws, 1, 1, 0, (hipStream_t)stream,
                                      nullptr, cfg));
    } else if (launch_apply(ap, (T / 4 + 63) / 64, nw, stream)) return fail(RQ_ERR_DEVICE, "k_apply launch failed");
    const size_t pack_bytes = (size_t)nz * T;
    if (po) {
        if ((rc = w->pk.ensure(pack_bytes)) || (rc = w->h_pack.ensure(pack_bytes))) return rc;
        z.pack = w->pk.as<uint8_t>();
        if (launch_pack_rows(z, stream)) return fail(RQ_ERR_DEVICE, "k_pack_rows launch failed");
    }
    // The downloads, then one event: `up` (the staging's readers are done; recorded after the downloads,
    // which is later than needed) doubles as the workspace's last-use marker (`done`).  Without zero
    // copy `up` was recorded after the upload and the call marks `last` as before.  (Two markers per call
    // measured ~2.5 us each between the kernels, profiles/r05_solve.)
    if (po) HIP_TRY(hipMemcpyAsync(w->h_pack.p, w->pk.p, pack_bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    if (!status_by_solver)
        HIP_TRY(hipMemcpyAsync(async ? (void*)status : w->h_status.p, dst_status, n_blocks * 4, hipMemcpyDeviceToHost,
                               (hipStream_t)stream));
    if (zero_copy) {
        HIP_TRY(hipEventRecord(w->up[set], (hipStream_t)stream));
        up_guard.armed = false;
        mark_guard.armed = false;
        w->done = w->up[set];
    } else {
        mark_guard.armed = false;
        if ((rc = w->mark(stream))) return rc;
    }
    if (async) return RQ_OK;  // statuses land in the caller's pinned array when the stream gets here
    if (fin == Fin::Deferred) return RQ_OK;  // decode_collect after the caller's stream sync
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    decode_collect(w, blk_map, eoff, T, status, po);
    return RQ_OK;
}

// Batched syndrome decode.  Caller holds ctx->mu.  Host arrays as in rq_decode_desc.  Sync calls run
// the subset pass and, for blocks whose subset was rank-deficient, the all-repairs pass (see
// g_subset_margin); async calls offer every received repair in one pass (no host decision between
// passes).  A deferred decode (the host-memory pipeline) is decode_begin now, decode_finish after
// its stream was synchronised: the subset pass, then the all-repairs pass like a sync call.
struct DecodeJob {
    Params p;
    uint32_t T = 0, n_blocks = 0;
    void* data = nullptr;
    uint64_t data_stride = 0;
    const uint32_t *erased = nullptr, *n_repair = nullptr, *repair_esi = nullptr;
    const void* repair = nullptr;
    int32_t* status = nullptr;
    int32_t* status_dev = nullptr;  // async: the status array's device address (k_solve writes it)
    void* stream = nullptr;
    std::vector<uint32_t> eoff, roff, blk_map, cnt;
    uint32_t rmax = 0;        // the largest received repair ESI (decode_args)
    bool all_repairs = false;  // every block to solve offers all its received repairs (async)
};

// decode_begin's host part: offsets, argument checks, host-decided statuses, the blocks to solve.
void lpt_order(std::vector<uint32_t>& map, const uint32_t* n_erased);

int decode_args(DecodeJob* j, const uint32_t* n_erased, Fin fin) {
    const uint32_t n_blocks = j->n_blocks;
    j->eoff.assign(n_blocks + 1, 0);
    j->roff.assign(n_blocks + 1, 0);
    for (uint32_t b = 0; b < n_blocks; ++b) {
        j->eoff[b + 1] = j->eoff[b] + n_erased[b];
        j->roff[b + 1] = j->roff[b] + j->n_repair[b];
    }
    // argument checks over the whole arrays (vectorised reductions), before any status is written
    const size_t n_er = j->eoff[n_blocks], n_rep = j->roff[n_blocks];
    uint32_t emax = 0, rmin = 0xFFFFFFFFu, rmax = 0, nrmax = 0;
    const uint32_t *er = j->erased, *re = j->repair_esi;
    for (size_t i = 0; i < n_er; ++i) emax = std::max(emax, er[i]);
    for (size_t i = 0; i < n_rep; ++i) {
        rmin = std::min(rmin, re[i]);
        rmax = std::max(rmax, re[i]);
    }
    for (uint32_t b = 0; b < n_blocks; ++b) nrmax = std::max(nrmax, j->n_repair[b]);
    // the solvers keep a received repair's index within its block as uint16 (rowid / xpiv)
    if (nrmax > 65535) return fail(RQ_ERR_UNSUPPORTED, "more than 65535 received repair symbols in one block");
    if (n_er && emax >= j->p.K) return fail(RQ_ERR_BAD_ARG, "erased ESI >= K");
    if (n_rep && rmin < j->p.K) return fail(RQ_ERR_BAD_ARG, "repair ESI < K");
    j->rmax = rmax;
    j->all_repairs = fin == Fin::Async;
    j->blk_map.clear();
    j->cnt.assign(n_blocks, 0);
    for (uint32_t b = 0; b < n_blocks; ++b) {
        const uint32_t e = n_erased[b], nr = j->n_repair[b];
        if (e > nr) { j->status[b] = RQ_ERR_NOT_ENOUGH; continue; }  // (K - e) + nr < K held symbols
        if (e == 0) { j->status[b] = 1; continue; }
        j->status[b] = ST_PENDING;
        j->cnt[b] = fin == Fin::Async ? nr : std::min(nr, e + g_subset_margin);
        j->blk_map.push_back(b);
    }
    lpt_order(j->blk_map, n_erased);
    return RQ_OK;
}

// The solve list in decreasing erasure count (stable; a counting sort).  The solvers' and the apply's
// workgroups are dealt out in list order and a block's work grows with e (e pivot steps; e^2 / 8 apply
// slices), so the largest blocks start first and the per-CU loads even out (longest-first scheduling).
// RQHIP_LPT=0 keeps the block order (experiments builds).  Blocks of equal e are interchangeable here:
// every per-block array is indexed by the block, and the list only sets the launch order.
void lpt_order(std::vector<uint32_t>& map, const uint32_t* n_erased) {
    static const bool off = [] { const char* e = knob("RQHIP_LPT"); return e && e[0] == '0'; }();
    if (off || map.size() < 2) return;
    uint32_t emax = 0;
    for (uint32_t b : map) emax = std::max(emax, n_erased[b]);
    if (emax >= (1u << 16)) return;
    static thread_local std::vector<uint32_t> cnt, out;
    cnt.assign(emax + 2, 0);
    for (uint32_t b : map) ++cnt[emax - n_erased[b] + 1];  // key emax - e: ascending key = descending e
    for (uint32_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
    out.resize(map.size());
    for (uint32_t b : map) out[cnt[emax - n_erased[b]]++] = b;
    map.swap(out);
    static const bool plain = [] { const char* e = knob("RQHIP_LPT"); return e && e[0] == '1'; }();
    if (plain) return;
    // Within each XCD's share (list positions x, x + 8, ...: workgroups are dealt to the XCDs round-robin),
    // every other row of 32 (one block per CU of the XCD) reversed, so that a CU's four blocks sum to
    // about the same work: solve 63.0 -> 62.2-62.3 us against the plain order (profiles/r06_lpt;
    // RQHIP_LPT=1 keeps the plain order in experiments builds)
    const size_t n = map.size();
    out = map;
    for (size_t x = 0; x < 8; ++x) {
        const size_t m = (n > x) ? (n - x + 7) / 8 : 0;
        for (size_t r = 0; r < m; ++r) {
            const size_t q = r / 32, base = 32 * q, len = std::min<size_t>(32, m - base), c = r - base;
            const size_t f = base + ((q & 1) ? len - 1 - c : c);
            map[x + 8 * r] = out[x + 8 * f];
        }
    }
}

// The largest candidate ESI of a pass over every block with all their received repairs: the argument
// check's maximum (0: plan_decode computes it).
uint32_t decode_mx_hint(const DecodeJob& j) {
    return j.all_repairs && j.blk_map.size() == j.n_blocks ? j.rmax : 0u;
}

int decode_begin(DevCtx* ctx, DecodeJob* j, const uint32_t* n_erased, PackOut* po, Fin fin) {
    int rc = decode_args(j, n_erased, fin);
    if (rc || j->blk_map.empty()) return rc;
    const uint32_t n_blocks = j->n_blocks;
    return decode_pass(ctx, j->p, j->T, n_blocks, j->data, j->data_stride, j->eoff, j->erased, j->roff, j->repair_esi,
                       j->cnt, j->blk_map, j->repair, j->status, j->stream, po, fin, decode_mx_hint(*j), j->status_dev);
}

// After a Sync pass (or a Deferred one and a sync of its stream): the all-repairs pass for the
// blocks whose subset was rank-deficient.
int decode_finish(DevCtx* ctx, DecodeJob* j, PackOut* po, bool collect, const RowSink* sink = nullptr) {
    if (j->blk_map.empty()) return RQ_OK;
    if (collect) decode_collect(ctx->wsp(j->stream), j->blk_map, j->eoff, j->T, j->status, po, sink);
    std::vector<uint32_t> again;
    for (uint32_t b : j->blk_map)
        if (j->status[b] == 0 && j->cnt[b] < j->n_repair[b]) {
            j->cnt[b] = j->n_repair[b];
            j->status[b] = ST_PENDING;
            again.push_back(b);
        }
    if (again.empty()) return RQ_OK;
    return decode_pass(ctx, j->p, j->T, j->n_blocks, j->data, j->data_stride, j->eoff, j->erased, j->roff,
                       j->repair_esi, j->cnt, again, j->repair, j->status, j->stream, po, Fin::Sync);
}

int decode_locked(DevCtx* ctx, const Params& p, uint32_t T, uint32_t n_blocks, void* data, uint64_t data_stride,
                  const uint32_t* n_erased, const uint32_t* erased, const uint32_t* n_repair,
                  const uint32_t* repair_esi, const void* repair, int32_t* status, void* stream,
                  PackOut* po = nullptr, Fin fin = Fin::Sync, int32_t* status_dev = nullptr) {
    DecodeJob j;
    j.p = p; j.T = T; j.n_blocks = n_blocks; j.data = data; j.data_stride = data_stride; j.erased = erased;
    j.n_repair = n_repair; j.repair_esi = repair_esi; j.repair = repair; j.status = status; j.stream = stream;
    j.status_dev = fin == Fin::Async ? status_dev : nullptr;
    int rc = decode_begin(ctx, &j, n_erased, po, fin);
    if (rc || fin == Fin::Async) return rc;
    return decode_finish(ctx, &j, po, false);
}

// ---------------- host-memory batches (rq_encode_batch_host / rq_decode_batch_host) ----------------
// Blocks per pipeline chunk of the host-memory paths, which are PCIe-bound: about eight chunks, so
// that every chunk's kernels, download and host scatter hide behind the next chunks' uploads, but
// each at least twice as long to upload (at ~50 GB/s) as its launches' fixed latency `launch_us`
// (one round of column-program items, the solver's pivot chain), and at least 16 MiB
// (profiles/r02ae: one 128 MiB chunk at K=512 T=256 left copies and kernels serial; 16 MiB chunks at
// K=2048 paid the 0.23 ms solve of e ~ 113 eight times).
uint64_t g_chunk_min_mib = 32, g_chunks = 4;
uint32_t chunk_blocks(uint64_t block_bytes, uint32_t n_blocks, double launch_us) {
#ifdef RQHIP_EXPERIMENTS
    static const bool once = [] {
        if (const char* e = knob("RQHIP_CHUNK_MIB")) g_chunk_min_mib = std::strtoull(e, nullptr, 10);
        if (const char* e = knob("RQHIP_CHUNKS")) g_chunks = std::strtoull(e, nullptr, 10);
        return true;
    }();
    (void)once;
#endif
    const uint64_t min_bytes = std::max<uint64_t>(g_chunk_min_mib << 20, (uint64_t)(launch_us * 1e5));
    const uint64_t min_b = (min_bytes + block_bytes - 1) / std::max<uint64_t>(block_bytes, 1);
    const uint64_t cb = std::max<uint64_t>((n_blocks + g_chunks - 1) / g_chunks, min_b);
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_blocks, cb));
}

// Fixed latency of one launch sequence (us), fitted on the K=512 / 2048 traces of profiles/r02ae:
// a round of column-program items ~0.075 us per source symbol; the decode solve ~2 us per pivot.
double encode_launch_us(uint32_t K) { return 0.075 * K + 20; }
double decode_launch_us(uint32_t K, uint32_t max_e) { return 0.075 * K + 2.0 * max_e + 50; }

int ensure_kdone(DevCtx* ctx) {
    for (hipEvent_t& e : ctx->kdone)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : ctx->updone)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return RQ_OK;
}

// Orders chunk c's upload on stage stream `s` after chunk c-1's (begin) and marks its end (end).
int upload_begin(DevCtx* ctx, uint32_t c, hipStream_t s) {
    if (c > 0) HIP_TRY(hipStreamWaitEvent(s, ctx->updone[(c - 1) % DevCtx::NST], 0));
    return RQ_OK;
}
int upload_end(DevCtx* ctx, uint32_t c, hipStream_t s) {
    HIP_TRY(hipEventRecord(ctx->updone[c % DevCtx::NST], s));
    return RQ_OK;
}

int ensure_stages(DevCtx* ctx) {
    for (Stage& s : ctx->stage)
        if (!s.s) HIP_TRY(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
    return RQ_OK;
}

// Copy n_rows rows of `width` bytes between strided layouts (one copy when both are dense).
int copy_rows(void* dst, uint64_t dpitch, const void* src, uint64_t spitch, uint64_t width, uint32_t n_rows,
              hipMemcpyKind kind, hipStream_t s) {
    if (!n_rows || !width) return RQ_OK;
    if (dpitch == width && spitch == width) {
        HIP_TRY(hipMemcpyAsync(dst, src, width * n_rows, kind, s));
        return RQ_OK;
    }
    for (uint32_t r = 0; r < n_rows; ++r)
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(dst) + r * dpitch, static_cast<const uint8_t*>(src) + r * spitch,
                               width, kind, s));
    return RQ_OK;
}

// Rows of `width` bytes between pitched layouts (the host's T-byte rows and the device staging's
// 4-byte-padded rows when T % 4 != 0): one 2D copy.
int copy_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows, hipMemcpyKind kind,
            hipStream_t s) {
    if (!rows || !width) return RQ_OK;
    if (dpitch == width && spitch == width) HIP_TRY(hipMemcpyAsync(dst, src, width * rows, kind, s));
    else HIP_TRY(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, kind, s));
    return RQ_OK;
}

// One device's shard [b0, b1) of a host-memory encode: chunk c runs on stage c % NST (H2D source,
// column program, D2H repairs); calls on one stream are ordered, so a stage's buffers are reused
// only after its previous chunk finished, and `kdone` keeps the stages' kernels in chunk order.
int encode_host_shard(int dev, const rq_encode_desc& d, const Params& p, uint32_t b0, uint32_t b1) {
    g_device = dev;
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if ((rc = ensure_stages(ctx)) || (rc = ensure_kdone(ctx))) return rc;
    // device rows are padded to Tp = T rounded up to 4 bytes (GF(256) work is bytewise: the pad bytes
    // only ever reach pad bytes)
    const uint32_t T = d.T, Tp = pad_row(T);
    const uint64_t in_b = (uint64_t)d.K * Tp, out_b = (uint64_t)d.n_esi * Tp;
    const uint32_t cb = chunk_blocks(in_b, b1 - b0, encode_launch_us(d.K));
    for (uint32_t c = 0, b = b0; b < b1; ++c, b += cb) {
        Stage& st = ctx->stage[c % DevCtx::NST];
        const uint32_t nb = std::min(cb, b1 - b);
        if ((rc = st.in.ensure(cb * in_b)) || (rc = st.out.ensure(cb * out_b))) return rc;
        const uint8_t* src = static_cast<const uint8_t*>(d.src) + b * d.src_stride;
        uint8_t* out = static_cast<uint8_t*>(d.out) + b * d.out_stride;
        if ((rc = upload_begin(ctx, c, st.s))) return rc;
        if (Tp == T) {
            rc = copy_rows(st.in.p, in_b, src, d.src_stride, in_b, nb, hipMemcpyHostToDevice, st.s);
        } else if (d.src_stride == (uint64_t)d.K * T) {
            rc = copy_2d(st.in.p, Tp, src, T, T, (size_t)nb * d.K, hipMemcpyHostToDevice, st.s);
        } else {
            for (uint32_t i = 0; i < nb && !rc; ++i)
                rc = copy_2d(st.in.as<uint8_t>() + i * in_b, Tp, src + i * d.src_stride, T, T, d.K,
                             hipMemcpyHostToDevice, st.s);
        }
        if (!rc) rc = upload_end(ctx, c, st.s);
        if (!rc && c > 0) rc = hipStreamWaitEvent(st.s, ctx->kdone[(c - 1) % DevCtx::NST], 0) == hipSuccess ? RQ_OK
                                  : fail(RQ_ERR_DEVICE, "hipStreamWaitEvent failed");
        if (rc || (rc = encode_locked(ctx, p, Tp, nb, st.in.p, in_b, d.esi, d.n_esi, st.out.p, out_b, st.s)))
            return rc;
        HIP_TRY(hipEventRecord(ctx->kdone[c % DevCtx::NST], st.s));  // the stages' kernels run in chunk order
        if (Tp == T) {
            rc = copy_rows(out, d.out_stride, st.out.p, out_b, out_b, nb, hipMemcpyDeviceToHost, st.s);
        } else if (d.out_stride == (uint64_t)d.n_esi * T) {
            rc = copy_2d(out, T, st.out.p, Tp, T, (size_t)nb * d.n_esi, hipMemcpyDeviceToHost, st.s);
        } else {
            for (uint32_t i = 0; i < nb && !rc; ++i)
                rc = copy_2d(out + i * d.out_stride, T, st.out.as<uint8_t>() + i * out_b, Tp, T, d.n_esi,
                             hipMemcpyDeviceToHost, st.s);
        }
        if (rc) return rc;
    }
    for (Stage& st : ctx->stage) HIP_TRY(hipStreamSynchronize(st.s));
    return RQ_OK;
}

// Host-memory decode input: block b's K*T data bytes at data[b] (recovered rows written back there)
// and its n_repair[b] received repair rows, consecutive, at rep[b].  Index arrays as in rq_decode_desc.
struct HostDecode {
    uint32_t T = 0, K = 0;
    std::vector<uint8_t*> data;
    std::vector<const uint8_t*> rep;
    const uint32_t *n_erased = nullptr, *erased = nullptr, *n_repair = nullptr, *repair_esi = nullptr;
    int32_t* status = nullptr;
};

// H2D of `n` blocks' regions of `bytes[i]` bytes from host pointers src[i] to consecutive device
// memory: one copy per run of host-contiguous blocks.
template <class P>
int upload_runs(uint8_t* dst, const P* src, const uint64_t* bytes, uint32_t n, hipStream_t s) {
    uint32_t i = 0;
    while (i < n) {
        uint64_t run = bytes[i];
        uint32_t j = i + 1;
        while (j < n && (const uint8_t*)src[j] == (const uint8_t*)src[i] + run) run += bytes[j++];
        if (run) HIP_TRY(hipMemcpyAsync(dst, src[i], run, hipMemcpyHostToDevice, s));
        dst += run;
        i = j;
    }
    return RQ_OK;
}

// One device's shard of a host-memory decode.  Per chunk: upload the data blocks and their received
// repair rows, decode, download only the recovered rows and scatter them into the caller's buffers
// for the blocks that decoded.  The uploads and kernels of the next NST - 1 chunks are queued on the
// other stages before a chunk is collected, so the link stays busy while the host scatters.
int decode_host_shard(int dev, const HostDecode& d, const Params& p, uint32_t b0, uint32_t b1,
                      const std::vector<uint64_t>& eoff, const std::vector<uint64_t>& roff) {
    g_device = dev;
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if ((rc = ensure_stages(ctx))) return rc;
    const uint32_t T = d.T, Tp = pad_row(T);  // device rows padded (see encode_host_shard)
    const uint64_t blk_b = (uint64_t)d.K * Tp;
    uint32_t max_e = 0;
    for (uint32_t b = b0; b < b1; ++b) max_e = std::max<uint32_t>(max_e, d.n_erased[b]);
    const uint32_t cb = chunk_blocks(blk_b, b1 - b0, decode_launch_us(d.K, max_e));
    uint32_t max_rep = 0;
    for (uint32_t b = b0; b < b1; b += cb)
        max_rep = std::max<uint32_t>(max_rep, (uint32_t)(roff[std::min(b1, b + cb)] - roff[b]));
    // phase timing on stderr (experiments builds, RQHIP_HOST_PROF)
#ifdef RQHIP_EXPERIMENTS
    static const bool hprof = knob("RQHIP_HOST_PROF") != nullptr;
#else
    constexpr bool hprof = false;
#endif
    const auto t_start = std::chrono::steady_clock::now();
    auto hp = [&](const char* what, uint32_t c) {
        if (hprof)
            std::fprintf(stderr, "[hprof]   %s %u %.3f\n", what, c,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    };
    auto upload = [&](uint32_t c) -> int {
        Stage& st = ctx->stage[c % DevCtx::NST];
        const uint32_t b = b0 + c * cb, nb = std::min(cb, b1 - b);
        int r;
        if ((r = st.in.ensure(cb * blk_b)) || (r = st.out.ensure(std::max<size_t>((size_t)max_rep * Tp, 4)))) return r;
        hp("ensured", c);
        if ((r = upload_begin(ctx, c, st.s))) return r;
        if (Tp == T) {
            std::vector<uint64_t> db(nb, blk_b), rb(nb);
            for (uint32_t i = 0; i < nb; ++i) rb[i] = (uint64_t)d.n_repair[b + i] * T;
            if ((r = upload_runs(st.in.as<uint8_t>(), d.data.data() + b, db.data(), nb, st.s))) return r;
            hp("data queued", c);
            if ((r = upload_runs(st.out.as<uint8_t>(), d.rep.data() + b, rb.data(), nb, st.s))) return r;
            hp("repairs queued", c);
            return upload_end(ctx, c, st.s);
        }
        uint8_t* rd = st.out.as<uint8_t>();
        for (uint32_t i = 0; i < nb; ++i) {
            if ((r = copy_2d(st.in.as<uint8_t>() + i * blk_b, Tp, d.data[b + i], T, T, d.K, hipMemcpyHostToDevice,
                             st.s)) ||
                (r = copy_2d(rd, Tp, d.rep[b + i], T, T, d.n_repair[b + i], hipMemcpyHostToDevice, st.s)))
                return r;
            rd += (size_t)d.n_repair[b + i] * Tp;
        }
        return upload_end(ctx, c, st.s);
    };
    const uint32_t n_chunks = (b1 - b0 + cb - 1) / cb;
    // chunk c+1 is uploaded and its kernels queued before chunk c's statuses and rows are collected
    // and scattered on the host (kernels of the two stages run in order: `kdone`), so the download,
    // the scatter and the next chunk's descriptor work overlap the device instead of idling it
    DecodeJob job[DevCtx::NST];
    PackOut po[DevCtx::NST];
    auto issue = [&](uint32_t c) -> int {
        Stage& st = ctx->stage[c % DevCtx::NST];
        const uint32_t b = b0 + c * cb, nb = std::min(cb, b1 - b);
        if (c > 0) HIP_TRY(hipStreamWaitEvent(st.s, ctx->kdone[(c - 1) % DevCtx::NST], 0));
        DecodeJob& j = job[c % DevCtx::NST];
        j = DecodeJob();
        j.p = p; j.T = Tp; j.n_blocks = nb; j.data = st.in.p; j.data_stride = blk_b; j.erased = d.erased + eoff[b];
        j.n_repair = d.n_repair + b; j.repair_esi = d.repair_esi + roff[b]; j.repair = st.out.p;
        j.status = d.status + b; j.stream = st.s;
        po[c % DevCtx::NST] = PackOut();
        int r = decode_begin(ctx, &j, d.n_erased + b, &po[c % DevCtx::NST], Fin::Deferred);
        if (!r) HIP_TRY(hipEventRecord(ctx->kdone[c % DevCtx::NST], st.s));
        return r;
    };
    auto finish = [&](uint32_t c) -> int {
        Stage& st = ctx->stage[c % DevCtx::NST];
        const uint32_t b = b0 + c * cb;
        HIP_TRY(hipStreamSynchronize(st.s));
        // the first pass's rows are scattered from the pinned download; a rank-deficient retry's
        // (rare) arrive in po
        const RowSink sink = [&](uint32_t lb, const uint8_t* rows) {
            const uint32_t gb = b + lb;
            for (uint64_t i = eoff[gb]; i < eoff[gb + 1]; ++i, rows += Tp)
                std::memcpy(d.data[gb] + (uint64_t)d.erased[i] * T, rows, T);
        };
        int r = decode_finish(ctx, &job[c % DevCtx::NST], &po[c % DevCtx::NST], true, &sink);
        if (r) return r;
        size_t k = 0;  // po holds the retry's recovered rows (Tp apart) of the blocks that decoded
        const PackOut& o = po[c % DevCtx::NST];
        for (uint32_t lb : o.blocks) {
            const uint32_t gb = b + lb;
            for (uint64_t i = eoff[gb]; i < eoff[gb + 1]; ++i, ++k)
                std::memcpy(d.data[gb] + (uint64_t)d.erased[i] * T, o.rows.data() + k * Tp, T);
        }
        return RQ_OK;
    };
    constexpr uint32_t AHEAD = DevCtx::NST - 1;  // chunks queued beyond the one being collected
    auto timed = [&](const char* what, uint32_t c, auto&& fn) {
        if (!hprof) return fn(c);
        auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count(); };
        const double t0 = ms();
        const int r = fn(c);
        std::fprintf(stderr, "[hprof] %s %u %.3f-%.3f\n", what, c, t0, ms());
        return r;
    };
    auto run_upload = [&](uint32_t c) { return timed("upload", c, upload); };
    auto run_issue = [&](uint32_t c) { return timed("issue", c, issue); };
    auto run_finish = [&](uint32_t c) { return timed("finish", c, finish); };
    if ((rc = ensure_kdone(ctx))) return rc;
    for (uint32_t c = 0; c < std::min(AHEAD, n_chunks); ++c)
        if ((rc = run_upload(c)) || (rc = run_issue(c))) {
            for (Stage& st : ctx->stage) (void)hipStreamSynchronize(st.s);  // no queued work behind the error
            return rc;
        }
    for (uint32_t c = 0; c < n_chunks; ++c) {
        if (c + AHEAD < n_chunks && ((rc = run_upload(c + AHEAD)) || (rc = run_issue(c + AHEAD)))) {
            for (Stage& st : ctx->stage) (void)hipStreamSynchronize(st.s);
            return rc;
        }
        if ((rc = run_finish(c))) return rc;
    }
    return RQ_OK;
}

// Split [0, n_blocks) contiguously over the devices of device_mask (0: the calling thread's
// device): shard i = devs[i], blocks [b0_i, b1_i).  `virt` > 1 (rq_debug_virtual_shards, tests) splits
// over that many host threads on the one device of a 0 / single-bit mask.
struct ShardPlan {
    std::vector<int> dev;
    std::vector<uint32_t> b0, b1;
};
uint32_t g_virtual_shards = 0;

int plan_shards(uint32_t device_mask, int n_dev, int cur_dev, uint32_t n_blocks, uint32_t virt, ShardPlan* sp) {
    std::vector<int> devs;
    if (device_mask == 0) {
        devs.push_back(cur_dev);
    } else {
        for (int i = 0; i < 32; ++i)
            if (device_mask >> i & 1u) {
                if (i >= n_dev) return fail(RQ_ERR_BAD_ARG, "device_mask names a device that does not exist");
                devs.push_back(i);
            }
    }
    if (virt > 1 && devs.size() == 1) devs.assign(virt, devs[0]);
    const uint32_t nd = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)devs.size(), n_blocks));
    *sp = ShardPlan();
    for (uint32_t i = 0; i < nd; ++i) {
        sp->dev.push_back(devs[i]);
        sp->b0.push_back((uint32_t)((uint64_t)n_blocks * i / nd));
        sp->b1.push_back((uint32_t)((uint64_t)n_blocks * (i + 1) / nd));
    }
    return RQ_OK;
}

// Run `shard(dev, b0, b1)` for every shard of the plan, one host thread per shard.
template <class F>
int run_sharded(uint32_t device_mask, uint32_t n_blocks, F shard) {
    int n = 0, cur = 0, rc;
    if (device_mask == 0) {
        if ((rc = current_device(&cur))) return rc;
    } else if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        return fail(RQ_ERR_DEVICE, "no HIP device available");
    }
    ShardPlan sp;
    if ((rc = plan_shards(device_mask, n, cur, n_blocks, g_virtual_shards, &sp))) return rc;
    const uint32_t nd = (uint32_t)sp.dev.size();
    if (nd == 1) return shard(sp.dev[0], 0u, n_blocks);
    std::vector<int> rcs(nd, RQ_OK);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    for (uint32_t i = 0; i < nd; ++i) {
        th.emplace_back([&, i] {
            rcs[i] = shard(sp.dev[i], sp.b0[i], sp.b1[i]);
            if (rcs[i]) errs[i] = g_err;
        });
    }
    for (auto& t : th) t.join();
    for (uint32_t i = 0; i < nd; ++i)
        if (rcs[i]) return fail(rcs[i], errs[i]);
    return RQ_OK;
}

}  // namespace
}  // namespace rq

using namespace rq;

// ====================================== C ABI ==============================================
struct rq_enc {
    Params p{};
    uint32_t T = 0, Tp = 0;
    std::vector<uint8_t> src;  // K x Tp, zero padded (GenSymbol for esi < K)
    std::vector<uint8_t> rep;  // repairs K .. K + n_rep - 1, Tp apart (GenSymbol served from host)
    uint32_t n_rep = 0;
    DevBuf d_src, d_C, d_esi, d_out;
};

// AddSymbol's bookkeeping alone (rq_tracker_*): which ESIs are held, no symbol bytes.
struct rq_tracker {
    Params p{};
    uint32_t T = 0;
    std::vector<uint8_t> have;       // K flags (the decoder's fast bitmap)
    uint32_t nfast = 0;
    std::unordered_set<uint32_t> slow;  // repair ESIs held (the decoder's slow map keys)
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
        case RQ_ERR_PLAN: return "program compilation failed";
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

int rq_debug_tuple(uint32_t K, uint32_t X, uint32_t out[6]) {
    Params p;
    const int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    const Tuple t = tuple_of(p, X);
    const uint32_t v[6] = {t.d, t.a, t.b, t.d1, t.a1, t.b1};
    std::memcpy(out, v, sizeof v);
    return RQ_OK;
}

int rq_stream_release(void* stream) {
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->internal(stream)) return fail(RQ_ERR_BAD_ARG, "not a caller stream");
    ctx->release_ws(stream);
    return RQ_OK;
}

int rq_launch_timing(int enable) {
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->timing = enable != 0;
    return RQ_OK;
}

int rq_launch_time(double* ms_total, uint32_t* n_launches, int reset) {
    if (!ms_total || !n_launches) return fail(RQ_ERR_BAD_ARG, "null output");
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    double sum = 0;
    for (size_t i = 0; i < ctx->tev_used; ++i) {
        HIP_TRY(hipEventSynchronize(ctx->tev[i].second));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ctx->tev[i].first, ctx->tev[i].second));
        sum += ms;
    }
    *ms_total = sum;
    *n_launches = (uint32_t)ctx->tev_used;
    if (reset) ctx->tev_used = 0;  // a new window
    return RQ_OK;
}

int rq_shutdown(void) {
    std::vector<std::shared_ptr<DevCtx>> gone;
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        for (auto& kv : g_ctx) gone.push_back(std::move(kv.second));
        g_ctx.clear();
    }
    // ~DevCtx (device sync, then every buffer, module, stream and event of the device) runs here, or
    // in a concurrent call that still holds the context, when that call returns
    gone.clear();
    return RQ_OK;
}

int rq_set_device(int device) {
    const int n = rq_device_count();
    if (device < 0 || device >= n) return fail(RQ_ERR_DEVICE, "bad device index");
    g_device = device;
    HIP_TRY(hipSetDevice(device));
    return RQ_OK;
}

int g_debug_passes = -1;  // rq_debug_colprog_passes: fixed IR schedule for the debug entry points

bool debug_compile(const Params& p, const uint32_t* esi, uint32_t n_out, const AllocOpts& o, ColIR* ir, MProg* mp,
                   std::string* err) {
    if (g_debug_passes < 0) return compile_colprog(p, esi, n_out, o, ir, mp, err);
    const uint32_t P = (uint32_t)g_debug_passes;
    const bool ok = esi ? build_colprog(p, esi, n_out, ir, err, P) : build_colprog_C(p, ir, err, P);
    return ok && allocate_colprog(*ir, o, mp, err);
}

int rq_debug_colprog_passes(int passes) {
    const int old = g_debug_passes;
    g_debug_passes = passes;
    return old;
}

int rq_debug_colprog_eval(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                          uint8_t* out, uint32_t stats[12]) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    ColIR ir;
    MProg mp;
    std::string err;
    if (!debug_compile(p, esi, n_out, alloc_options(), &ir, &mp, &err)) return fail(RQ_ERR_PLAN, err);
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
                             uint8_t* out, const uint32_t opts[9], uint32_t stats[18], char* asm_buf, size_t asm_cap,
                             size_t* asm_len) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    ColIR ir;
    std::string err;
    AllocOpts o = alloc_options();
    if (opts) {
        if (opts[0]) o.n_vgpr = std::min<uint32_t>(opts[0], V_ALLOC);
        if (opts[1]) o.n_agpr = std::min<uint32_t>(opts[1], 256);
        if (opts[2]) o.la_load = opts[2];
        if (opts[3]) o.la_reload = opts[3];
        if (opts[4]) o.max_vmem = std::min<uint32_t>(opts[4], 60);
        if (opts[5]) o.n_lds = std::min<uint32_t>(opts[5] - 1, 512);
        if (opts[6]) o.cip = opts[6] - 1;
        if (opts[7]) o.cip_batch = opts[7];
        if (opts[8]) o.cip_gap = opts[8];
    }
    MProg mp;
    if (!debug_compile(p, esi, n_out, o, &ir, &mp, &err)) return fail(RQ_ERR_PLAN, err);
    if (src && out && !emulate_colprog(mp, src, T, out, &err)) return fail(RQ_ERR_PLAN, err);
    if (stats) {
        const auto& s = mp.st;
        const uint32_t v[18] = {(uint32_t)mp.ins.size(), s.valu, s.ldsrc, s.stout, s.spst, s.spld, s.accw, s.accr,
                                s.wait, s.nop, s.sync_reload, mp.n_slots, (uint32_t)ir.nodes.size(), ir.st.xt + ir.st.xtx,
                                s.ldst, s.ldld, s.waitl, mp.n_lds_slots};
        std::memcpy(stats, v, sizeof v);
    }
    if (asm_len) {
        (void)colprog_launch_shape(&mp);
        const std::string a = emit_colprog_asm(mp, "rq_colprog");
        *asm_len = a.size();
        if (asm_buf && asm_cap >= a.size()) std::memcpy(asm_buf, a.data(), a.size());
    }
    return RQ_OK;
}

int rq_debug_colprog_assemble(uint32_t K, const uint32_t* esi, uint32_t n_out, size_t* code_bytes) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    ColIR ir;
    std::string err;
    MProg mp;
    std::vector<char> co;
    if (g_debug_passes < 0) {  // the kernel the engine would build: the pair split where it is chosen
        PairProg pp;
        bool pair = false;
        if (!compile_engine_program(p, esi, n_out, alloc_options(), true, true, &ir, &mp, &pp, &pair, &err))
            return fail(RQ_ERR_PLAN, err);
        if (pair) {
            if (!comgr_assemble(emit_pair_asm(pp, "rq_colprog_pair"), &co, &err)) return fail(RQ_ERR_PLAN, err);
            if (code_bytes) *code_bytes = co.size();
            return RQ_OK;
        }
    } else if (!debug_compile(p, esi, n_out, alloc_options(), &ir, &mp, &err)) {
        return fail(RQ_ERR_PLAN, err);
    }
    (void)colprog_launch_shape(&mp);
    if (!comgr_assemble(emit_colprog_asm(mp, "rq_colprog"), &co, &err)) return fail(RQ_ERR_PLAN, err);
    if (code_bytes) *code_bytes = co.size();
    return RQ_OK;
}

int rq_debug_cache_roundtrip(const char* path, uint32_t n_rows, uint32_t n_dma4) {
    if (!path) return fail(RQ_ERR_BAD_ARG, "no path");
    CacheHdr h;
    std::memset(&h, 0, sizeof h);
    std::memcpy(h.magic, CACHE_MAGIC, 8);
    const std::string name = "rq_colprog_cache_test";
    std::vector<char> co(4096);
    for (size_t i = 0; i < co.size(); ++i) co[i] = (char)(i * 131 + 7);
    std::vector<uint32_t> rows((size_t)n_rows + n_dma4);
    for (size_t i = 0; i < rows.size(); ++i) rows[i] = (uint32_t)(i * 2654435761u);
    h.n_rows = n_rows;
    h.n_dma4 = n_dma4;
    h.name_len = (uint32_t)name.size();
    h.co_len = co.size();
    h.body_hash = cache_body_hash(name, co, rows);
    {  // cache_store writes through a temporary name in cache_dir(): write the entry directly here
        FILE* f = std::fopen(path, "wb");
        if (!f) return fail(RQ_ERR_BAD_ARG, "cannot write the entry");
        const bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(name.data(), 1, name.size(), f) == name.size() &&
                        std::fwrite(co.data(), 1, co.size(), f) == co.size() &&
                        std::fwrite(rows.data(), 4, rows.size(), f) == rows.size();
        std::fclose(f);
        if (!ok) return fail(RQ_ERR_BAD_ARG, "cannot write the entry");
    }
    CacheHdr g;
    std::string n2;
    std::vector<char> co2;
    std::vector<uint32_t> r2;
    if (!cache_load(path, &g, &n2, &co2, &r2)) return fail(RQ_ERR_PLAN, "cache entry rejected on load");
    if (n2 != name || co2 != co || r2 != rows || g.n_rows != n_rows || g.n_dma4 != n_dma4)
        return fail(RQ_ERR_PLAN, "cache entry differs after the round trip");
    return RQ_OK;
}

int rq_debug_assemble(const char* src, size_t len, size_t* code_bytes) {
    if (!src) return fail(RQ_ERR_BAD_ARG, "no source");
    std::vector<char> co;
    std::string err;
    if (!comgr_assemble(std::string(src, len), &co, &err)) return fail(RQ_ERR_PLAN, err);
    if (code_bytes) *code_bytes = co.size();
    return RQ_OK;
}

int rq_debug_colprog_bound(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                           uint8_t* out, uint64_t src_bytes, uint32_t* row_end) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    ColIR ir;
    MProg mp;
    std::string err;
    if (!debug_compile(p, esi, n_out, alloc_options(), &ir, &mp, &err)) return fail(RQ_ERR_PLAN, err);
    if (row_end) *row_end = colprog_row_end(mp);
    if (src && out && !emulate_colprog(mp, src, T, out, &err, src_bytes)) return fail(RQ_ERR_PLAN, err);
    return RQ_OK;
}

int rq_debug_decode_plan(uint32_t T, uint32_t K, uint32_t n_blocks, const uint32_t* n_erased, const uint32_t* erased,
                         const uint32_t* n_repair, const uint32_t* repair_esi, uint32_t iters, double* us_per_call,
                         uint32_t* n_idx_words) {
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    std::vector<int32_t> status(n_blocks);
    std::vector<uint32_t> idx;
    double total = 0;
    for (uint32_t it = 0; it < std::max<uint32_t>(iters, 1); ++it) {
        const auto t0 = std::chrono::steady_clock::now();
        DecodeJob j;
        j.p = p; j.T = T; j.n_blocks = n_blocks; j.erased = erased; j.n_repair = n_repair; j.repair_esi = repair_esi;
        j.status = status.data();
        // decode_begin's host part (Async: every received repair offered), then decode_pass's
        if ((rc = decode_args(&j, n_erased, Fin::Async))) return rc;
        DecodePlan& pl = decode_plan_scratch();
        if (!j.blk_map.empty()) {
            if ((rc = plan_decode(p, n_blocks, j.eoff, j.roff, repair_esi, j.cnt, j.blk_map, false, &pl, decode_mx_hint(j))))
                return rc;
            if (idx.size() < pl.n_idx) idx.resize(pl.n_idx);  // (the engine writes into pinned staging)
            fill_decode_idx(pl, n_blocks, j.eoff, erased, j.roff, repair_esi, j.cnt, j.blk_map, status.data(), idx.data());
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (it) total += std::chrono::duration<double, std::micro>(t1 - t0).count();  // the first call warms up
        if (n_idx_words) *n_idx_words = j.blk_map.empty() ? 0u : (uint32_t)pl.n_idx;
    }
    if (us_per_call) *us_per_call = iters > 1 ? total / (iters - 1) : total;
    return RQ_OK;
}

int rq_debug_dma4_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src, uint8_t* out,
                          uint32_t quads, uint32_t la, uint32_t stats[8], size_t* code_bytes) {
#ifndef RQHIP_EXPERIMENTS
    (void)K; (void)T; (void)esi; (void)n_out; (void)src; (void)out; (void)quads; (void)la; (void)stats; (void)code_bytes;
    return fail(RQ_ERR_BAD_ARG, "four-row staging is in the experiments build only (tools/build_experiments.sh)");
#else
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 16) return fail(RQ_ERR_BAD_ARG, "four-row staging needs T a multiple of 16");
    ColIR ir;
    MProg mp, m4;
    std::string err;
    uint32_t passes = 0;
    if (!compile_colprog(p, esi, n_out, alloc_options(), &ir, &mp, &err, &passes, false)) return fail(RQ_ERR_PLAN, err);
    if (!compile_colprog_dma4(ir, alloc_options(), quads, la ? la : dma4_cfg().la, &m4, &err)) return fail(RQ_ERR_PLAN, err);
    if (src && out && !emulate_colprog(m4, src, T, out, &err)) return fail(RQ_ERR_PLAN, err);
    if (stats) {
        const uint32_t v[8] = {(uint32_t)m4.ins.size(), m4.st.valu, m4.st.dma, m4.n_slots, m4.lds_base, m4.n_lds_slots,
                               (uint32_t)mp.ins.size(), (passes & SCHED_4R) ? 1u : 0u};
        std::memcpy(stats, v, sizeof v);
    }
    if (code_bytes) {
        (void)colprog_launch_shape(&m4);
        std::vector<char> co;
        if (!comgr_assemble(emit_colprog_asm(m4, "rq_colprog_dma4"), &co, &err)) return fail(RQ_ERR_PLAN, err);
        *code_bytes = co.size();
    }
    return RQ_OK;
#endif
}

int rq_debug_pair_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                          uint8_t* out, const uint32_t cfg[5], uint32_t stats[16], size_t* code_bytes) {
#ifndef RQHIP_EXPERIMENTS
    (void)K; (void)T; (void)esi; (void)n_out; (void)src; (void)out; (void)cfg; (void)stats; (void)code_bytes;
    return fail(RQ_ERR_BAD_ARG, "pair programs are in the experiments build only (tools/build_experiments.sh)");
#else
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    if (T == 0 || T % 4) return fail(RQ_ERR_BAD_ARG, "T must be a positive multiple of 4");
    if (!esi || !n_out) return fail(RQ_ERR_BAD_ARG, "pair programs need output ESIs");
    const PairCfg& c = pair_cfg();
    const uint32_t lag = cfg && cfg[0] ? cfg[0] : c.lag, xfer = cfg && cfg[1] ? cfg[1] : c.xfer,
                   ring = cfg && cfg[2] ? cfg[2] : c.ring;
    ColIR ir;
    MProg mp;
    PairProg pp;
    std::string err;
    uint32_t passes = 0;
    if (!compile_colprog(p, esi, n_out, alloc_options(), &ir, &mp, &err, &passes, false)) return fail(RQ_ERR_PLAN, err);
    AllocOpts pa = alloc_options();
    pa.dma4 = !cfg || !cfg[3] ? c.dma4 : cfg[3] == 0xFFFFFFFFu ? 0u : cfg[3];  // wave A's four-row staging
    pa.la_dma = c.la_dma;
    const uint32_t ha = cfg && cfg[4] ? (cfg[4] == 0xFFFFFFFFu ? 0u : cfg[4]) : c.ha;
    if (ha) {
        ColIR irh;
        if (!build_colprog(p, esi, n_out, &irh, &err, passes | (ha << SCHED_HA_SHIFT))) return fail(RQ_ERR_PLAN, err);
        ir = std::move(irh);
    }
    if (!compile_pair(ir, pa, 0xA, lag, xfer, ring, &pp, &err)) return fail(RQ_ERR_PLAN, err);
    if (src && out && !emulate_pair(pp, src, T, out, &err, 2)) return fail(RQ_ERR_PLAN, err);
    if (stats) {
        const uint32_t v[16] = {(uint32_t)pp.A.ins.size(), pp.A.st.valu, pp.A.st.ldsrc, pp.A.st.accw + pp.A.st.accr,
                                pp.A.st.rst, pp.A.st.bar, (uint32_t)pp.B.ins.size(), pp.B.st.valu, pp.B.st.rld,
                                pp.B.st.stout, pp.ring, pp.n_xfer, pp.n_cross, pair_lds_bytes(pp), pp.A.st.dma,
                                (passes & SCHED_4R) ? 1u : 0u};
        std::memcpy(stats, v, sizeof v);
    }
    if (code_bytes) {
        std::vector<char> co;
        if (!comgr_assemble(emit_pair_asm(pp, "rq_colprog_pair"), &co, &err)) return fail(RQ_ERR_PLAN, err);
        *code_bytes = co.size();
    }
    return RQ_OK;
#endif
}

int rq_debug_shard_plan(uint32_t device_mask, int n_devices, uint32_t n_blocks, uint32_t virtual_shards, int* dev,
                        uint32_t* b0, uint32_t* b1, uint32_t cap) {
    ShardPlan sp;
    const int rc = plan_shards(device_mask, n_devices, 0, n_blocks, virtual_shards, &sp);
    if (rc) return rc;
    for (uint32_t i = 0; i < sp.dev.size() && i < cap; ++i) {
        if (dev) dev[i] = sp.dev[i];
        if (b0) b0[i] = sp.b0[i];
        if (b1) b1[i] = sp.b1[i];
    }
    return (int)sp.dev.size();
}

uint32_t rq_debug_virtual_shards(uint32_t n) {
    const uint32_t old = g_virtual_shards;
    g_virtual_shards = n;
    return old;
}

int rq_debug_apply_gi_asm(uint32_t kc, uint32_t g, uint32_t pdg, uint32_t cpl, char* text, size_t cap, size_t* text_len,
                          size_t* code_bytes) {
    GiShape sh;
    sh.KC = kc; sh.G = g; sh.PDG = pdg; sh.CPL = cpl & 0xff; sh.PACK = (cpl >> 8) & 1; sh.SX = (cpl >> 9) & 1;
    if (!gi_shape_ok(sh))
        return fail(RQ_ERR_BAD_ARG, "apply shape: KC 4..16 (a multiple of 4, of 8 packed), G 4..6, PDG 1..2, CPL 1..2 "
                                    "(| 256 packed, | 512 precomputed syndromes), <= 256 VGPRs");
    const std::string src = emit_apply_gi_asm(sh);
    std::string cerr;
    if (!check_apply_gi_asm(src, sh, &cerr)) return fail(RQ_ERR_PLAN, cerr);
    if (text_len) *text_len = src.size();
    if (text && cap) {
        const size_t n = std::min(cap - 1, src.size());
        std::memcpy(text, src.data(), n);
        text[n] = 0;
    }
    if (code_bytes) {
        std::vector<char> co;
        std::string err;
        if (!comgr_assemble(src, &co, &err)) return fail(RQ_ERR_PLAN, err);
        *code_bytes = co.size();
    }
    return RQ_OK;
}

int rq_debug_gi_stream(uint32_t e, uint32_t max_e, uint32_t solved, const uint8_t* X, const uint16_t* piv,
                       const uint32_t* erased, const uint32_t* rep_uidx, uint32_t nr, uint32_t n_union, uint32_t T,
                       uint32_t bi, uint32_t* out, size_t out_words, uint32_t layout[7]) {
    const GiShape sh;  // the shipped shape, which the solvers write (xb_on)
    if (e == 0 || e > max_e || (solved && (!X || !piv || !erased || !rep_uidx)) || !out || !layout)
        return fail(RQ_ERR_BAD_ARG, "gi stream emulation arguments");
    const GiLayout L = gi_layout(max_e, sh);
    layout[0] = L.nslm; layout[1] = L.ngrm; layout[2] = L.er; layout[3] = L.of; layout[4] = L.ix;
    layout[5] = L.ix_slice; layout[6] = L.block;
    if ((uint64_t)(bi + 1) * L.block > out_words) return fail(RQ_ERR_BAD_ARG, "gi stream buffer too small");
    for (uint32_t m = 0; solved && m < e; ++m)
        if (piv[m] >= nr || rep_uidx[piv[m]] >= n_union) return fail(RQ_ERR_BAD_ARG, "pivot row out of range");
    const uint32_t eoff[2] = {0, e}, roff[2] = {0, nr};
    XbitsArgs a{};
    a.erased_off = eoff;
    a.erased = erased;
    a.rep_off = roff;
    a.rep_uidx = rep_uidx;
    a.recv = reinterpret_cast<const uint8_t*>(uintptr_t(0x100000000ull));  // addresses only (header words)
    a.r0 = reinterpret_cast<const uint8_t*>(uintptr_t(0x200000000ull));
    a.data = reinterpret_cast<uint8_t*>(uintptr_t(0x300000000ull));
    a.data_stride = (uint64_t)T * 65536;
    a.gi = out;
    a.L = L;
    a.T = T;
    a.n_union = n_union;
    auto XF = [&](uint32_t k, uint32_t m) { return (uint32_t)X[(size_t)k * e + m]; };
    auto PF = [&](uint32_t m) { return (uint32_t)piv[m]; };
    for (uint32_t tid = 0; tid < 256; ++tid)  // the solvers' 256 threads, one after another
        gi_stream<8, 5, 2>(a, bi, 0, e, solved != 0, tid, 256, XF, PF);
    return RQ_OK;
}

int rq_debug_apply_gi_check(uint32_t kc, uint32_t g, uint32_t pdg, uint32_t cpl, const char* text) {
    GiShape sh;
    sh.KC = kc; sh.G = g; sh.PDG = pdg; sh.CPL = cpl & 0xff; sh.PACK = (cpl >> 8) & 1; sh.SX = (cpl >> 9) & 1;
    if (!text || !gi_shape_ok(sh)) return fail(RQ_ERR_BAD_ARG, "apply shape or text");
    std::string err;
    return check_apply_gi_asm(text, sh, &err) ? RQ_OK : fail(RQ_ERR_PLAN, err);
}

uint32_t rq_debug_solve_mode(uint32_t mode) {
    const uint32_t old = g_solve_ip;
#ifdef RQHIP_EXPERIMENTS
    if (mode <= 1) g_solve_ip = mode;
#else
    (void)mode;  // the release library has k_solve_pq only (k_solve_ip: experiments library)
#endif
    return old;
}

uint32_t rq_debug_apply_mode(uint32_t mode) {
    const uint32_t old = g_apply_mode;
    if (mode <= 1) g_apply_mode = mode;
    return old;
}

uint32_t rq_debug_apply_sx(uint32_t on) {
    const uint32_t old = g_apply_sx;
#ifdef RQHIP_EXPERIMENTS
    if (on <= 1) g_apply_sx = on;
#else
    (void)on;  // the release library has no syndrome workgroups (experiments library only)
#endif
    return old;
}

int rq_debug_gi_fits(uint32_t max_e, uint32_t n_solve) { return gi_stream_fits(max_e, n_solve, apply_gi_shape()) ? 1 : 0; }

uint32_t rq_debug_decode_margin(uint32_t margin) {
    const uint32_t old = g_subset_margin;
    g_subset_margin = margin;
    return old;
}

int rq_encode_batch(const rq_encode_desc* d) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->T % 4 || d->T < 8 || d->K == 0 || (!d->src && d->n_blocks))
        return fail(RQ_ERR_BAD_ARG, "bad encode descriptor (T: a multiple of 4, at least 8; K; src)");
    if (d->n_blocks == 0 || d->n_esi == 0) return RQ_OK;
    if (!d->esi || !d->out) return fail(RQ_ERR_BAD_ARG, "n_esi without esi/out");
    if (d->src_stride < (uint64_t)d->K * d->T || d->out_stride < (uint64_t)d->n_esi * d->T)
        return fail(RQ_ERR_BAD_ARG, "stride smaller than a block");
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    CtxRef ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return encode_locked(ctx, p, d->T, d->n_blocks, d->src, d->src_stride, d->esi, d->n_esi, d->out, d->out_stride,
                         d->stream);
}

int rq_decode_batch(const rq_decode_desc* d) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->T % 4 || d->T < 8 || d->K == 0) return fail(RQ_ERR_BAD_ARG, "bad decode descriptor (T: a multiple of 4, at least 8; K)");
    if (d->n_blocks == 0) return RQ_OK;
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    CtxRef ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return decode_locked(ctx, p, d->T, d->n_blocks, d->data, d->data_stride, d->n_erased, d->erased, d->n_repair,
                         d->repair_esi, d->repair, d->status, d->stream);
}

int rq_decode_batch_async(const rq_decode_desc* d) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->T % 4 || d->T < 8 || d->K == 0) return fail(RQ_ERR_BAD_ARG, "bad decode descriptor (T: a multiple of 4, at least 8; K)");
    if (d->n_blocks == 0) return RQ_OK;
    hipPointerAttribute_t pa;
    if (!d->status || hipPointerGetAttributes(&pa, d->status) != hipSuccess || pa.type != hipMemoryTypeHost) {
        (void)hipGetLastError();
        return fail(RQ_ERR_BAD_ARG, "rq_decode_batch_async: status must be pinned host memory");
    }
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    CtxRef ctx;
    if ((rc = get_ctx(&ctx))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    // the device's view of the pinned status array (k_solve writes the final statuses straight into it)
    int32_t* status_dev = static_cast<int32_t*>(pa.devicePointer);
    return decode_locked(ctx, p, d->T, d->n_blocks, d->data, d->data_stride, d->n_erased, d->erased, d->n_repair,
                         d->repair_esi, d->repair, d->status, d->stream, nullptr, Fin::Async, status_dev);
}

int rq_encode_batch_host(const rq_encode_desc* d, uint32_t device_mask) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->K == 0 || (!d->src && d->n_blocks)) return fail(RQ_ERR_BAD_ARG, "bad encode descriptor (K, src)");
    if (d->n_blocks == 0 || d->n_esi == 0) return RQ_OK;
    if (!d->esi || !d->out) return fail(RQ_ERR_BAD_ARG, "n_esi without esi/out");
    if (d->src_stride < (uint64_t)d->K * d->T || d->out_stride < (uint64_t)d->n_esi * d->T)
        return fail(RQ_ERR_BAD_ARG, "stride smaller than a block");
    if (d->c_out) return fail(RQ_ERR_BAD_ARG, "c_out is not supported by the host-memory batch");
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    return run_sharded(device_mask, d->n_blocks,
                       [&](int dev, uint32_t b0, uint32_t b1) { return encode_host_shard(dev, *d, p, b0, b1); });
}

int rq_decode_batch_host(const rq_decode_desc* d, uint32_t device_mask) {
    if (!d || d->T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (d->K == 0) return fail(RQ_ERR_BAD_ARG, "bad decode descriptor (K)");
    if (d->n_blocks == 0) return RQ_OK;
    if (!d->data || !d->n_erased || !d->n_repair || !d->status) return fail(RQ_ERR_BAD_ARG, "null decode array");
    if (d->data_stride < (uint64_t)d->K * d->T) return fail(RQ_ERR_BAD_ARG, "stride smaller than a block");
    Params p;
    int rc = params_for_K(d->K, &p);
    if (rc) return fail(rc, "k is too big");
    std::vector<uint64_t> eoff(d->n_blocks + 1, 0), roff(d->n_blocks + 1, 0);
    for (uint32_t b = 0; b < d->n_blocks; ++b) {
        eoff[b + 1] = eoff[b] + d->n_erased[b];
        roff[b + 1] = roff[b] + d->n_repair[b];
    }
    HostDecode h;
    h.T = d->T; h.K = d->K;
    h.n_erased = d->n_erased; h.erased = d->erased; h.n_repair = d->n_repair; h.repair_esi = d->repair_esi;
    h.status = d->status;
    for (uint32_t b = 0; b < d->n_blocks; ++b) {
        h.data.push_back(static_cast<uint8_t*>(d->data) + b * d->data_stride);
        h.rep.push_back(static_cast<const uint8_t*>(d->repair) + roff[b] * d->T);
    }
    return run_sharded(device_mask, d->n_blocks, [&](int dev, uint32_t b0, uint32_t b1) {
        return decode_host_shard(dev, h, p, b0, b1, eoff, roff);
    });
}

int rq_decode_blocks_host(uint32_t K, uint32_t T, rq_block_io* blocks, uint32_t n_blocks, uint32_t device_mask) {
    if (T == 0) return fail(RQ_ERR_SYMBOL_SIZE_ZERO, "symbol size cannot be zero");
    if (K == 0) return fail(RQ_ERR_BAD_ARG, "bad decode arguments (K)");
    if (n_blocks == 0) return RQ_OK;
    if (!blocks) return fail(RQ_ERR_BAD_ARG, "null blocks");
    Params p;
    int rc = params_for_K(K, &p);
    if (rc) return fail(rc, "k is too big");
    HostDecode h;
    h.T = T; h.K = K;
    std::vector<uint32_t> ne(n_blocks), nr(n_blocks), er, re;
    std::vector<int32_t> st(n_blocks, 0);
    std::vector<uint64_t> eoff(n_blocks + 1, 0), roff(n_blocks + 1, 0);
    for (uint32_t b = 0; b < n_blocks; ++b) {
        const rq_block_io& x = blocks[b];
        if (!x.data || (x.n_erased && !x.erased) || (x.n_repair && (!x.repair || !x.repair_esi)))
            return fail(RQ_ERR_BAD_ARG, "null block buffer");
        ne[b] = x.n_erased;
        nr[b] = x.n_repair;
        er.insert(er.end(), x.erased, x.erased + x.n_erased);
        re.insert(re.end(), x.repair_esi, x.repair_esi + x.n_repair);
        eoff[b + 1] = eoff[b] + ne[b];
        roff[b + 1] = roff[b] + nr[b];
        h.data.push_back(x.data);
        h.rep.push_back(x.repair);
    }
    er.push_back(0);
    re.push_back(0);
    h.n_erased = ne.data(); h.erased = er.data(); h.n_repair = nr.data(); h.repair_esi = re.data();
    h.status = st.data();
    rc = run_sharded(device_mask, n_blocks, [&](int dev, uint32_t b0, uint32_t b1) {
        return decode_host_shard(dev, h, p, b0, b1, eoff, roff);
    });
    for (uint32_t b = 0; b < n_blocks; ++b) blocks[b].status = st[b];
    return rc;
}

void* rq_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        fail(RQ_ERR_DEVICE, "hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

void rq_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// ---------------- per-object encoder (CreateEncoder / GenSymbol) ----------------
// CreateEncoder computes the intermediate symbols C on the GPU (the column program with all L
// outputs, one program per K', cached on disk) and gathers the first repair symbols K..K+R_hw-1 in
// the same stream (k_gather), so the GenSymbol calls a sender makes (0..N-1, transfer.go:180,
// raptorq_eval main.go:216) are served from host memory without touching the GPU.  Other ESIs are
// gathered from the device-resident C on demand.
constexpr uint32_t high_water(uint32_t K) { return K / 4 > 32 ? K / 4 : 32; }

int obj_stream(DevCtx* ctx, hipStream_t* s) {  // per-device stream of the per-object API (ctx->mu held)
    if (!ctx->obj_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->obj_stream, hipStreamNonBlocking));
    *s = ctx->obj_stream;
    return RQ_OK;
}

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
    e->Tp = pad_row(T);
    e->src.assign((size_t)p.K * e->Tp, 0);
    for (uint32_t i = 0; i < p.K; ++i) {
        const size_t off = (size_t)i * T;
        const size_t n = off >= len ? 0 : std::min<size_t>(T, len - off);
        if (n) std::memcpy(&e->src[(size_t)i * e->Tp], data + off, n);
    }
    CtxRef ctx;
    if ((rc = get_ctx(&ctx))) { *err = rc; return nullptr; }
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t st;
    if ((rc = ensure_tables(ctx)) || (rc = obj_stream(ctx, &st))) { *err = rc; return nullptr; }
    const uint32_t R = high_water(p.K);
    if ((rc = e->d_src.ensure(e->src.size())) || (rc = e->d_C.ensure((size_t)p.L * e->Tp)) ||
        (rc = e->d_esi.ensure(R * 4)) || (rc = e->d_out.ensure((size_t)R * e->Tp)) ||
        (rc = ctx->obj_h.ensure(std::max<size_t>(e->src.size(), (size_t)R * e->Tp)))) { *err = rc; return nullptr; }
    // source and the high-water ESI list travel in one pinned upload
    uint8_t* h = ctx->obj_h.as<uint8_t>();
    std::memcpy(h, e->src.data(), e->src.size());
    std::vector<uint32_t> esi(R);
    for (uint32_t i = 0; i < R; ++i) esi[i] = p.K + i;
    if (hipMemcpyAsync(e->d_src.p, h, e->src.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(e->d_esi.p, esi.data(), R * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        *err = fail(RQ_ERR_DEVICE, "hipMemcpyAsync H2D failed");
        return nullptr;
    }
    ColKernel* k;
    if ((rc = get_col_kernel(ctx, p, nullptr, 0, true, &k)) ||
        (rc = launch_col(ctx, k, e->Tp, 1, e->d_src.p, e->src.size(), e->d_C.p, (uint64_t)p.L * e->Tp, st))) {
        *err = rc;
        return nullptr;
    }
    if (launch_gather(dev_params(p), e->d_C.as<uint8_t>(), e->Tp, e->d_esi.as<uint32_t>(), R, e->d_out.as<uint8_t>(), st)) {
        *err = fail(RQ_ERR_DEVICE, "k_gather launch failed");
        return nullptr;
    }
    if (hipMemcpyAsync(h, e->d_out.p, (size_t)R * e->Tp, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        *err = fail(RQ_ERR_DEVICE, "encode failed");
        return nullptr;
    }
    e->rep.assign(h, h + (size_t)R * e->Tp);
    e->n_rep = R;
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
        else if (esi - K < e->n_rep) std::memcpy(out + (size_t)i * T, &e->rep[(size_t)(esi - K) * e->Tp], T);
        else rep.push_back((uint32_t)esi);
    }
    if (rep.empty()) return RQ_OK;
    CtxRef ctx;
    int rc = get_ctx(&ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t st;
    if ((rc = obj_stream(ctx, &st)) || (rc = e->d_esi.ensure(rep.size() * 4)) ||
        (rc = e->d_out.ensure(rep.size() * e->Tp)) || (rc = ctx->obj_h.ensure(rep.size() * e->Tp)))
        return rc;
    HIP_TRY(hipMemcpyAsync(e->d_esi.p, rep.data(), rep.size() * 4, hipMemcpyHostToDevice, st));
    const int le = launch_gather(dev_params(e->p), e->d_C.as<uint8_t>(), e->Tp, e->d_esi.as<uint32_t>(),
                                 (uint32_t)rep.size(), e->d_out.as<uint8_t>(), st);
    if (le) return fail(RQ_ERR_DEVICE, "k_gather launch failed");
    const uint8_t* buf = ctx->obj_h.as<uint8_t>();
    HIP_TRY(hipMemcpyAsync(ctx->obj_h.p, e->d_out.p, rep.size() * e->Tp, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    size_t r = 0;
    for (uint32_t i = 0; i < count; ++i) {
        const uint64_t esi = (uint64_t)first + i;
        if (esi >= K && esi - K >= e->n_rep) std::memcpy(out + (size_t)i * T, &buf[(r++) * e->Tp], T);
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

rq_tracker* rq_tracker_create(uint64_t data_size, uint32_t T, int* err) {
    int dummy;
    if (!err) err = &dummy;
    Params p;
    const int rc = calc_params(data_size, T, &p);
    if (rc) { *err = fail(rc, rc == RQ_ERR_SYMBOL_SIZE_ZERO ? "failed to calc params: symbol size cannot be zero"
                                                           : "failed to calc params: k is too big"); return nullptr; }
    rq_tracker* t = new rq_tracker();
    t->p = p;
    t->T = T;
    t->have.assign(p.K, 0);
    *err = RQ_OK;
    return t;
}

uint32_t rq_tracker_k(const rq_tracker* t) { return t ? t->p.K : 0; }

int rq_tracker_add(rq_tracker* t, uint32_t esi, size_t len, int* can_try) {
    if (!t) return fail(RQ_ERR_BAD_ARG, "null tracker");
    if (len != t->T) {  // the decoder's check and message (RQ/decoder.go:39-57)
        char buf[96];
        std::snprintf(buf, sizeof buf, "incorrect symbol size %zu, should be %u", len, t->T);
        return fail(RQ_ERR_SYMBOL_SIZE, buf);
    }
    if (esi < t->p.K) {
        if (!t->have[esi]) {
            t->have[esi] = 1;
            t->nfast++;
        }
    } else {
        t->slow.insert(esi);
    }
    if (can_try) *can_try = t->p.K <= t->nfast + (uint32_t)t->slow.size();
    return RQ_OK;
}

uint32_t rq_tracker_held(const rq_tracker* t) { return t ? t->nfast + (uint32_t)t->slow.size() : 0; }

void rq_tracker_free(rq_tracker* t) { delete t; }

// Decode: the library's fast path when every source symbol is held; otherwise the batched syndrome
// decode on one block (subset of e + 8 received repairs first, all of them if that is
// rank-deficient), staged through the device's pinned per-object buffer and stream.
int rq_decoder_decode(rq_dec* d, uint8_t* out, int* ok) {
    if (!d || !ok) return fail(RQ_ERR_BAD_ARG, "null decoder/ok");
    const uint32_t K = d->p.K, T = d->T;
    *ok = 0;
    if (K > d->nfast + (uint32_t)d->slow.size()) return fail(RQ_ERR_NOT_ENOUGH, "not enough symbols to decode");
    if (d->nfast < K) {
        const uint32_t Tp = pad_row(T);
        std::vector<uint32_t> erased, resi;
        for (uint32_t i = 0; i < K; ++i)
            if (!d->have[i]) erased.push_back(i);
        CtxRef ctx;
        int rc = get_ctx(&ctx);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(ctx->mu);
        hipStream_t st;
        const size_t data_b = (size_t)K * Tp, rep_b = std::max<size_t>((size_t)d->slow.size() * Tp, 4);
        if ((rc = obj_stream(ctx, &st)) || (rc = ctx->obj_h.ensure(data_b + rep_b)) ||
            (rc = ctx->obj_d.ensure(data_b + rep_b)))
            return rc;
        uint8_t* h = ctx->obj_h.as<uint8_t>();
        if (Tp == T) {
            std::memcpy(h, d->fast.data(), data_b);
        } else {
            std::memset(h, 0, data_b);
            for (uint32_t i = 0; i < K; ++i) std::memcpy(h + (size_t)i * Tp, &d->fast[(size_t)i * T], T);
        }
        size_t r = 0;
        for (auto& kv : d->slow) {
            resi.push_back(kv.first);
            std::memcpy(h + data_b + (r++) * Tp, kv.second.data(), T);
        }
        uint8_t* dd = ctx->obj_d.as<uint8_t>();
        HIP_TRY(hipMemcpyAsync(dd, h, data_b + r * Tp, hipMemcpyHostToDevice, st));
        const uint32_t ne = (uint32_t)erased.size(), nr = (uint32_t)resi.size();
        int32_t status = 0;
        PackOut po;
        rc = decode_locked(ctx, d->p, Tp, 1, dd, data_b, &ne, erased.data(), &nr, resi.data(), dd + data_b, &status, st,
                           &po);
        if (rc) return rc;
        if (status != 1) return RQ_OK;  // rank-deficient: (false, nil, nil)
        for (size_t i = 0; i < erased.size(); ++i)
            std::memcpy(&d->fast[(size_t)erased[i] * T], po.rows.data() + i * Tp, T);
        // The library fills the missing rows into its own buffer as well (RQ/decoder.go:126-130).
        for (uint32_t i : erased) { d->have[i] = 1; d->nfast++; }
    }
    std::memcpy(out, d->fast.data(), d->size);
    *ok = 1;
    return RQ_OK;
}

void rq_decoder_free(rq_dec* d) { delete d; }

}  // extern "C"
