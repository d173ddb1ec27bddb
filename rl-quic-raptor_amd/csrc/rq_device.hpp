// rq_device.hpp -- argument blocks shared by the host runtime (rq_engine.cpp) and the HIP
// kernels (rq_kernels.hip).  Plain structs, passed by value as kernel arguments.
#pragma once
#include <cstdint>

namespace rq {

// Per-K' constants the device needs to recompute LT tuples (RQ/params.go:83-112).
struct DevParams {
    uint32_t K, Kp, J, S, H, W, L, P, P1;
};

struct EncArgs {
    DevParams p;
    const uint8_t* src;        // block b row i at src + b*src_stride + i*T
    uint64_t src_stride;
    uint32_t T;                // bytes, multiple of 4
    uint32_t n_slots;
    uint32_t sd;               // strip width in dwords (<= group size)
    uint32_t n_levels;
    const uint16_t* load_slot; // [K']
    const uint32_t* wstream;   // wave program (WaveProgram::words)
    const uint32_t* wave_off;  // [n_waves] stream offsets
    uint32_t n_waves;
    const uint16_t* col_slot;  // [L]
    const uint32_t* blk_map;   // optional: grid.y -> block index
    // erasures (decode): per block [erased_off[b], erased_off[b+1]) into erased[] (source ESIs)
    const uint32_t* erased_off;
    const uint32_t* erased;
    // outputs: shared ESI list (esi, n_out) or per block [out_off[b], out_off[b+1]) of out_esi
    const uint32_t* out_esi;
    uint32_t n_out;
    const uint32_t* out_off;   // optional per-block ranges (decode)
    uint8_t* out;              // shared list: out + b*out_stride + r*T; per-block: out + o*T
    uint64_t out_stride;
    const uint8_t* xor_in;     // optional, indexed like out (syndrome: received repair rows)
    uint8_t* c_out;            // optional intermediate symbols: c_out + b*c_stride + c*T
    uint64_t c_stride;
    unsigned long long* stamp; // diagnostics only: s_memtime per level of workgroup (0,0), or null
    uint32_t dbg;              // ablation bits (timing experiments only): 1 no source loads, 2 no program, 4 no outputs
};

struct SolveArgs {
    DevParams p;
    const uint32_t* blk_map;    // grid.x -> block index
    const uint32_t* erased_off; // per block ranges into erased[]
    const uint32_t* erased;
    const uint32_t* rep_off;    // per block ranges into rep_esi[]
    const uint32_t* rep_esi;
    const uint8_t* cid;         // A^-1 restricted to source columns: L rows x cid_stride bytes
    uint32_t cid_stride;
    uint8_t* xmat;              // per block max_e*max_e coefficient matrix
    uint16_t* xpiv;             // per block max_e original received-repair indices
    int32_t* status;            // per block: 1 ok, 0 rank-deficient
    uint32_t max_e;
};

struct ApplyArgs {
    const uint32_t* blk_map;
    const uint32_t* erased_off;
    const uint32_t* erased;
    const uint32_t* rep_off;
    const uint8_t* sigma;       // syndromes, rows of T bytes indexed by global repair index
    const uint8_t* xmat;
    const uint16_t* xpiv;
    const int32_t* status;
    uint8_t* data;
    uint64_t data_stride;
    uint32_t T;
    uint32_t max_e;
};

// Launchers (rq_kernels.hip).  Return hipError_t as int.
int launch_encode(const EncArgs& a, uint32_t n_strips, uint32_t n_blocks, uint32_t group, void* stream);
int launch_solve(const SolveArgs& a, uint32_t n_blocks, uint32_t lds_bytes, void* stream);
int launch_apply(const ApplyArgs& a, uint32_t n_strips, uint32_t n_blocks, uint32_t lds_bytes, void* stream);
int launch_gf_selftest(const uint32_t* x, uint32_t n, const uint32_t* tabs, uint32_t* out);
int launch_gather(const DevParams& p, const uint8_t* C, uint32_t T, const uint32_t* esi, uint32_t n, uint8_t* out,
                  void* stream);
int upload_tables();  // rand / degree tables to __constant__ memory (once per device)

}  // namespace rq
