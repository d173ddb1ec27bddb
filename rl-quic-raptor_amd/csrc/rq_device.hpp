// rq_device.hpp -- argument blocks shared by the host runtime (rq_engine.cpp) and the HIP
// kernels (rq_kernels.hip).  Plain structs, passed by value as kernel arguments.
//
// The encode hot path is not here: it is a generated straight-line code object per (K', K,
// outputs) (rq_colprog.hpp, rq_colasm.hpp).  These kernels are the decode-side helpers around it
// and the per-object GenSymbol gather.
#pragma once
#include <cstddef>
#include <cstdint>

#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif

namespace rq {

// Per-K' constants the device needs to recompute LT tuples (RQ/params.go:83-112).
struct DevParams {
    uint32_t K, Kp, J, S, H, W, L, P, P1;
};

// Decode, per block b: erased source rows E = erased[erased_off[b] .. erased_off[b+1]) and
// received repair symbols j = rep_off[b] .. rep_off[b+1] (rows of `recv`, T bytes each) whose
// ESIs sit at index rep_uidx[j] of the column program's output list ("union").
//   r0   : column program outputs on the data as received (erased rows hold whatever bytes g_E),
//          n_union rows per block; s = recv ^ r0 = M (x_E ^ g_E)
//   mrep : column program outputs on the identity payload: mrep[u*mrep_stride + i] = coefficient
//          of source row i in output u (the repair rows of G*A^-1 restricted to source columns)
struct PackArgs {
    const uint32_t* blk;        // [n] block index of each recovered row
    const uint32_t* row;        // [n] recovered source row
    uint8_t* data;
    uint64_t data_stride;
    uint32_t T, n;
    uint8_t* pack;              // k_pack_rows: row i of the list -> pack + i*T
};

// Per solved block bi (block b = blk_map[bi], e erased rows): X (e x xs bytes, xs = x_stride(e))
// at xcoef + 64 * xoff[bi], X[k][m] at row m, byte k; the e received repairs it combines (indices
// within the block) at xpiv + erased_off[b].
__host__ __device__ inline uint32_t x_stride(uint32_t e) { return 64u * ((e + 63u) / 64u); }

// The register-table apply (rq_applygi.cpp): x_E = g_E ^ X s as 8 GF(2) bit planes.  Shape: KC outputs
// per wave (8 or 16), syndromes in groups of G (4..6) whose 2^G subset XORs form a table in VGPRs,
// syndrome loads PDG groups ahead (1..2).
struct GiShape {
    uint32_t KC = 8, G = 5, PDG = 2;
    uint32_t CPL = 1;   // dword columns per lane (64-column strips per wave), 1 or 2
    uint32_t PACK = 0;  // 1: two subset numbers per index dword (the high one by s_lshr_b32)
    uint32_t diag = 0;  // experiments (timing only, wrong bytes): 1 no index loads, 2 no syndrome loads, 4 no lookups
    uint32_t stpol = 0; // experiments: recovered-row store policy, 0 plain, 1 nt, 2 sc1, 3 sc0 sc1
    // 1: the syndromes s = received ^ r0 are already in the r0 rows (the first solver launch's XOR
    // workgroups, SolveArgs::sx_wgs, experiments library): one load per syndrome, a ring of G values per slot
    uint32_t SX = 0;
};

// Per block bi of the solve list, the dword stream k_xbits writes at gi + bi * block and the apply kernel
// reads with scalar loads.  The layout is fixed by the batch's largest e (every address follows from
// (bi, slice) and the kernel arguments, so a wave needs one round of scalar loads before its first
// syndrome load); for the block's own e: ngr = ceil(e / G) groups, nsl = ceil(e / KC) slices.
//   header (16 dwords): status (1 = solved), e, ngr, 0, then the 64-bit base addresses of the block's
//            received repair rows, r0 rows and data rows
//   er:      nslm records of 16 dwords: slice s's output row byte offsets (E[s KC + k] * T, 0 past e)
//   of:      ngrm + PDG + 1 records of 16 dwords; record q: (received row, r0 row) byte offsets of
//            syndrome m = G q + t at dwords 2t, 2t + 1 (0 past e: row 0, loaded and never looked up)
//   ix:      per slice ngrm records of 8 KC dwords: record g, output k, bit b = the G-bit subset of group
//            g's syndromes whose coefficients in X[s KC + k] have bit b set
struct GiLayout {
    uint32_t nslm, ngrm;        // slices / groups of the batch's largest e
    uint32_t er, of, ix, ix_slice, block;  // dwords
};
__host__ __device__ inline GiLayout gi_layout(uint32_t max_e, const GiShape& s) {
    GiLayout L;
    L.nslm = (max_e + s.KC - 1) / s.KC;
    L.ngrm = (max_e + s.G - 1) / s.G;
    L.er = 16;
    L.of = L.er + 16 * L.nslm;
    L.ix = L.of + 16 * (L.ngrm + s.PDG + 1);
    L.ix_slice = (s.PACK ? 4 : 8) * s.KC * L.ngrm;
    L.block = L.ix + L.nslm * L.ix_slice;
    return L;
}

struct XbitsArgs {
    const uint32_t* blk_map;
    const int32_t* status;
    const uint32_t* erased_off;
    const uint32_t* erased;
    const uint32_t* rep_off;
    const uint32_t* rep_uidx;
    const uint8_t* xcoef;
    const uint32_t* xoff;
    const uint16_t* xpiv;
    const uint8_t* recv;
    const uint8_t* r0;
    uint8_t* data;
    uint64_t data_stride;
    uint32_t* gi;
    GiLayout L;
    uint32_t T, n_union;
};

struct SolveArgs {
    const uint32_t* blk_map;    // grid.x -> block index
    const uint32_t* erased_off; // per block ranges into erased[]
    const uint32_t* erased;
    const uint32_t* rep_off;    // per block: first received repair row in rep_uidx[] / recv
    const uint32_t* rep_cnt;    // per block: received repairs the solvers may use (the first rep_cnt[b])
    const uint32_t* rep_uidx;
    const uint8_t* mrep;
    uint32_t mrep_stride;
    uint8_t* xcoef;             // X of solved block bi at xcoef + 64 * xoff[bi]
    const uint32_t* xoff;
    uint16_t* xpiv;             // xpiv[erased_off[b] + m]: received repair (index within block b) of X row m
    int32_t* status;            // per block: 1 ok, 0 rank-deficient, ST_FALLBACK (general solver)
    uint8_t* gws;               // general solver: basis of block bi at gws + 64 * goff[bi] when e > lds_e
    const uint32_t* goff;
    uint32_t lds_e;             // largest e whose basis the general solver keeps in LDS
    // host-decided statuses of all n_all blocks (ST_PENDING for the solver's blocks), read by the
    // first solver launch in place of an upload (nullptr: status already holds them)
    const int32_t* status_init;
    uint32_t n_all;
    // first pass (k_solve_pm<1, ...>): use at most e + row_margin received repairs (0 = up to 64); a
    // block rank-deficient on them is deferred to the later passes like one beyond 64
    uint32_t row_margin;
    uint32_t n_map;             // entries of blk_map (the general solver's grid strides over them)
    uint32_t diag_steps;        // experiments builds (RQHIP_SOLVE_STEPS): pivot steps of k_solve_pq (timing only)
    // experiments builds (RQHIP_SOLVE_DIAG, timing only, wrong X): k_solve_pq's step without its pinfo read
    // (1), dependent table read (4), GF(256) row updates (8).  Every mode keeps the pivot choice uniform
    // and within the block's rows (a no-barrier mode did not: the waves chose different pivots, the
    // stream named received rows past the block's, and the apply read past the received-row buffer)
    uint32_t diag;
    // k_solve also writes the register-table apply's index stream (the shipped shape 8, 5, 2) when set
    uint32_t xb_on;
    XbitsArgs xb;
    // k_solve (the last solver launch) also writes every block's final status here: the caller's pinned
    // status array as the device sees it, so an async decode needs no status download (nullptr: none)
    int32_t* host_status;
    // The first solver (k_solve_pq<1, ...>) finishes a block that is rank-deficient on its first e + margin
    // rows with every received repair itself (general_block on its LDS rows) instead of deferring it, and
    // writes host_status for its blocks.  Set when no block has e > 64: no later solver launch then.
    uint32_t inline_general;
    // Experiments library (RQHIP_APPLY_SX=1; measured not to pay):
    // the last sx_wgs workgroups of the first solver launch (k_solve_pq<1, 4>) solve nothing: they XOR
    // every received repair row of the solve list into its r0 row (xb.recv, xb.r0), so the apply reads
    // s = received ^ r0 with one load per syndrome.  They need no HBM bandwidth the solvers use and run
    // on the wave slots the solvers leave free.  0: off.
    uint32_t sx_wgs;
    uint32_t sx_pol;            // experiments (RQHIP_SX_POL): 1 non-temporal s stores, 2 non-temporal received loads
};
constexpr int32_t ST_PENDING = -100;   // queued for the solver
constexpr int32_t ST_FALLBACK = -101;  // beyond the fast solvers: the general solver decides
// General-solver basis row width (coefficients then combination of selected rows), 16-byte aligned.
__host__ __device__ inline uint32_t basis_width(uint32_t e) { return (2u * e + 15u) & ~15u; }

struct ApplyArgs {
    const uint32_t* blk_map;
    const uint32_t* erased_off;
    const uint32_t* erased;
    const uint32_t* rep_off;
    const uint32_t* rep_uidx;
    const uint8_t* recv;        // received repair rows (T bytes each), rep_off order
    const uint8_t* r0;          // n_union rows of T bytes per block
    uint32_t n_union;
    const uint8_t* xcoef;
    const uint32_t* xoff;
    const uint16_t* xpiv;
    const int32_t* status;
    uint8_t* data;
    uint64_t data_stride;
    uint32_t T;
    uint32_t max_e;             // largest e of the batch (slice sizing)
    uint32_t out_sc1 = 0;       // 1: recovered rows stored sc1 (written through, not left dirty in L2)
};

// Kernel arguments of the generated apply kernel; its prologue loads them at these byte offsets.
struct ApplyGiArgs {
    const uint32_t* gi;         // 0
    uint32_t block_bytes;       // 8: 4 * GiLayout::block
    uint32_t of_bytes;          // 12
    uint32_t ix_bytes;          // 16
    uint32_t ix_slice_bytes;    // 20
    uint32_t n_blocks;          // 24: entries of the solve list
    uint32_t T;                 // 28
    uint32_t strips;            // 32: ceil(T / 256)
    uint32_t nsg;               // 36: strip groups of ws waves (one workgroup each)
    uint32_t sg_magic;          // 40: ceil(2^31 / nsg) (y / nsg = (2y * magic) >> 32)
    uint32_t ws;                // 44: waves per workgroup
};
static_assert(sizeof(ApplyGiArgs) == 48, "apply kernel argument layout");

// Launchers (rq_kernels.hip).  Return hipError_t as int.
int launch_xbits(const XbitsArgs& a, uint32_t n_blocks, const GiShape& s, void* stream);
// Host-memory decode: copy the recovered rows (the same (blk, row) list) into a dense buffer so only
// e*T bytes per block travel back over PCIe.
int launch_pack_rows(const PackArgs& a, void* stream);
// Fast solves (e <= 64 on the first 64 received repairs, e <= 128 on the first 128), then the
// general solver (any e, every received repair) for the blocks they deferred.
// need_general: some block may end in the general solver (e or candidate repairs > 64); wide: some
// block has 64 < e <= 128 (the two-row-per-lane fast solver runs first).
// xbits_done (optional): set when the launches also wrote the index stream of a.xb (a.xb_on and k_solve ran).
// sx_done (optional): set when the first launch also ran a.sx_wgs syndrome workgroups (the r0 rows then
// hold s = received ^ r0 for every received repair of the solve list).
int launch_solve(const SolveArgs& a, uint32_t n_blocks, bool need_general, bool wide, uint32_t max_lds_e,
                 void* stream, bool* xbits_done = nullptr, bool* sx_done = nullptr);
int launch_apply(const ApplyArgs& a, uint32_t n_strips, uint32_t n_blocks, void* stream);
int launch_gather(const DevParams& p, const uint8_t* C, uint32_t T, const uint32_t* esi, uint32_t n, uint8_t* out,
                  void* stream);
// General-solver working set for e erased rows; the largest e it keeps in LDS.
size_t solve_ws_bytes(uint32_t e);
uint32_t solve_lds_e_max();
int upload_tables();  // rand / degree tables to __constant__ memory (once per device)
// the first solve pass: 1 = k_solve_ip (in place), 0 = k_solve_pq<1, 4> (rq_debug_solve_mode)
extern uint32_t g_solve_ip;

}  // namespace rq
