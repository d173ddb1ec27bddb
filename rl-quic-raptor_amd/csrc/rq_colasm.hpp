// rq_colasm.hpp -- register allocation, gfx950 assembly emission and CPU emulation of the
// column program (rq_colprog.hpp).
//
// Storage tiers of a value (one dword per lane): arch VGPR (operand of a VALU op), AGPR (one
// v_accvgpr_read/write away; also a direct target/source of buffer loads/stores), a per-wave LDS
// slot (256 B; ds_write/ds_read, off the vector-memory path), and a per-wave global scratch slot
// (256 B per value, L2/MALL-resident in practice).  Allocation is Belady's
// furthest-next-use rule over the straight-line program; source-row loads and scratch reloads
// are issued ahead of their use (look-ahead windows) and waited for with exact vmcnt counts.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rq_colprog.hpp"

namespace rq {

enum MOp : uint8_t {
    MI_XOR2 = 0, MI_XOR3, MI_XT, MI_XTX, MI_ZERO,
    MI_LDSRC,   // d <- source row imm (buffer_load; d is a VGPR or an AGPR)
    MI_STOUT,   // output row imm <- a
    MI_SPST,    // scratch slot imm <- a
    MI_SPLD,    // d <- scratch slot imm
    MI_ACCW,    // AGPR d <- VGPR a
    MI_ACCR,    // VGPR d <- AGPR a
    MI_WAIT,    // s_waitcnt vmcnt(imm)
    MI_NOP,     // s_nop imm
    MI_LDST,    // LDS slot imm <- a (ds_write_b32)
    MI_LDLD,    // d <- LDS slot imm (ds_read_b32)
    MI_WAITL,   // s_waitcnt lgkmcnt(imm)
    MI_DMA,     // LDS slot d <- source row imm (buffer_load ... lds: no register, counts in vmcnt)
    MI_RST,     // pair programs: ring slot imm <- a (ds_write_b32)
    MI_RLD,     // pair programs: d <- ring slot imm (ds_read_b32)
    MI_BAR,     // pair programs: s_barrier (after an lgkmcnt(0) the allocator emits)
    MI_DMAT,    // four-row staging: row offsets of group imm -> reserved table VGPR d (ds_read_b32)
    MI_DMA4,    // four-row staging: the four rows of group imm -> LDS quad d (buffer_load_dwordx4 ... lds)
    // Cross-item prefetch (AllocOpts::cip): MI_HEAD is one of the item's first source loads, d <- row imm,
    // issued by the previous item's MI_PFX (or the kernel prologue for a wave's first item), so it emits
    // nothing in the body; MI_PFX issues the next item's head loads cip_reg / cip_row [imm >> 16, + (imm &
    // 0xffff)) into their registers, which nothing writes after it.
    MI_HEAD,
    MI_PFX,
};

constexpr int REG_A0 = 256;       // register ids: 0..255 VGPR, 256..511 AGPR
constexpr int V_ALLOC = 250;      // at most v0..v249 allocatable; 6 reserved VGPRs sit just above
// Reserved VGPRs of a program with n allocatable VGPRs: v(n)..v(n+5).  lds2 = scroff + 64 KiB
// addresses LDS slots 256.. (the ds offset field is 16 bits).
constexpr int N_RESERVED = 6;
// Four-row staging programs reserve four more just above those: the lane group's table offset
// ((lane / 16) * 4), the lane's 16-B chunk base in the source block, and two table registers.
constexpr int N_RESERVED_DMA4 = 10;
struct Reserved {
    int t2, t1, scroff, outoff, srcoff, lds2, grp4, dmabase, tbl0, tbl1;
    explicit Reserved(uint32_t n)
        : t2((int)n), t1((int)n + 1), scroff((int)n + 2), outoff((int)n + 3), srcoff((int)n + 4), lds2((int)n + 5),
          grp4((int)n + 6), dmabase((int)n + 7), tbl0((int)n + 8), tbl1((int)n + 9) {}
};

struct MInst {
    uint8_t op = MI_NOP;
    int16_t d = -1, a = -1, b = -1, c = -1;
    uint32_t imm = 0;
};

struct AllocOpts {
    uint32_t n_vgpr = V_ALLOC;   // allocatable VGPRs (<= V_ALLOC)
    uint32_t n_agpr = 256;       // allocatable AGPRs
    uint32_t la_load = 320;      // look-ahead (IR nodes) for source-row loads
    uint32_t la_reload = 160;    // look-ahead (IR nodes) for scratch reloads
    uint32_t max_vmem = 56;      // outstanding vector-memory operations per wave
    uint32_t n_lds = 156;        // LDS spill slots per wave (256 B each; 4 waves/CU -> 40 KB; <= 512)
    uint32_t lds_horizon = 200;  // push an LDS resident out only if its next use is this much further
    uint32_t la_dma = 0;         // look-ahead (IR nodes) for LDS-DMA source staging (0 = off)
    // Four-row staging (0 = off): source rows go to LDS four at a time, one buffer_load_dwordx4 ... lds
    // per group of four rows (1 KiB: 16 B per lane, lane group g = lane / 16 on row g), into `dma4`
    // quads of four LDS slots taken from the top of n_lds, la_dma IR nodes ahead; each row then reaches
    // a register by ds_read_b32.  Four times the bytes per outstanding vector-memory operation (the
    // vmcnt budget bounds a wave's bytes in flight).  Needs T and the block stride multiples of 16 and
    // n_vgpr <= 246 (four more reserved VGPRs).
    uint32_t dma4 = 0;
    uint32_t src_bias = 100;     // victim choice: a source row's next use counts this % as far
    uint32_t src_lds = 1;        // evicted source rows may take LDS slots (else dropped at once)
    uint32_t wait_age = 320;     // a vmcnt wait also covers operations issued this many instructions ago
    uint32_t lwait_age = 48;     // the same for lgkmcnt (LDS) waits
    uint32_t load_batch = 1;     // source-row prefetches issued in groups of this many (experiments)
    // Cross-item prefetch: the next item's first `cip` source rows are loaded during this item's load-free
    // tail (after its last source load), cip_batch at a time every cip_gap IR nodes, into registers the
    // tail then leaves alone; the item finds them in place.  0 = off (W > 1, pair and four-row programs,
    // several waves per SIMD).  K=1024: 0.340 -> 0.335 ms per launch (profiles/r06c/cip_ab.log).
    uint32_t cip = 64;
    uint32_t cip_batch = 8;
    uint32_t cip_gap = 24;
    uint32_t cip_agpr = 0;  // experiments: this many more head rows, into the top AGPRs
    uint32_t la_extra = 0, la_free = 96;  // experiments: look-ahead + la_extra while la_free registers are free
};

struct MProg {
    std::vector<MInst> ins;
    uint32_t n_slots = 0;        // scratch slots per wave (256 B each)
    uint32_t n_lds_slots = 0;    // LDS slots per wave used (256 B each)
    uint32_t n_vgpr = V_ALLOC;   // allocatable VGPRs / AGPRs the program was allocated for
    uint32_t n_agpr = 256;
    uint32_t n_out = 0;
    uint32_t K = 0;
    uint32_t wg_waves = 1;       // waves per workgroup (emit_colprog_asm): W consecutive items per CU
    uint32_t lds_base = 0;       // LDS slot of the program's spill slot 0 (pair programs: after the ring)
    uint32_t ring_base = 0;      // LDS slot of ring slot 0 (pair programs: after the four-row table)
    // four-row staging: quads, the first quad slot (spill slots below it), and the rows of every group
    // (4 per group, padded with the group's first row)
    uint32_t dma4_quads = 0, dma4_slot0 = 0;
    std::vector<uint32_t> dma4_rows;
    // cross-item prefetch: the head loads' registers and rows, in issue order (MI_HEAD / MI_PFX)
    std::vector<int16_t> cip_reg;
    std::vector<uint32_t> cip_row;
    struct Stats {
        uint32_t valu = 0, ldsrc = 0, stout = 0, spst = 0, spld = 0, accw = 0, accr = 0, wait = 0, nop = 0;
        uint32_t sync_reload = 0;  // reloads that were not prefetched
        uint32_t ldst = 0, ldld = 0, waitl = 0;  // LDS spill stores / reloads / lgkm waits
        uint32_t migrate = 0;                    // LDS residents pushed out to global scratch
        uint32_t dma = 0;                        // source rows staged through LDS by DMA
        uint32_t rst = 0, rld = 0, bar = 0;      // pair programs: ring stores / loads, barriers
        uint32_t cip_evict = 0;                  // values moved out of the head registers for the prefetch
    } st;
};

bool allocate_colprog(const ColIR& ir, const AllocOpts& o, MProg* mp, std::string* err);

// Builds and allocates the column program for (K, outputs; esi = NULL: all L intermediate symbols),
// choosing the IR schedule (build_colprog's `passes`) that minimises the launch-time model
// colprog_cost: the demand-driven scan when it needs no global scratch, else the number of Horner
// passes that best trades the extra VALU work against spill traffic.  *passes_out = the choice.
// search_waves: a program that fits on chip is re-allocated for 2 / 4 / 8 waves per SIMD while it
// still needs no global scratch and at most 1.5x the instructions (the engine's choice; the debug
// entry points keep the caller's register budget).
bool compile_colprog(const Params& p, const uint32_t* esi, uint32_t n_out, const AllocOpts& o, ColIR* ir, MProg* mp,
                     std::string* err, uint32_t* passes_out = nullptr, bool search_waves = false);
// Model of one launch's time per 64-column item (units: issue slots): every instruction of the one
// resident wave per SIMD takes an issue slot, plus a stall term per global-scratch spill / reload;
// fitted on the K=1024 schedule sweep of round 2 (profiles/r02g).
double colprog_cost(const MProg& mp);

// Kernel argument block of the emitted kernel (must match the prologue in emit_colprog_asm).
struct ColKernArgs {
    uint64_t src;         // block b row i at src + b*src_stride + i*T
    uint64_t out;         // output r of block b at out + b*out_stride + r*T
    uint64_t scratch;     // per-wave scratch: n_slots * 256 bytes per workgroup
    uint32_t src_stride;  // bytes (< 4 GiB spans: the host splits larger batches)
    uint32_t out_stride;
    uint32_t T;           // bytes, multiple of 4
    uint32_t n_cols;      // n_blocks * T/4
    uint32_t magic, shift;  // b = mulhi(g, magic) >> shift == g / (T/4) for g < n_cols
    uint32_t scr_per_wave;  // bytes
    uint32_t xcd_q, xcd_n;  // XCD-aware item order: q = items / 8, n = 8q (0, 0 = identity order)
    uint32_t src_bytes;   // source buffer resource size: the launch's source span (loads beyond it read 0)
    uint32_t n_items;     // workgroup iterations: ceil(64-column items / W) (W = MProg::wg_waves)
    uint32_t n_wg;        // persistent grid size (workgroups): workgroup g takes iterations g, g + n_wg, ...
                          // and its wave w the item iteration * W + w
    uint64_t row_off;     // uint32 table: soffset of the program's j-th source load (colprog_src_rows[j] * T)
    // descriptor fetch (a decode's syndrome launch): workgroups n_wg, n_wg + 1, ... copy cp_bytes (a
    // multiple of 16) from cp_src (pinned host memory) to cp_dst, cp_chunk bytes each, and exit
    uint64_t cp_src;
    uint64_t cp_dst;
    uint32_t cp_bytes, cp_chunk;
};
static_assert(sizeof(ColKernArgs) == 104, "kernarg layout");

std::string emit_colprog_asm(const MProg& mp, const std::string& kname);
// Source rows of the program's buffer loads in issue order (the kernel's row_off table is these
// times T, padded to a multiple of 16 entries).
std::vector<uint32_t> colprog_src_rows(const MProg& mp);
// 1 + the largest source row any load of the program reads (the source resource's extent per block).
uint32_t colprog_row_end(const MProg& mp);
// The kernel's row-offset buffer for symbol size T: colprog_src_rows * T (padded to 16 entries + 16),
// then, for four-row staging, every group's four row offsets (dma4_rows * T).  Both waves of a pair
// read it through the same pointer; colprog_dma4_table_offset is where the group table starts (bytes).
std::vector<uint32_t> colprog_row_table(const MProg& mp, uint32_t T);
uint32_t colprog_dma4_table_offset(const MProg& mp);
// Registers (VGPR + AGPR, allocation granule 8) per lane of the emitted kernel.
uint32_t colprog_regs(const MProg& mp);
uint32_t colprog_acc_off(const MProg& mp);

// Executes the machine program on the host for one block (T/4 lanes), checking vmcnt waits and
// scratch ordering as it goes.  Test infrastructure for the allocator, not a product path.
// src_bytes: the source buffer resource's extent as the kernel sets it (ColKernArgs::src_bytes); a
// source dword at or beyond it reads 0, as a bounds-checked buffer load does on the GPU.
bool emulate_colprog(const MProg& mp, const uint8_t* src, uint32_t T, uint8_t* out, std::string* err,
                     uint64_t src_bytes = UINT64_MAX);

// ---- two-wave (pair) column programs (split_pair in rq_colprog.hpp) ----
struct PairProg {
    MProg A, B;              // wave 0 (A: loads, forward pass, pushes) and wave 1 (B: HDPC, dense, outputs)
    uint32_t lag = 0, ring = 0, n_xfer = 0, n_cross = 0;
    uint32_t bmask = 0;      // IrNode::grp values run by wave B
    uint32_t tbl_slots = 0;  // four-row staging: LDS slots of A's group table (at LDS 0)
};
// Splits and allocates (both waves with the budget of `o`, one wave per SIMD; LDS: A's four-row group
// table, the ring, A's spill slots and quads, B's spill slots; at most 80 KiB per workgroup so that two
// workgroups share a CU).  o.dma4 / o.la_dma apply to wave A (its source rows staged four at a time).
bool compile_pair(const ColIR& ir, const AllocOpts& o, uint32_t bmask, uint32_t lag, uint32_t max_xfer, uint32_t ring,
                  PairProg* pp, std::string* err);
// Model of a pair launch's time per item (issue slots of the longer wave), comparable with
// colprog_cost of a single-wave program.
double pair_cost(const PairProg& pp);
uint32_t pair_lds_bytes(const PairProg& pp);
std::string emit_pair_asm(const PairProg& pp, const std::string& kname);
// Runs wave A's and wave B's machine programs over `iters` consecutive items of one block (the ring
// carries across items as on the GPU), checking that every ring read in B's barrier interval m sees
// the last value A wrote before barrier m and that no A write to that slot lands in interval m.
bool emulate_pair(const PairProg& pp, const uint8_t* src, uint32_t T, uint8_t* out, std::string* err,
                  uint32_t iters = 2);

// In-process assembly (amd_comgr, rq_comgr.cpp): assembly text -> gfx950 code object.
bool comgr_assemble(const std::string& src, std::vector<char>* co, std::string* err);

// magic/shift such that (uint64(g) * magic) >> (32 + shift) == g / d for all g < limit.
// Re-allocate a single-wave program with four-row staging of its source rows (quads of four LDS slots,
// la IR nodes ahead): the group table at LDS 0, spill slots after it (lds_base); one wave per workgroup,
// 16-B aligned rows only.
bool compile_colprog_dma4(const ColIR& ir, const AllocOpts& o, uint32_t quads, uint32_t la, MProg* mp,
                          std::string* err);
bool divmagic(uint32_t d, uint32_t limit, uint32_t* magic, uint32_t* shift);

}  // namespace rq
