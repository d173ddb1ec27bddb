/*
 * rqhip_debug.h -- test-only diagnostics of librqhip.so (not part of the drop-in boundary).
 *
 * include/rqhip.h is the product C-ABI that the cgo shim binds (go/fec/raptorq_rqhip.go).  The entry
 * points below expose the engine's internals to the test suite and the tools (the column program's IR,
 * allocator and emitter on the host, the decode's kernel choices, the host-memory shard plan); no
 * product caller uses them, and none replaces a reference interface.  The library exports them so the
 * tests can reach them through ctypes; they take and return plain host data like the product entries.
 */
#ifndef RQHIP_DEBUG_H
#define RQHIP_DEBUG_H

#include "rqhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- diagnostics (host only) ----------------
 * The encode hot path is a straight-line gfx950 program generated per (K', K, outputs): the
 * "column program" (rl-quic-raptor_amd/csrc/rq_colprog.hpp).  These entry points expose its
 * stages for verification without a GPU.
 *
 * Build the column program for (K, output ESIs; esi = NULL -> all L intermediate symbols) and,
 * if src/out are given, evaluate its IR on one block on the host (src: K x T, out: n_out x T).
 * stats[0..11] = {nodes, xor2, xor3, xt, xtx, load, store, zero, u, n_pivots,
 *                 n_remaining_rows, n_out}. */
int rq_debug_colprog_eval(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                          uint8_t* out, uint32_t stats[12]);
/* Allocate the column program (opts = {n_vgpr, n_agpr, la_load, la_reload, max_vmem, n_lds + 1,
 * cross-item prefetch rows + 1, its batch, its gap}, 0 = default), emulate the machine program on one block when src/out are given (checks vmcnt and
 * lgkmcnt waits and scratch ordering), and optionally return its gfx950 assembly (size first with
 * NULL).  stats[0..17] = {instructions, valu, src loads, out stores, spill stores, spill loads,
 * accw, accr, waits, nops, unprefetched reloads, scratch slots, ir nodes, xtimes, LDS spill
 * stores, LDS reloads, lgkm waits, LDS slots}. */
int rq_debug_colprog_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                             uint8_t* out, const uint32_t opts[9], uint32_t stats[18], char* asm_buf, size_t asm_cap,
                             size_t* asm_len);
/* Assemble the column program in process (amd_comgr) and return the code object size. */
int rq_debug_colprog_assemble(uint32_t K, const uint32_t* esi, uint32_t n_out, size_t* code_bytes);
/* Tests of the round-4 code-generation guards (rq_comgr.cpp check_registers, ColKernArgs::src_bytes):
 * rq_debug_assemble runs `len` bytes of gfx950 assembly text through the in-process assembler with the
 * register check that precedes every generated program (an architectural VGPR at or above
 * .amdhsa_accum_offset, or an AGPR past the allocation, is RQ_ERR_PLAN with the register named in
 * rq_last_error).  rq_debug_colprog_bound emulates the (K, esi) program on one block with the source
 * buffer resource bounded at src_bytes (dwords at or beyond it read 0, as on the GPU) and returns in
 * row_end 1 + the largest source row the program reads (the engine sets src_bytes = (blocks - 1) *
 * stride + row_end * T). */
int rq_debug_assemble(const char* src, size_t len, size_t* code_bytes);
/* Tests: writes a synthetic column-program cache entry (n_rows source-load rows and n_dma4 four-row staging
 * rows) at `path` in the on-disk cache format and reads it back through the engine's loader;
 * RQ_OK when every byte survives (the loader hashes and returns both row lists). */
int rq_debug_cache_roundtrip(const char* path, uint32_t n_rows, uint32_t n_dma4);
int rq_debug_colprog_bound(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                           uint8_t* out, uint64_t src_bytes, uint32_t* row_end);
/* The two-wave (pair) split of the output program for (K, esi) -- wave A: source loads, forward pass,
 * pushes; wave B: HDPC bit accumulation, dense part, outputs; an LDS ring between them -- evaluated on
 * the host over two consecutive items of one block (the ring carries across items as on the GPU), every
 * ring read checked against the barrier intervals (tests).  cfg = {lag, max transfer, ring slots, wave A's
 * four-row staging quads (UINT32_MAX = none), HDPC rows accumulated by wave A (UINT32_MAX = none)},
 * 0 = the engine's default; stats[16] = A {instructions,
 * VALU, source loads, AGPR moves, ring stores, barriers}, B {instructions, VALU, ring loads, output
 * stores}, ring, transfers, values handed over, LDS bytes per workgroup, A's four-row DMAs, 1 if the
 * program uses the bit-accumulation schedule.
 * code_bytes (optional): the kernel assembled in process. */
int rq_debug_pair_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                          uint8_t* out, const uint32_t cfg[5], uint32_t stats[16], size_t* code_bytes);
/* Tests: the host side of one rq_decode_batch_async call on these descriptor arrays (argument checks,
 * host-decided statuses, the union of the candidate repairs, the descriptor words), no device work;
 * repeated `iters` times, the mean wall time of calls 2..iters in us.  n_idx_words: descriptor words. */
int rq_debug_decode_plan(uint32_t T, uint32_t K, uint32_t n_blocks, const uint32_t* n_erased, const uint32_t* erased,
                         const uint32_t* n_repair, const uint32_t* repair_esi, uint32_t iters, double* us_per_call,
                         uint32_t* n_idx_words);
/* Tests: the single-wave program of (K, esi) re-allocated with four-row staging of its source rows
 * (`quads` quads of four LDS slots, `la` IR nodes ahead, 0 = the engine's default), evaluated on the
 * host over one item (T a multiple of 16).  stats[8] = {instructions, VALU, four-row DMAs, global
 * scratch slots, LDS table slots, LDS slots after them, instructions without staging, 1 if the program
 * uses the bit-accumulation schedule}.  code_bytes (optional): the kernel assembled in process. */
int rq_debug_dma4_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src, uint8_t* out,
                          uint32_t quads, uint32_t la, uint32_t stats[8], size_t* code_bytes);
/* Synchronous decodes first solve each block on its first e + margin received repairs (default 8)
 * and re-solve on all of them only if that subset is rank-deficient.  Sets the margin (tests force
 * the second pass with 0) and returns the previous one.  Results never depend on it. */
uint32_t rq_debug_decode_margin(uint32_t margin);
/* The decode's apply step: 1 (default) = the register-table kernel (k_xbits + the generated
 * rq_apply_gi kernel, rq_applygi.cpp), 0 = k_apply's v_perm byte tables.  Sets the mode (values > 1
 * leave it) and returns the previous one; both give the same bytes.  Mode 1 also takes k_apply for a
 * batch beyond the register-table stream's bound (rq_debug_gi_fits). */
uint32_t rq_debug_apply_mode(uint32_t mode);
/* Experiments library: 1 = with the register-table apply, the first solver launch also XORs the received
 * repair rows into their r0 rows (s = received ^ r0, beside the solves) and the apply loads one row per
 * syndrome; 0 (the default) = the apply loads both rows.  Taken only for T % 16 == 0 and a 16-byte aligned
 * repair buffer.  Sets the switch (values > 1 leave it) and returns the previous one; both give the same
 * bytes.  The release library has no such path: it returns 0 and leaves the switch at 0. */
uint32_t rq_debug_apply_sx(uint32_t on);
/* 1 if a decode whose solve list has n_solve blocks and largest erasure count max_e runs the
 * register-table apply (its index stream: e <= 512 and at most 512 MiB for the list), 0 if k_apply. */
int rq_debug_gi_fits(uint32_t max_e, uint32_t n_solve);
/* The decode's first solve pass (e <= 64), experiments library only: 1 = in place (k_solve_ip: rows of
 * e bytes, the eliminated column holds the pivot row's identity column), 0 = Gauss-Jordan on [M | I]
 * (k_solve_pq).  Sets the mode (values > 1 leave it) and returns the previous one; both give the same X.
 * The release library has k_solve_pq only: it returns 0 and leaves the mode at 0. */
uint32_t rq_debug_solve_mode(uint32_t mode);
/* The register-table apply kernel's assembly for shape (KC outputs per wave, groups of G syndromes,
 * loads PDG groups ahead, CPL dword columns per lane in bits 7:0 of cpl, two subset numbers per index
 * dword when bit 8 is set, one precomputed syndrome row per syndrome instead of the received and r0
 * rows when bit 9 is set): copied into text (cap bytes, NUL-terminated) when given, its length in
 * *text_len, and, when code_bytes is given, assembled in process (its code object size). */
int rq_debug_apply_gi_asm(uint32_t kc, uint32_t g, uint32_t pdg, uint32_t cpl, char* text, size_t cap, size_t* text_len,
                          size_t* code_bytes);
/* The index-mode check every generated apply kernel passes before assembly (rq_applygi.cpp
 * check_apply_gi_asm), on the given text for shape (kc, g, pdg, cpl as above): RQ_OK, or RQ_ERR_PLAN with
 * the offending line in rq_last_error. */
int rq_debug_apply_gi_check(uint32_t kc, uint32_t g, uint32_t pdg, uint32_t cpl, const char* text);
/* The register-table apply's index stream (the shipped shape KC 8, G 5, PDG 2) for one block, written on
 * the host by the same code the solvers and k_xbits run on the GPU (rq_gistream.hpp gi_stream): block
 * index bi of a stream laid out for the batch's largest erasure count max_e; e erased rows (erased[e]),
 * nr received repairs (rep_uidx[nr]: their rows in the n_union-row r0), X[k * e + m] = the coefficient of
 * syndrome m in output k, piv[m] = the received repair (index < nr) of syndrome m; solved = 0 writes the
 * header only (a rank-deficient block).  out: at least (bi + 1) * layout[6] words; layout = {nslm, ngrm,
 * er, of, ix, ix_slice, block} in dwords. */
int rq_debug_gi_stream(uint32_t e, uint32_t max_e, uint32_t solved, const uint8_t* X, const uint16_t* piv,
                       const uint32_t* erased, const uint32_t* rep_uidx, uint32_t nr, uint32_t n_union, uint32_t T,
                       uint32_t bi, uint32_t* out, size_t out_words, uint32_t layout[7]);
/* The engine's LT tuple of ISI X at library K (rq_core.hpp tuple_of; RQ/params.go:83-112):
 * out = {d, a, b, d1, a1, b1}. */
int rq_debug_tuple(uint32_t K, uint32_t X, uint32_t out[6]);
/* The column program's IR schedule for the three rq_debug_colprog_* entry points: -1 (default)
 * chooses like the engine (cost model over the schedules), 0 = one demand-driven column scan,
 * P >= 1 = peeling-order production with P Horner passes.  Returns the previous setting. */
int rq_debug_colprog_passes(int passes);
/* How the host-memory batch calls split n_blocks over the devices of device_mask (0 = the calling
 * thread's device, reported as device 0 here) when n_devices exist: returns the shard count (<= cap
 * entries written: device, first block, end block) or a negative error (a mask bit beyond n_devices:
 * RQ_ERR_BAD_ARG).  virtual_shards > 1 splits a one-device mask over that many host threads. */
int rq_debug_shard_plan(uint32_t device_mask, int n_devices, uint32_t n_blocks, uint32_t virtual_shards, int* dev,
                        uint32_t* b0, uint32_t* b1, uint32_t cap);
/* Sets the virtual shard count the host-memory batch calls use on a one-device mask (tests drive the
 * per-device host threads on one GPU with it); returns the previous value (default 0 = off). */
uint32_t rq_debug_virtual_shards(uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* RQHIP_DEBUG_H */
