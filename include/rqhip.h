/*
 * rqhip.h -- C-ABI of the MI355X-native RaptorQ engine (librqhip.so).
 *
 * Drop-in boundary for the reference's go/fec RaptorQ path (go/fec/raptorq_wrap.go:13-124),
 * which wraps github.com/xssnick/raptorq v1.1.0.  Plain pointers and sizes only: no HIP or
 * torch types, so a cgo shim needs no ROCm headers (see INTEGRATION.md for the Go binding).
 * Device pointers appear only in the batch API and are documented as such; streams are passed
 * as opaque `void*` (a hipStream_t, or NULL for the null stream).
 *
 * Error model: functions return 0 (RQ_OK) or a negative RQ_ERR_* code; rq_strerror() gives the
 * reference's message text where one exists; rq_last_error() gives the detail of the calling
 * thread's last failure.  No exceptions cross the ABI.  Handles are independent: distinct
 * handles may be used concurrently from different threads (the reference Decoder is not
 * thread-safe per handle, and neither is this one).
 */
#ifndef RQHIP_H
#define RQHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RQ_OK 0
#define RQ_ERR_SYMBOL_SIZE_ZERO (-1) /* "symbol size cannot be zero"      RQ/params.go:31-61   */
#define RQ_ERR_K_TOO_BIG (-2)        /* "k is too big"                    RQ/raw-params.go:14  */
#define RQ_ERR_NOT_ENOUGH (-3)       /* "not enough symbols to decode"    RQ/decoder.go:65-66  */
#define RQ_ERR_SYMBOL_SIZE (-4)      /* "incorrect symbol size %d, should be %d" RQ/decoder.go:39-57 */
#define RQ_ERR_BAD_ARG (-5)          /* wrapper argument errors ("bad K or L", "bad N/K/L", ...) */
#define RQ_ERR_DEVICE (-6)           /* HIP runtime failure or no usable gfx950 device            */
#define RQ_ERR_UNSUPPORTED (-7)      /* shape outside the device path's limits    */
#define RQ_ERR_PLAN (-8)             /* schedule compiler failure (singular system; never expected) */

const char* rq_strerror(int code);
const char* rq_last_error(void);

/* ---------------- parameters (xssnick calcParams, RQ/params.go:31-61) ---------------- */
/* out[11] = {K, K', J, S, H, W, L, P, P1, U, B} for a payload of `size` bytes, symbol size T.
 * P1 is the smallest prime strictly greater than P (the library's deviation from RFC 6330). */
int rq_params(uint64_t size, uint32_t T, uint32_t out[11]);

/* ---------------- encoder: replaces rqq.NewRaptorQ(L).CreateEncoder(data) -----------------
 * go/fec/raptorq_wrap.go:29-40 (NewRaptorQEncoder), :44-46 (GenSymbol), :49 (BaseSymbolsNum);
 * library RQ/encoder.go:15-41.  The payload is copied; symbols are computed on the GPU. */
typedef struct rq_enc rq_enc;
rq_enc* rq_encoder_create(const uint8_t* data, size_t len, uint32_t T, int* err);
uint32_t rq_encoder_k(const rq_enc* e);           /* BaseSymbolsNum: library K = ceil(len/T) */
uint32_t rq_encoder_symbol_size(const rq_enc* e);
/* GenSymbol(esi): T bytes into out.  esi < K -> padded source symbol, else repair symbol. */
int rq_encoder_symbol(rq_enc* e, uint32_t esi, uint8_t* out);
/* count consecutive symbols first_esi.. into out (count*T bytes); one GPU launch for repairs. */
int rq_encoder_symbols(rq_enc* e, uint32_t first_esi, uint32_t count, uint8_t* out);
void rq_encoder_free(rq_enc* e);

/* ---------------- decoder: replaces rqq.NewRaptorQ(L).CreateDecoder(size) -----------------
 * go/fec/raptorq_wrap.go:52-74; library RQ/decoder.go:23-134. */
typedef struct rq_dec rq_dec;
rq_dec* rq_decoder_create(uint64_t data_size, uint32_t T, int* err);
uint32_t rq_decoder_k(const rq_dec* d);           /* FastSymbolsNumRequired (RQ/decoder.go:61) */
/* AddSymbol: *can_try = (K <= unique symbols held), the library's bool (RQ/decoder.go:47,57). */
int rq_decoder_add(rq_dec* d, uint32_t esi, const uint8_t* sym, size_t len, int* can_try);
/* Decode: *ok = 1 and data_size bytes in out; *ok = 0 if the system is rank-deficient
 * (library returns (false, nil, nil)); RQ_ERR_NOT_ENOUGH if fewer than K unique symbols. */
int rq_decoder_decode(rq_dec* d, uint8_t* out, int* ok);
void rq_decoder_free(rq_dec* d);

/* ---------------- batched, device-resident API (the hot path) ---------------------------
 * All blocks of one call share T and K (hence K').  Pointers marked (device) are HIP device
 * memory on the current device; (host) are host memory.  Work is enqueued on `stream`;
 * rq_encode_batch returns without synchronising, rq_decode_batch synchronises once to report
 * per-block status. */
typedef struct {
    uint32_t T;              /* symbol size in bytes: a multiple of 4, at least 8 (device-resident
                                calls; the host-memory calls take any T and pad rows internally) */
    uint32_t K;              /* source symbols per block (library K)                           */
    uint32_t n_blocks;
    const void* src;         /* (device) block b symbol i at src + b*src_stride + i*T          */
    uint64_t src_stride;     /* bytes between blocks (>= K*T)                                  */
    uint32_t n_esi;          /* repair symbols to generate per block                           */
    const uint32_t* esi;     /* (host) n_esi ESIs (>= K), the same for every block             */
    void* out;               /* (device) repair r of block b at out + b*out_stride + r*T       */
    uint64_t out_stride;     /* bytes between blocks (>= n_esi*T)                              */
    void* c_out;             /* optional (device): intermediate symbols, L rows per block      */
    uint64_t c_stride;
    void* stream;            /* hipStream_t or NULL                                            */
} rq_encode_desc;
int rq_encode_batch(const rq_encode_desc* d);

typedef struct {
    uint32_t T, K, n_blocks;
    void* data;                  /* (device) block b source row i at data + b*data_stride + i*T;
                                    received rows present, erased rows are overwritten on success */
    uint64_t data_stride;
    const uint32_t* n_erased;    /* (host) [n_blocks] erased source symbols per block          */
    const uint32_t* erased;      /* (host) concatenated erased source ESIs (< K), unique        */
    const uint32_t* n_repair;    /* (host) [n_blocks] received repair symbols per block        */
    const uint32_t* repair_esi;  /* (host) concatenated repair ESIs (>= K), unique per block   */
    const void* repair;          /* (device) repair rows (T bytes each) in repair_esi order     */
    int32_t* status;             /* (host out) [n_blocks]: 1 decoded, 0 rank-deficient (every
                                    received symbol considered), RQ_ERR_NOT_ENOUGH if received < K.
                                    Any erasure count; at most 65535 received repairs per block
                                    (RQ_ERR_UNSUPPORTED beyond).                                  */
    void* stream;
} rq_decode_desc;
int rq_decode_batch(const rq_decode_desc* d);
/* The same without the final synchronisation: returns once the work is queued on d->stream, and
 * d->status, which must be pinned host memory (hipHostMalloc), holds the per-block results once
 * the stream has reached the end of this call's work (ST_PENDING = -100 until then for the blocks
 * that go to the solver).  Lets a caller queue the next batch while this one runs. */
int rq_decode_batch_async(const rq_decode_desc* d);

/* ---------------- batched, host-memory API (fecquic windows) ------------
 * The batch path for callers without device memory (the cgo shim): the same descriptors, with
 * src/out (encode) and data/repair (decode) in HOST memory; `stream` and `c_out` are not used.
 * Any symbol size T (the device-resident API needs T % 4 == 0; here rows are padded in staging).
 * Blocks are split contiguously over the devices of device_mask (bit d = HIP device d; 0 = the
 * calling thread's device), one host thread per device, no device-to-device traffic.  Each device
 * pipelines H2D, kernels and D2H over two internal streams in chunks of blocks.  Synchronous.
 * Pinned buffers (hipHostMalloc / hipHostRegister) copy at full PCIe rate; pageable ones work.
 * Decode uploads each data block once and downloads only the recovered rows (e*T bytes per
 * block) into `data`; blocks whose status is not 1 are left as they were.
 * Replaces: the per-block GenSymbol loop of fecquic's sender window (go/fecquic/transfer.go:166-268)
 * and the per-block Decode of the receiver workers (go/fecquic/rxbuf.go:336-377). */
int rq_encode_batch_host(const rq_encode_desc* d, uint32_t device_mask);
int rq_decode_batch_host(const rq_decode_desc* d, uint32_t device_mask);

/* Host-memory decode of blocks that each live in their own buffers -- a receiver's per-block
 * staging (go/fecquic/rxbuf.go keeps each block's symbols in its own slabs, :436-468): block b's
 * K*T data bytes at data (received source rows in place, erased rows overwritten on success) and its
 * n_repair received repair rows, consecutive, at repair, in repair_esi order.  All blocks of one call
 * share K and T.  status as in rq_decode_desc.  Synchronous; device_mask as above. */
typedef struct {
    uint8_t* data;
    const uint8_t* repair;
    uint32_t n_erased;
    const uint32_t* erased;
    uint32_t n_repair;
    const uint32_t* repair_esi;
    int32_t status;              /* out */
} rq_block_io;
int rq_decode_blocks_host(uint32_t K, uint32_t T, rq_block_io* blocks, uint32_t n_blocks, uint32_t device_mask);

/* Pinned (page-locked) host memory for ingest staging, so H2D copies run at full PCIe rate
 * (hipHostMalloc).  NULL on failure. */
void* rq_host_alloc(size_t bytes);
void rq_host_free(void* p);

/* ---------------- device control ---------------- */
int rq_device_count(void);
int rq_set_device(int device);      /* selects the HIP device for subsequent calls on this thread */
/* The library keeps per-stream device workspaces for the batched device-resident calls (descriptors,
 * syndromes, scratch).  At most 8 caller streams per device keep one: beyond that the least recently
 * used is retired, and freed once the work of its last call has completed (an event recorded on its
 * stream; no device synchronisation).  rq_stream_release retires the workspace of `stream` (a
 * hipStream_t; NULL = the default stream) on the current device the same way -- call it when a stream
 * is retired.  No reference counterpart (the Go library has no device state). */
int rq_stream_release(void* stream);
/* Releases every device resource of the library (workspaces, compiled programs, internal streams and
 * events, staging) after synchronising each device.  Optional: nothing is released at process exit
 * (static teardown may run after the HIP runtime's), so a process that wants a clean HIP teardown
 * calls this before exiting.  Any later call re-creates what it needs.  Safe beside concurrent calls:
 * each call holds its device context until it returns, and a context taken out by rq_shutdown is
 * destroyed when the last such call returns (in that call's thread). */
int rq_shutdown(void);

/* Measurement (bench.py's roofline): while timing is on for the current device, every column-program
 * launch (the encode hot path and decode's syndrome pass) is issued with start / stop events recorded
 * by its own dispatch (hipExtModuleLaunchKernel), so the time is the kernel's alone, with no marker
 * command between it and its neighbours.  rq_launch_time waits for the launches timed since the last
 * reset and returns their summed milliseconds and count (reset != 0: then starts a new window).  No
 * reference counterpart. */
int rq_launch_timing(int enable);
int rq_launch_time(double* ms_total, uint32_t* n_launches, int reset);

/* ---------------- diagnostics (host only; tests and tools) ----------------
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
/* Allocate the column program (opts = {n_vgpr, n_agpr, la_load, la_reload, max_vmem, n_lds + 1},
 * 0 = default), emulate the machine program on one block when src/out are given (checks vmcnt and
 * lgkmcnt waits and scratch ordering), and optionally return its gfx950 assembly (size first with
 * NULL).  stats[0..17] = {instructions, valu, src loads, out stores, spill stores, spill loads,
 * accw, accr, waits, nops, unprefetched reloads, scratch slots, ir nodes, xtimes, LDS spill
 * stores, LDS reloads, lgkm waits, LDS slots}. */
int rq_debug_colprog_emulate(uint32_t K, uint32_t T, const uint32_t* esi, uint32_t n_out, const uint8_t* src,
                             uint8_t* out, const uint32_t opts[6], uint32_t stats[18], char* asm_buf, size_t asm_cap,
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
 * leave it) and returns the previous one; both give the same bytes. */
uint32_t rq_debug_apply_mode(uint32_t mode);
/* The decode's first solve pass (e <= 64): 1 = in place (k_solve_ip: rows of e bytes, the eliminated
 * column holds the pivot row's identity column), 0 = Gauss-Jordan on [M | I] (k_solve_pq).  Sets the
 * mode (values > 1 leave it) and returns the previous one; both give the same X. */
uint32_t rq_debug_solve_mode(uint32_t mode);
/* The register-table apply kernel's assembly for shape (KC outputs per wave, groups of G syndromes,
 * loads PDG groups ahead, CPL dword columns per lane in bits 7:0 of cpl, two subset numbers per index
 * dword when bit 8 is set): copied into text (cap bytes, NUL-terminated) when given, its length in
 * *text_len, and, when code_bytes is given, assembled in process (its code object size). */
int rq_debug_apply_gi_asm(uint32_t kc, uint32_t g, uint32_t pdg, uint32_t cpl, char* text, size_t cap, size_t* text_len,
                          size_t* code_bytes);
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
#endif /* RQHIP_H */
