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

/* ---------------- AddSymbol bookkeeping without the symbol bytes ----------------------------
 * A receiver that stages symbols itself (go/fecquic's ingest writes each symbol once into its block's
 * pinned staging, rxbuf.go:497-538) still needs the decoder's AddSymbol bool to decide readiness
 * (rxbuf.go:472: haveU counts the true returns).  The tracker is that bookkeeping alone: the same
 * checks and the same bool as rq_decoder_add (RQ/decoder.go:39-57: len != T -> "incorrect symbol size
 * %d, should be %d"; duplicates ignored; *can_try = K <= unique symbols held), no copy, no device work.
 * The staged block is then decoded by rq_decode_blocks_host. */
typedef struct rq_tracker rq_tracker;
rq_tracker* rq_tracker_create(uint64_t data_size, uint32_t T, int* err);  /* NewRaptorQDecoder's params */
uint32_t rq_tracker_k(const rq_tracker* t);       /* library K = ceil(data_size / T)           */
int rq_tracker_add(rq_tracker* t, uint32_t esi, size_t len, int* can_try);
uint32_t rq_tracker_held(const rq_tracker* t);    /* unique symbols held                        */
void rq_tracker_free(rq_tracker* t);

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

#ifdef __cplusplus
}
#endif
#endif /* RQHIP_H */
