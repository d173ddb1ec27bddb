// RaptorQ for package fec on the MI355X engine (librqhip.so, include/rqhip.h).
//
// Drop-in for go/fec/raptorq_wrap.go (reference lines 13-124): delete that file, add this one, and
// point cgo at this repository (the #cgo lines below assume it sits at go/fec/ of this repo; from
// another tree set CGO_CFLAGS=-I<repo>/include and CGO_LDFLAGS=-L<repo>/rl-quic-raptor_amd/build
// -lrqhip instead).  The exported names, signatures, wrapper error strings ("bad K or L",
// "bad dataSize or L", "bad N/K/L") and the Packet type (go/fec/packet_polar.go:87-90) are those
// callers already use: go/fecquic/transfer.go:180, go/fecquic/rxbuf.go:351,437,472 and
// go/cmd/raptorq_eval/main.go:85-103,199-222 compile unchanged.  Library errors carry the library's
// own message (rq_last_error: "symbol size cannot be zero", "not enough symbols to decode", ...).
//
// Ownership: every returned slice is Go memory (copied out of C), except HostAlloc's pinned C memory;
// C keeps no Go pointer (rq_encoder_create and rq_decoder_add copy their inputs; rq_tracker_add reads
// none).  Handles are freed by finalizers.
// tests/test_go_shim.py checks every C.rq_* call here against the prototypes of include/rqhip.h.
package fec

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../rl-quic-raptor_amd/build -lrqhip -Wl,-rpath,${SRCDIR}/../../rl-quic-raptor_amd/build
#include <stdlib.h>
#include "rqhip.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"unsafe"
)

// Wrapper argument errors: the reference's exact strings.
var (
	errBadKL    = errors.New("bad K or L")
	errBadSizeL = errors.New("bad dataSize or L")
	errBadNKL   = errors.New("bad N/K/L")
	// batch-path argument errors (this shim's own API, not the reference's)
	errBadBatch = errors.New("decode blocks: data, repair, erased and repairESI differ in length")
	errShortBuf = errors.New("decode blocks: a block's data or repair slice is shorter than its symbols")
)

type RaptorQEncoder struct {
	K int
	L int
	h *C.rq_enc
}

type RaptorQDecoder struct {
	K    int
	L    int
	h    *C.rq_dec
	size int
}

// libErr turns a non-zero RQ_* code into the library's message for this thread's last failure.
func libErr(code C.int) error {
	if msg := C.GoString(C.rq_last_error()); msg != "" {
		return errors.New(msg)
	}
	return errors.New(C.GoString(C.rq_strerror(code)))
}

func u8ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// NewRaptorQEncoder: K only gates the arguments; the library's K is ceil(len(data)/L).  The encoder's
// intermediate symbols and its first repairs are computed by one GPU launch here.
func NewRaptorQEncoder(data []byte, K, L int) (*RaptorQEncoder, error) {
	if K <= 0 || L <= 0 {
		return nil, errBadKL
	}
	var code C.int
	h := C.rq_encoder_create(u8ptr(data), C.size_t(len(data)), C.uint32_t(L), &code)
	runtime.KeepAlive(data)
	if h == nil {
		return nil, libErr(code)
	}
	enc := &RaptorQEncoder{K: K, L: L, h: h}
	runtime.SetFinalizer(enc, func(x *RaptorQEncoder) { C.rq_encoder_free(x.h) })
	return enc, nil
}

// GenSymbol: id < K is the zero-padded source symbol, otherwise the repair symbol of ISI id+K'-K.
func (e *RaptorQEncoder) GenSymbol(id uint32) []byte {
	sym := make([]byte, int(C.rq_encoder_symbol_size(e.h)))
	if C.rq_encoder_symbol(e.h, C.uint32_t(id), u8ptr(sym)) != 0 {
		return nil
	}
	runtime.KeepAlive(e)
	return sym
}

func (e *RaptorQEncoder) BaseSymbolsNum() uint32 {
	k := uint32(C.rq_encoder_k(e.h))
	runtime.KeepAlive(e)
	return k
}

func NewRaptorQDecoder(dataSize int, L int) (*RaptorQDecoder, error) {
	if dataSize < 0 || L <= 0 {
		return nil, errBadSizeL
	}
	var code C.int
	h := C.rq_decoder_create(C.uint64_t(dataSize), C.uint32_t(L), &code)
	if h == nil {
		return nil, libErr(code)
	}
	dec := &RaptorQDecoder{K: int(C.rq_decoder_k(h)), L: L, h: h, size: dataSize}
	runtime.SetFinalizer(dec, func(x *RaptorQDecoder) { C.rq_decoder_free(x.h) })
	return dec, nil
}

// AddSymbol's bool is the library's "K <= unique symbols held" (RQ/decoder.go:47,57), also when the
// symbol was a duplicate; a wrong-size symbol is an error.
func (d *RaptorQDecoder) AddSymbol(id uint32, data []byte) (bool, error) {
	var canTry C.int
	code := C.rq_decoder_add(d.h, C.uint32_t(id), u8ptr(data), C.size_t(len(data)), &canTry)
	runtime.KeepAlive(data)
	runtime.KeepAlive(d)
	if code != 0 {
		return canTry != 0, libErr(code)
	}
	return canTry != 0, nil
}

// Decode: (true, payload, nil); (false, nil, nil) for a rank-deficient system; an error
// ("not enough symbols to decode") with fewer than K unique symbols.
func (d *RaptorQDecoder) Decode() (bool, []byte, error) {
	payload := make([]byte, d.size)
	var ok C.int
	code := C.rq_decoder_decode(d.h, u8ptr(payload), &ok)
	runtime.KeepAlive(d)
	if code != 0 {
		return false, nil, libErr(code)
	}
	if ok == 0 {
		return false, nil, nil
	}
	return true, payload, nil
}

// RaptorQTracker is RaptorQDecoder's AddSymbol bookkeeping without the symbol bytes (rq_tracker_*): a
// receiver that stages each symbol once in its own pinned buffer (go/fecquic/rq_stage.go) keeps the
// decoder's readiness rule -- AddSymbol's bool, K <= unique symbols held (RQ/decoder.go:47,57; the
// receiver counts the true returns, rxbuf.go:472) -- and decodes the staged blocks with DecodeBlocks.
// No reference counterpart: the library's decoder always copies (RQ/decoder.go:39-57).
type RaptorQTracker struct {
	K int
	L int
	h *C.rq_tracker
}

func NewRaptorQTracker(dataSize int, L int) (*RaptorQTracker, error) {
	if dataSize < 0 || L <= 0 {
		return nil, errBadSizeL
	}
	var code C.int
	h := C.rq_tracker_create(C.uint64_t(dataSize), C.uint32_t(L), &code)
	if h == nil {
		return nil, libErr(code)
	}
	t := &RaptorQTracker{K: int(C.rq_tracker_k(h)), L: L, h: h}
	runtime.SetFinalizer(t, func(x *RaptorQTracker) { C.rq_tracker_free(x.h) })
	return t, nil
}

// AddSymbol has RaptorQDecoder.AddSymbol's signature, checks and bool; only len(data) is read.
func (t *RaptorQTracker) AddSymbol(id uint32, data []byte) (bool, error) {
	var canTry C.int
	code := C.rq_tracker_add(t.h, C.uint32_t(id), C.size_t(len(data)), &canTry)
	runtime.KeepAlive(t)
	if code != 0 {
		return canTry != 0, libErr(code)
	}
	return canTry != 0, nil
}

// RaptorQEncodeBlock returns symbols 0..N-1 of one block of at most K*L bytes (longer data is cut
// to K*L).  The repairs come from one batched call instead of N-K GenSymbol calls.
func RaptorQEncodeBlock(data []byte, N, K, L int) ([]Packet, error) {
	if N <= 0 || K <= 0 || L <= 0 || K > N {
		return nil, errBadNKL
	}
	if len(data) > K*L {
		data = data[:K*L]
	}
	enc, err := NewRaptorQEncoder(data, K, L)
	if err != nil {
		return nil, err
	}
	all := make([]byte, N*L)
	if code := C.rq_encoder_symbols(enc.h, 0, C.uint32_t(N), u8ptr(all)); code != 0 {
		return nil, libErr(code)
	}
	runtime.KeepAlive(enc)
	pkts := make([]Packet, N)
	for i := range pkts {
		pkts[i] = Packet{Index: i, Data: all[i*L : (i+1)*L : (i+1)*L]}
	}
	return pkts, nil
}

// RaptorQDecodeBytes feeds every packet whose Index is in [0, N) to a fresh decoder (a symbol the
// decoder refuses is skipped) and returns the payload, or (nil, false) when decoding fails.
func RaptorQDecodeBytes(recv []Packet, N, K, L, dataSize int) ([]byte, bool) {
	if K <= 0 || L <= 0 || dataSize < 0 {
		return nil, false
	}
	dec, err := NewRaptorQDecoder(dataSize, L)
	if err != nil {
		return nil, false
	}
	for i := range recv {
		if recv[i].Index >= 0 && recv[i].Index < N {
			_, _ = dec.AddSymbol(uint32(recv[i].Index), recv[i].Data)
		}
	}
	ok, payload, err := dec.Decode()
	if err != nil || !ok {
		return nil, false
	}
	return payload, true
}

// ---- batch path for go/fecquic (SURVEY.md sec. 8f): one call per window of blocks ----

// EncodeWindow returns the repair symbols K..N-1 of every block of a window (blocks[b] holds at most
// K*L bytes; short blocks are zero padded as splitToSymbols does).  deviceMask 0 = the default GPU,
// 0xff = all eight GPUs of a node (blocks split contiguously, no device-to-device traffic).
func EncodeWindow(blocks [][]byte, N, K, L int, deviceMask uint32) ([][]byte, error) {
	if N <= K || K <= 0 || L <= 0 {
		return nil, errBadNKL
	}
	nb := len(blocks)
	if nb == 0 {
		return nil, nil
	}
	srcBytes, repBytes := K*L, (N-K)*L
	src := C.malloc(C.size_t(nb * srcBytes)) // C memory: the library keeps no Go pointer
	defer C.free(src)
	dst := C.malloc(C.size_t(nb * repBytes))
	defer C.free(dst)
	in := unsafe.Slice((*byte)(src), nb*srcBytes)
	for b, blk := range blocks {
		n := copy(in[b*srcBytes:(b+1)*srcBytes], blk)
		clear(in[b*srcBytes+n : (b+1)*srcBytes])
	}
	esi := (*C.uint32_t)(C.malloc(C.size_t(N-K) * 4))
	defer C.free(unsafe.Pointer(esi))
	esis := unsafe.Slice(esi, N-K)
	for i := range esis {
		esis[i] = C.uint32_t(K + i)
	}
	desc := C.rq_encode_desc{T: C.uint32_t(L), K: C.uint32_t(K), n_blocks: C.uint32_t(nb),
		src: src, src_stride: C.uint64_t(srcBytes), n_esi: C.uint32_t(N - K), esi: esi,
		out: dst, out_stride: C.uint64_t(repBytes)}
	if code := C.rq_encode_batch_host(&desc, C.uint32_t(deviceMask)); code != 0 {
		return nil, libErr(code)
	}
	out := unsafe.Slice((*byte)(dst), nb*repBytes)
	reps := make([][]byte, nb)
	for b := range reps {
		reps[b] = append([]byte(nil), out[b*repBytes:(b+1)*repBytes]...)
	}
	return reps, nil
}

// DecodeBlocks decodes several received blocks in one call (the receiver workers of
// go/fecquic/rxbuf.go:336-377).  data[b] is K*L bytes of the block's staging (ideally from
// HostAlloc) with its received source rows in place, repair[b] its received repair rows in
// repairESI[b] order, erased[b] its missing source ESIs.  Status per block: 1 decoded (data[b] is
// complete), 0 rank-deficient (the reference's (false, nil, nil)), RQ_ERR_NOT_ENOUGH (-3).
func DecodeBlocks(K, L int, data [][]byte, repair [][]byte, erased, repairESI [][]uint32,
	deviceMask uint32) ([]int32, error) {
	n := len(data)
	if n == 0 {
		return nil, nil
	}
	if K <= 0 || L <= 0 {
		return nil, errBadKL
	}
	// the library reads K*L bytes of data[b] and len(repairESI[b])*L of repair[b] and writes the
	// recovered rows into data[b]: check every length before a pointer is taken
	if len(repair) != n || len(erased) != n || len(repairESI) != n {
		return nil, errBadBatch
	}
	for b := 0; b < n; b++ {
		if len(data[b]) < K*L || len(repair[b]) < len(repairESI[b])*L {
			return nil, errShortBuf
		}
	}
	ioBytes := C.size_t(n) * C.size_t(unsafe.Sizeof(C.rq_block_io{}))
	ioMem := C.malloc(ioBytes)
	defer C.free(ioMem)
	io := unsafe.Slice((*C.rq_block_io)(ioMem), n)
	// the library reads these slices during the call only; Pin keeps Go memory in place and is a no-op
	// on memory that is not Go's (HostAlloc's pinned C memory: runtime.Pinner ignores non-heap pointers)
	var pin runtime.Pinner
	defer pin.Unpin()
	for b := 0; b < n; b++ {
		io[b] = C.rq_block_io{n_erased: C.uint32_t(len(erased[b])), n_repair: C.uint32_t(len(repairESI[b]))}
		pin.Pin(&data[b][0])
		io[b].data = (*C.uint8_t)(unsafe.Pointer(&data[b][0]))
		if len(erased[b]) > 0 {
			pin.Pin(&erased[b][0])
			io[b].erased = (*C.uint32_t)(unsafe.Pointer(&erased[b][0]))
		}
		if len(repairESI[b]) > 0 {
			pin.Pin(&repairESI[b][0])
			pin.Pin(&repair[b][0])
			io[b].repair_esi = (*C.uint32_t)(unsafe.Pointer(&repairESI[b][0]))
			io[b].repair = (*C.uint8_t)(unsafe.Pointer(&repair[b][0]))
		}
	}
	if code := C.rq_decode_blocks_host(C.uint32_t(K), C.uint32_t(L), &io[0], C.uint32_t(n),
		C.uint32_t(deviceMask)); code != 0 {
		return nil, libErr(code)
	}
	status := make([]int32, n)
	for b := range status {
		status[b] = int32(io[b].status)
	}
	return status, nil
}

// HostAlloc / HostFree: pinned staging for a receiver's blocks (full-rate PCIe copies).
func HostAlloc(n int) []byte {
	p := C.rq_host_alloc(C.size_t(n))
	if p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(p), n)
}

func HostFree(b []byte) {
	if len(b) > 0 {
		C.rq_host_free(unsafe.Pointer(&b[0]))
	}
}
