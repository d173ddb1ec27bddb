// Sender side of the batch path (SURVEY.md sec. 8f row 1): one GPU call per window of blocks.
//
// The reference sender reads one K*L block, calls fec.RaptorQEncodeBlock on it and emits its N packets
// (go/fecquic/transfer.go:166-181).  windowReader keeps that loop and its per-block packets, but reads
// up to windowBlocks full blocks ahead and encodes them with one fec.EncodeWindow call
// (rq_encode_batch_host: H2D, the column program, D2H on the GPU, pipelined over chunks), then hands
// the blocks out one next() call at a time, in file order.  transfer.go.patch swaps the two calls.
//
// A short last block keeps the per-object path: its library K is ceil(n/L) (the receiver builds its
// decoder from the block's data size, rxbuf.go:437), and a padded block would be encoded under the
// window's K instead.
//
// Latency: the reference emits a block's packets as soon as that block is encoded.  A window delays the
// first packet by one window's read + encode, and holds the window's source and repairs in memory, so
// the windows grow: firstWindowBlocks (4 blocks, ~5 MB at K=1024 L=1200) first, then doubling up to
// windowBlocks (256 blocks, ~315 MB, enough for the library's H2D / kernel / D2H pipeline to run at the
// PCIe rate, DESIGN.md sec. 5.6).  A file of a few blocks is sent after a few blocks' encode, not the
// whole file's; encTime in transfer.go then measures each window's encode on the block that triggered it.
package fecquic

import (
	"io"

	"github.com/quic-go/quic-go/fec"
)

// blocks per EncodeWindow call: the first window is small (time to first packet), later ones double
// up to windowBlocks (256 blocks of K=1024, L=1200 are 315 MB of source, enough for the library's H2D /
// kernel / D2H pipeline to reach the PCIe rate, DESIGN.md sec. 5.6)
const (
	firstWindowBlocks = 4
	windowBlocks      = 256
)

type windowBlock struct {
	pkts []fec.Packet
	n    int // bytes of the block (K*L but for the last)
}

type windowReader struct {
	r          io.Reader
	N, K, L    int
	deviceMask uint32
	queue      []windowBlock
	done       bool
	window     int // blocks the next fill reads (firstWindowBlocks, doubling up to windowBlocks)
}

func newWindowReader(r io.Reader, N, K, L int, deviceMask uint32) *windowReader {
	return &windowReader{r: r, N: N, K: K, L: L, deviceMask: deviceMask, window: firstWindowBlocks}
}

// next returns the next block's N packets in ESI order (the K source symbols, the last zero padded as
// splitToSymbols pads it, then the N-K repairs) -- what fec.RaptorQEncodeBlock returns for the same
// bytes -- and the block's byte count; (nil, 0, io.EOF) after the last block.
func (w *windowReader) next() ([]fec.Packet, int, error) {
	if len(w.queue) == 0 {
		if w.done {
			return nil, 0, io.EOF
		}
		if err := w.fill(); err != nil {
			return nil, 0, err
		}
		if len(w.queue) == 0 {
			return nil, 0, io.EOF
		}
	}
	b := w.queue[0]
	w.queue = w.queue[1:]
	return b.pkts, b.n, nil
}

// fill reads up to w.window blocks and encodes the full ones in one call; the next window is twice as
// large, up to windowBlocks.
func (w *windowReader) fill() error {
	blockBytes := w.K * w.L
	want := w.window
	if w.window < windowBlocks {
		w.window *= 2
		if w.window > windowBlocks {
			w.window = windowBlocks
		}
	}
	full := make([][]byte, 0, want)
	var tail []byte
	for len(full) < want {
		buf := make([]byte, blockBytes)
		n, err := io.ReadFull(w.r, buf)
		if err == io.EOF || err == io.ErrUnexpectedEOF {
			w.done = true
			if n > 0 {
				tail = buf[:n]
			}
			break
		}
		if err != nil {
			return err
		}
		full = append(full, buf)
	}
	if len(full) > 0 {
		reps, err := fec.EncodeWindow(full, w.N, w.K, w.L, w.deviceMask)
		if err != nil {
			return err
		}
		for i, blk := range full {
			pkts := make([]fec.Packet, 0, w.N)
			for s := 0; s < w.K; s++ {
				pkts = append(pkts, fec.Packet{Index: s, Data: blk[s*w.L : (s+1)*w.L : (s+1)*w.L]})
			}
			for r := 0; r < w.N-w.K; r++ {
				pkts = append(pkts, fec.Packet{Index: w.K + r, Data: reps[i][r*w.L : (r+1)*w.L : (r+1)*w.L]})
			}
			w.queue = append(w.queue, windowBlock{pkts: pkts, n: blockBytes})
		}
	}
	if tail != nil {
		pkts, err := fec.RaptorQEncodeBlock(tail, w.N, w.K, w.L)
		if err != nil {
			return err
		}
		w.queue = append(w.queue, windowBlock{pkts: pkts, n: len(tail)})
	}
	return nil
}
