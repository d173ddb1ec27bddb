// Receiver side of the batch path (SURVEY.md sec. 8f rows 1 and 3): the decode workers batch the
// blocks that are ready into one GPU call.
//
// The reference worker takes one ready block from decodeQ and calls its per-object decoder's Decode
// (go/fecquic/rxbuf.go:336-377).  batchDecodeWorker keeps everything around that call -- the classifier
// and its AddSymbol bookkeeping (haveU counts the true returns of the fec.RaptorQTracker; a block is
// ready at haveU >= K), the 50 ms DDL scheduler, the receive budget -- and replaces the call: it drains
// up to decodeBatchMax queued blocks and decodes them with one fec.DecodeBlocks call per (library K, L),
// on the rows ingest already staged in each block's pinned buffer (rq_stage.go): no host copy of a
// received symbol between the datagram and the GPU.  The recovered block is written to the file from the
// same buffer.  rxbuf.go.patch points the workers here.  A status other than 1 is the reference's failed
// Decode: the block waits for more symbols (queued = false).
package fecquic

import (
	"sort"
	"time"

	"github.com/quic-go/quic-go/fec"
)

// ready blocks per DecodeBlocks call (one worker drains the queue without waiting for more)
const decodeBatchMax = 256

// batchDecodeWorker runs in place of the reference worker loop until decodeQ closes.
func (m *rxManager) batchDecodeWorker() {
	for b := range m.decodeQ {
		batch := []*rxBlock{b}
	drain:
		for len(batch) < decodeBatchMax {
			select {
			case nb, ok := <-m.decodeQ:
				if !ok {
					break drain
				}
				batch = append(batch, nb)
			default:
				break drain
			}
		}
		m.decodeBatch(batch)
	}
}

// libraryK is the decoder's K for a block of dataSize bytes (NewRaptorQDecoder(dataSize, L)).
func libraryK(dataSize, L int) int { return (dataSize + L - 1) / L }

type groupKey struct{ kl, L int }

func (m *rxManager) decodeBatch(batch []*rxBlock) {
	groups := map[groupKey][]*rxBlock{} // one DecodeBlocks call shares K and L
	for _, b := range batch {
		if b.done {
			continue
		}
		if b.haveU < b.K {
			b.queued = false // not ready yet (the reference worker's first check)
			continue
		}
		k := groupKey{libraryK(b.dataSize, b.L), b.L}
		groups[k] = append(groups[k], b)
	}
	for k, blocks := range groups {
		m.decodeGroup(k.kl, k.L, blocks)
	}
}

type stagedBlock struct {
	b         *rxBlock
	st        *blockStage
	data      []byte   // library K x L bytes: the staging's first rows
	repair    []byte   // the received library repairs' rows, consecutive
	erased    []uint32 // source ESIs < library K not received
	repairESI []uint32
}

func (m *rxManager) decodeGroup(kl, L int, blocks []*rxBlock) {
	// the ESIs the classifier accepted (a queued block's set no longer changes: the classifier drops its
	// new symbols, rxbuf.go:446-458)
	accepted := make([][]int, len(blocks))
	m.mu.Lock()
	for i, b := range blocks {
		for esi := range b.syms {
			accepted[i] = append(accepted[i], esi)
		}
	}
	m.mu.Unlock()
	st := make([]stagedBlock, 0, len(blocks))
	for i, b := range blocks {
		bs := m.stage.lookup(b.id)
		if bs == nil {
			b.queued = false
			continue
		}
		bs.mu.Lock()
		bs.frozen = true // from here no ingest writes into bs.buf
		bs.mu.Unlock()
		sb := stagedBlock{b: b, st: bs, data: bs.buf[:kl*L]}
		have := make([]bool, kl)
		var reps []int // library repairs: ESI >= kl (rows esi below the wrapper K, K + i above it)
		for _, esi := range accepted[i] {
			if esi < kl {
				have[esi] = true
			} else {
				reps = append(reps, esi)
			}
		}
		sort.Slice(reps, func(x, y int) bool { return bs.rowOf[reps[x]] < bs.rowOf[reps[y]] })
		contiguous := true
		for j, esi := range reps {
			sb.repairESI = append(sb.repairESI, uint32(esi))
			contiguous = contiguous && int(bs.rowOf[esi]) == kl+j
		}
		if contiguous {
			sb.repair = bs.buf[kl*L : (kl+len(reps))*L] // the common case: the rows as ingest staged them
		} else {
			// a hole among the rows (a symbol the ring or the budget dropped, a short last block with a
			// missing symbol below the wrapper K): these rows alone are gathered
			sb.repair = make([]byte, len(reps)*L)
			for j, esi := range reps {
				r := int(bs.rowOf[esi])
				copy(sb.repair[j*L:(j+1)*L], bs.buf[r*L:(r+1)*L])
			}
		}
		for esi := 0; esi < kl; esi++ {
			if !have[esi] {
				sb.erased = append(sb.erased, uint32(esi))
			}
		}
		st = append(st, sb)
	}
	if len(st) == 0 {
		return
	}
	data := make([][]byte, len(st))
	repair := make([][]byte, len(st))
	erased := make([][]uint32, len(st))
	repairESI := make([][]uint32, len(st))
	for i := range st {
		data[i], repair[i], erased[i], repairESI[i] = st[i].data, st[i].repair, st[i].erased, st[i].repairESI
	}
	m.decodeAttempts.Add(int64(len(st)))
	t0 := time.Now()
	status, err := fec.DecodeBlocks(kl, L, data, repair, erased, repairESI, 0)
	m.decTimeTotal.Add(time.Since(t0).Milliseconds())
	for i := range st {
		b, bs := st[i].b, st[i].st
		if err != nil || status[i] != 1 {
			// the reference's failed Decode: likely needs more symbols
			m.decodeFailures.Add(1)
			bs.mu.Lock()
			bs.frozen = false
			bs.mu.Unlock()
			b.queued = false
			continue
		}
		// the block is whole in its staging: one write from there (the writer goroutine's bounds and
		// counters, rxbuf.go:320-334), then the staging goes back to the free list
		off := int64(int(b.id) * b.K * b.L)
		out := bs.buf[:b.dataSize]
		if rem := int64(m.fileSize) - off; rem < int64(len(out)) {
			if rem < 0 {
				rem = 0
			}
			out = out[:rem]
		}
		tw := time.Now()
		_, _ = m.out.WriteAt(out, off)
		dw := time.Since(tw)
		m.writeTimeMs.Add(dw.Milliseconds())
		m.writeTimeUs.Add(dw.Microseconds())
		m.written.Add(uint64(len(out)))
		m.decBlocks.Add(1)
		m.mu.Lock()
		for _, s := range b.syms {
			m.inUse.Add(int64(-s.n))
		}
		b.syms = nil
		b.done = true
		delete(m.blocks, b.id)
		m.mu.Unlock()
		m.stage.release(b.id)
	}
}
