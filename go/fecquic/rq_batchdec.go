// Receiver side of the batch path (SURVEY.md sec. 8f rows 1 and 3): the decode workers batch the
// blocks that are ready into one GPU call.
//
// The reference worker takes one ready block from decodeQ and calls its per-object decoder's Decode
// (go/fecquic/rxbuf.go:336-377).  batchDecodeWorker keeps everything around that call -- the classifier
// and its AddSymbol bookkeeping (haveU counts the true returns; a block is ready at haveU >= K), the
// 50 ms DDL scheduler, the receive budget, the single writer -- and replaces the call: it drains up to
// decodeBatchMax queued blocks, stages each block's received symbols in pinned memory (fec.HostAlloc:
// source rows in place, repairs in ESI order) and decodes them with one fec.DecodeBlocks call per
// library K.  rxbuf.go.patch points the workers here.  A status other than 1 is the reference's failed
// Decode: the block waits for more symbols (queued = false).
package fecquic

import (
	"sort"
	"time"

	"github.com/quic-go/quic-go/fec"
)

// ready blocks per DecodeBlocks call (one worker drains the queue without waiting for more)
const decodeBatchMax = 256

type stagedBlock struct {
	b         *rxBlock
	data      []byte   // library K x L bytes of the pinned staging
	repair    []byte   // the received repair rows, repairESI order
	erased    []uint32 // source ESIs < library K not received
	repairESI []uint32
}

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

func (m *rxManager) decodeBatch(batch []*rxBlock) {
	groups := map[int][]*rxBlock{} // by library K: one DecodeBlocks call shares K
	for _, b := range batch {
		if b.done {
			continue
		}
		if b.haveU < b.K {
			b.queued = false // not ready yet (the reference worker's first check)
			continue
		}
		kl := libraryK(b.dataSize, b.L)
		groups[kl] = append(groups[kl], b)
	}
	for kl, blocks := range groups {
		m.decodeGroup(kl, blocks)
	}
}

func (m *rxManager) decodeGroup(kl int, blocks []*rxBlock) {
	L := blocks[0].L
	stage := fec.HostAlloc(len(blocks) * kl * L)
	if stage == nil {
		stage = make([]byte, len(blocks)*kl*L) // pageable still works, at a lower PCIe rate
	} else {
		defer fec.HostFree(stage)
	}
	st := make([]stagedBlock, len(blocks))
	m.mu.Lock() // a queued block's symbols no longer change (the classifier drops new ones), but
	// the slabs are shared with the pool: copy under the lock
	for i, b := range blocks {
		sb := &st[i]
		sb.b = b
		sb.data = stage[i*kl*L : (i+1)*kl*L]
		esis := make([]int, 0, len(b.syms))
		for esi := range b.syms {
			esis = append(esis, esi)
		}
		sort.Ints(esis)
		have := make([]bool, kl)
		for _, esi := range esis {
			s := b.syms[esi]
			if esi < kl {
				n := copy(sb.data[esi*L:(esi+1)*L], s.b[:s.n])
				clear(sb.data[esi*L+n : (esi+1)*L])
				have[esi] = true
			} else {
				sb.repairESI = append(sb.repairESI, uint32(esi))
				row := make([]byte, L)
				copy(row, s.b[:s.n])
				sb.repair = append(sb.repair, row...)
			}
		}
		for esi := 0; esi < kl; esi++ {
			if !have[esi] {
				sb.erased = append(sb.erased, uint32(esi))
			}
		}
	}
	m.mu.Unlock()

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
		b := st[i].b
		if err != nil || status[i] != 1 {
			// the reference's failed Decode: likely needs more symbols
			m.decodeFailures.Add(1)
			b.queued = false
			continue
		}
		// one contiguous write per block, out of the pinned staging (freed when this call returns)
		out := make([]byte, b.dataSize)
		copy(out, st[i].data)
		m.writeQ <- writeTask{off: int64(int(b.id) * b.K * b.L), data: out}
		m.decBlocks.Add(1)
		m.mu.Lock()
		for _, s := range b.syms {
			m.inUse.Add(int64(-s.n))
			s.n = 0
			m.slabs.Put(s)
		}
		b.syms = nil
		b.done = true
		delete(m.blocks, b.id)
		m.mu.Unlock()
	}
}
