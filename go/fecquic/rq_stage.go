// Receiver ingest straight into per-block pinned staging (SURVEY.md sec. 8f row 3).
//
// The reference copies every received symbol into a pool slab (ingest, go/fecquic/rxbuf.go:497-538)
// and feeds it to a per-block decoder that keeps a copy of its own (AddSymbol, rxbuf.go:472;
// RQ/decoder.go:39-57); the round-5 batch worker then copied the slabs a third time into pinned memory
// for the GPU call.  Here ingest copies the datagram payload once, into the row its block's pinned
// staging reserves for it, and the classifier's AddSymbol is the bookkeeping-only fec.RaptorQTracker
// (the same bool, no bytes).  decodeGroup (rq_batchdec.go) hands the staged rows to fec.DecodeBlocks
// where they lie, and writes the recovered block to the file from the same memory.
//
// A block's staging is N rows of L bytes (fec.HostAlloc, reused across blocks): source ESI e < K at
// row e, repairs appended in arrival order from row K.  A symbol that is a duplicate, that belongs to a
// block the decode worker has frozen or finished, or that the ring refuses is dropped at ingest with the
// reference's counters (the classifier drops the same symbols in rxbuf.go:446-468); its row, if one was
// taken, is simply never used.
package fecquic

import (
	"sync"
	"time"

	"github.com/quic-go/quic-go/fec"
)

// blockStage is one block's staging.  mu orders ingest's row copies against the decode worker's freeze.
type blockStage struct {
	mu      sync.Mutex
	buf     []byte
	pinned  bool
	K, N, L int
	rowOf   []int32 // by ESI < N: the row holding that symbol, -1 if none
	nRep    int     // repairs appended: rows K .. K+nRep-1
	frozen  bool    // the decode worker is reading the rows: later symbols are dropped
}

// stageTable maps block ids to their staging; released pinned buffers are kept for the next blocks.
type stageTable struct {
	mu     sync.Mutex
	blocks map[uint16]*blockStage
	done   map[uint16]bool  // decoded blocks: their late symbols are dropped, not re-staged
	free   map[int][][]byte // released pinned buffers by size
}

func newStageTable() *stageTable {
	return &stageTable{blocks: make(map[uint16]*blockStage), done: make(map[uint16]bool), free: make(map[int][][]byte)}
}

// get returns the block's staging, created on the block's first symbol; nil once the block is decoded.
func (t *stageTable) get(id uint16, N, K, L int) *blockStage {
	t.mu.Lock()
	defer t.mu.Unlock()
	if t.done[id] {
		return nil
	}
	if st := t.blocks[id]; st != nil {
		return st
	}
	size := N * L
	st := &blockStage{K: K, N: N, L: L, rowOf: make([]int32, N)}
	for i := range st.rowOf {
		st.rowOf[i] = -1
	}
	if l := t.free[size]; len(l) > 0 {
		st.buf, st.pinned = l[len(l)-1], true
		t.free[size] = l[:len(l)-1]
	} else if p := fec.HostAlloc(size); p != nil {
		st.buf, st.pinned = p, true
	} else {
		st.buf = make([]byte, size) // pageable still works, at a lower PCIe rate
	}
	t.blocks[id] = st
	return st
}

// lookup returns the block's staging (nil if it has none).
func (t *stageTable) lookup(id uint16) *blockStage {
	t.mu.Lock()
	defer t.mu.Unlock()
	return t.blocks[id]
}

// release retires a decoded block: its buffer goes back to the free list.
func (t *stageTable) release(id uint16) {
	t.mu.Lock()
	defer t.mu.Unlock()
	t.done[id] = true
	st := t.blocks[id]
	if st == nil {
		return
	}
	delete(t.blocks, id)
	if st.pinned {
		t.free[len(st.buf)] = append(t.free[len(st.buf)], st.buf)
	}
}

// close frees every pinned buffer (closeAndFinalize, once the workers have stopped).
func (t *stageTable) close() {
	t.mu.Lock()
	defer t.mu.Unlock()
	for id, st := range t.blocks {
		if st.pinned {
			fec.HostFree(st.buf)
		}
		delete(t.blocks, id)
	}
	for size, l := range t.free {
		for _, b := range l {
			fec.HostFree(b)
		}
		delete(t.free, size)
	}
}

// stageIngest is ingest's body (rxbuf.go.patch): the reference's admission and counters, with the copy
// going into the block's staging instead of a pool slab.  The Symbol the classifier receives carries the
// staged row (Buf) and a slab describing it (for the classifier's accounting of len(s.Buf) and s.n).
func (m *rxManager) stageIngest(blockID uint16, esi int, N, K, L int, data []byte, dataSize int) bool {
	t0 := time.Now()
	isRepair := esi >= K
	dropped := func(afterQueue bool) bool {
		switch {
		case afterQueue && isRepair:
			m.dropAfterQRep.Add(1)
		case afterQueue:
			m.dropAfterQSys.Add(1)
			m.dropsSystem.Add(1)
		case isRepair:
			m.dropsRepairs.Add(1)
		default:
			m.dropsSystem.Add(1)
		}
		return false
	}
	// a staging row holds exactly one L-byte symbol of ESI < N (the sender's packets, transfer.go:186-198);
	// a symbol of another size is one the decoder's AddSymbol would refuse (RQ/decoder.go:39-57)
	if esi < 0 || esi >= N || K <= 0 || N < K || L <= 0 || len(data) != L {
		return dropped(false)
	}
	st := m.stage.get(blockID, N, K, L)
	if st == nil {
		return dropped(true) // decoded already
	}
	st.mu.Lock()
	if st.frozen {
		st.mu.Unlock()
		return dropped(true)
	}
	if st.K != K || st.N != N || st.L != L {
		st.mu.Unlock()
		return dropped(false)
	}
	if st.rowOf[esi] >= 0 {
		st.mu.Unlock()
		m.dupSymbols.Add(1)
		return false
	}
	row := esi
	if isRepair {
		row = K + st.nRep
		st.nRep++
	}
	p := st.buf[row*L : (row+1)*L]
	copy(p, data)
	st.rowOf[esi] = int32(row)
	st.mu.Unlock()
	s := Symbol{
		BlockID:  blockID,
		ESI:      esi,
		N:        N,
		K:        K,
		L:        L,
		DataSize: dataSize,
		IsRepair: isRepair,
		Arrival:  time.Now().UnixNano(),
		Buf:      p,
		slab:     &slab{b: p, n: len(p)},
	}
	if !m.ring.tryPush(s) {
		if isRepair {
			m.dropsRepairs.Add(1)
			m.ringDropRepairs.Add(1)
		} else {
			m.dropsSystem.Add(1)
			m.ringDropSystem.Add(1)
		}
		st.mu.Lock()
		st.rowOf[esi] = -1 // a retransmission may stage it again
		st.mu.Unlock()
		return false
	}
	d := time.Since(t0)
	m.ingressProcMs.Add(d.Milliseconds())
	m.ingressProcUs.Add(d.Microseconds())
	return true
}

// unstage forgets the staged row of a symbol the classifier did not accept (its block was queued or
// done, or it was over the receive budget: rxbuf.go:416-456), so a retransmission can be staged again.
func (m *rxManager) unstage(s Symbol) {
	st := m.stage.lookup(s.BlockID)
	if st == nil || s.ESI < 0 || s.ESI >= len(st.rowOf) {
		return
	}
	st.mu.Lock()
	st.rowOf[s.ESI] = -1
	st.mu.Unlock()
}
