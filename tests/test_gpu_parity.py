"""GPU parity: the HIP path (through the C-ABI) against the oracle, bit for bit.

Covers the per-object API (NewRaptorQEncoder/GenSymbol, NewRaptorQDecoder/AddSymbol/Decode as
go/fec/raptorq_wrap.go exposes them), the batched device-resident API on the BASELINE.json
configs, short final blocks, T not a multiple of 4, rank-deficient decodes (ok=false parity),
and size-independent properties at full size (encode -> erase -> decode round trips)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rand_bytes(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("K,T", [(5, 1100), (26, 1500), (64, 1200), (64, 1201), (1, 16), (128, 256)])
def test_encoder_symbols_match_oracle(gpu, rq, oracle, K, T):
    rng = np.random.default_rng(K * 7 + T)
    data = rand_bytes(rng, K * T - (T // 3))
    enc = rq.NewRaptorQEncoder(data, K, T)
    ref = oracle.OracleEncoder(data, T)
    assert enc.BaseSymbolsNum() == ref.p["K"]
    N = ref.p["K"] + max(8, ref.p["K"] // 4)
    got = enc.GenSymbols(0, N)
    for i in range(N):
        assert got[i] == ref.gen_symbol(i).tobytes(), i
    for i in (0, ref.p["K"], N + 1000, 70000):  # single GenSymbol, far ESIs
        assert enc.GenSymbol(i) == ref.gen_symbol(i).tobytes()


def test_encode_block_packets(gpu, rq, oracle):
    rng = np.random.default_rng(11)
    data = rand_bytes(rng, 26 * 1500 + 100)  # clamped to K*L by RaptorQEncodeBlock
    pk = rq.RaptorQEncodeBlock(data, 32, 26, 1500)
    ref = oracle.OracleEncoder(data[:26 * 1500], 1500)
    assert [p.Index for p in pk] == list(range(32))
    for p in pk:
        assert p.Data == ref.gen_symbol(p.Index).tobytes()


@pytest.mark.parametrize("K,T,N,loss,seed", [(64, 1200, 80, 0.10, 1), (26, 1500, 32, 0.15, 2),
                                              (256, 64, 282, 0.05, 3), (5, 1100, 8, 0.3, 4)])
def test_decoder_matches_oracle(gpu, rq, oracle, K, T, N, loss, seed):
    rng = np.random.default_rng(seed)
    for trial in range(6):
        data = rand_bytes(rng, K * T - int(rng.integers(0, T)))
        ref_enc = oracle.OracleEncoder(data, T)
        syms = [ref_enc.gen_symbol(i).tobytes() for i in range(N)]
        keep = [i for i in range(N) if rng.random() >= loss]
        dec = rq.NewRaptorQDecoder(len(data), T)
        rdec = oracle.OracleDecoder(len(data), T)
        for i in keep:
            assert dec.AddSymbol(i, syms[i]) == rdec.add_symbol(i, syms[i])
        try:
            ref = rdec.decode()
        except RuntimeError:
            with pytest.raises(rq.RaptorQError, match="not enough symbols"):
                dec.Decode()
            continue
        got = dec.Decode()
        assert got[0] == ref[0]
        if ref[0]:
            assert got[1] == ref[1] == data


def find_rank_deficient(oracle, K, T, tries, seed):
    """Received = K patterns that the oracle reports unsolvable (SURVEY.md sec. 7 census:
    ~0.7% at received = K)."""
    rng = np.random.default_rng(seed)
    found = []
    data = rand_bytes(rng, K * T)
    enc = oracle.OracleEncoder(data, T)
    N = K + K // 2
    syms = [enc.gen_symbol(i).tobytes() for i in range(N)]
    for _ in range(tries):
        ids = sorted(rng.choice(N, K, replace=False).tolist())
        d = oracle.OracleDecoder(len(data), T)
        for i in ids:
            d.add_symbol(i, syms[i])
        ok, _ = d.decode()
        if not ok:
            found.append(ids)
            if len(found) >= 3:
                break
    return data, syms, found


def test_rank_deficient_parity(gpu, rq, oracle):
    K, T = 64, 16
    data, syms, found = find_rank_deficient(oracle, K, T, 3000, 7)
    assert found, "no rank-deficient pattern found"
    for ids in found:
        dec = rq.NewRaptorQDecoder(len(data), T)
        for i in ids:
            dec.AddSymbol(i, syms[i])
        assert dec.Decode() == (False, None)
        # one more symbol makes it solvable in practice (received = K+1 census: 0 failures)
        extra = max(ids) + 1 if max(ids) + 1 < len(syms) else [i for i in range(len(syms)) if i not in ids][0]
        dec.AddSymbol(extra, syms[extra])
        d2 = oracle.OracleDecoder(len(data), T)
        for i in ids + [extra]:
            d2.add_symbol(i, syms[i])
        assert dec.Decode() == d2.decode()


def _batch_encode(rq, gpu, K, T, n_blocks, esis, seed):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, 256, (n_blocks, K * T), dtype=torch.uint8, generator=g).to(gpu)
    out = torch.empty((n_blocks, len(esis) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    return src, out


# (1024, 64, 1, 552): a launch of one 16-column item (its cross-item prefetch has no next item and
# re-reads its own rows); (1024, 1200, 1023, 76): ~4 800 items over the persistent grid, the last one
# partial (20 columns) and some wave's fifth: the previous item's tail prefetches it under its lane mask
@pytest.mark.parametrize("K,T,n_blocks,R", [(256, 1200, 8, 26), (1024, 1200, 2, 76), (64, 1200, 16, 16),
                                             (2048, 256, 1, 40), (128, 256, 4, 20), (512, 1200, 2, 33),
                                             (1024, 64, 1, 552), (1024, 1200, 1023, 76)])
def test_batch_encode_matches_oracle(gpu, rq, oracle, K, T, n_blocks, R):
    esis = list(range(K, K + R))
    src, out = _batch_encode(rq, gpu, K, T, n_blocks, esis, K + R)
    src_h, out_h = src.cpu().numpy(), out.cpu().numpy()
    for b in sorted({0, 1, n_blocks - 1} & set(range(n_blocks))):
        ref = oracle.OracleEncoder(src_h[b].tobytes(), T)
        for r, e in enumerate(esis):
            assert np.array_equal(out_h[b, r * T:(r + 1) * T], ref.gen_symbol(e)), (b, e)


def _erase_and_decode(rq, gpu, src, out, K, T, N, n_erase, rng):
    """Erase exactly n_erase of the N symbols per block, decode in one batch."""
    n_blocks = src.shape[0]
    R = N - K
    erased_lists, rep_lists, rep_rows = [], [], []
    for b in range(n_blocks):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        erased_lists.append(sorted(i for i in lost if i < K))
        rl = [K + r for r in range(R) if (K + r) not in lost]
        rep_lists.append(rl)
        rep_rows.extend((b, r - K) for r in rl)
    data = src.clone()
    for b, el in enumerate(erased_lists):
        for i in el:
            data[b, i * T:(i + 1) * T] = 0xA5  # garbage in erased rows
    rep = torch.empty((max(len(rep_rows), 1), T), dtype=torch.uint8, device=gpu)
    if rep_rows:
        idx_b = torch.tensor([b for b, _ in rep_rows], device=gpu)
        idx_r = torch.tensor([r for _, r in rep_rows], device=gpu)
        rep[:len(rep_rows)] = out.view(n_blocks, R, T)[idx_b, idx_r]
    db = rq.DecodeBatch(K, T, erased_lists, rep_lists)
    st = db.run(data, rep)
    torch.cuda.synchronize()
    return data, st, erased_lists, rep_lists


# BASELINE.json configs 2-4 and the mixed stream of config 5 (K in {128, 512, 2048} x T in {256, 1200},
# N = K + K/10 + 8, 5 % of N erased)
@pytest.mark.parametrize("K,T,N,n_blocks,n_erase", [(1024, 1200, 1100, 4, 55), (256, 1200, 282, 8, 14),
                                                     (64, 1200, 80, 16, 8), (2048, 256, 2200, 2, 110),
                                                     (128, 256, 148, 8, 7), (128, 1200, 148, 8, 7),
                                                     (512, 256, 571, 4, 29), (512, 1200, 571, 4, 29),
                                                     (2048, 1200, 2260, 2, 113)])
def test_batch_decode_round_trip(gpu, rq, oracle, K, T, N, n_blocks, n_erase):
    rng = np.random.default_rng(K + n_erase)
    esis = list(range(K, N))
    src, out = _batch_encode(rq, gpu, K, T, n_blocks, esis, 99)
    data, st, el, rl = _erase_and_decode(rq, gpu, src, out, K, T, N, n_erase, rng)
    # property at full size: every solvable block is recovered bit-exactly
    for b in range(n_blocks):
        assert st[b] in (0, 1)
        if st[b] == 1:
            assert torch.equal(data[b], src[b]), b
    assert (st == 1).mean() > 0.5
    # ok/fail parity and bytes against the oracle: every block (the first two at K >= 1024, where
    # the oracle's dense elimination takes seconds per block)
    for b in range(n_blocks if K < 1024 else min(n_blocks, 2)):
        src_h = src[b].cpu().numpy().tobytes()
        ref_enc = oracle.OracleEncoder(src_h, T)
        rdec = oracle.OracleDecoder(len(src_h), T)
        for i in range(K):
            if i not in el[b]:
                rdec.add_symbol(i, ref_enc.gen_symbol(i).tobytes())
        for e in rl[b]:
            rdec.add_symbol(e, ref_enc.gen_symbol(e).tobytes())
        ok, ref_out = rdec.decode()
        assert ok == (st[b] == 1), b
        if ok:
            assert data[b].cpu().numpy().tobytes() == ref_out, b


def test_batch_decode_not_enough_and_fast_path(gpu, rq):
    K, T, N = 64, 64, 70
    esis = list(range(K, N))
    src, out = _batch_encode(rq, gpu, K, T, 3, esis, 5)
    erased = [[], [1, 2, 3], list(range(10))]
    reps = [[], [K, K + 1, K + 2], list(range(K, N))]  # block 2: 54 + 6 < 64
    rep = out.view(3, N - K, T)[1, :3].contiguous()
    rep_all = torch.cat([rep, out.view(3, N - K, T)[2]], 0).contiguous()
    data = src.clone()
    db = rq.DecodeBatch(K, T, erased, reps)
    st = db.run(data, rep_all)
    torch.cuda.synchronize()
    assert st[0] == 1 and st[2] == rq.RQ_ERR_NOT_ENOUGH
    assert st[1] in (0, 1)
    assert torch.equal(data[0], src[0])


def test_concurrent_streams_independent(gpu, rq):
    """Batches on two HIP streams run concurrently with per-stream workspaces: results equal the
    single-stream results bit for bit (the fecquic batch path pipelines chunks this way)."""
    K, T, R, nb = 256, 1200, 26, 64
    esis = list(range(K, K + R))
    g = torch.Generator().manual_seed(12)
    src = torch.randint(0, 256, (2, nb, K * T), dtype=torch.uint8, generator=g).to(gpu)
    ref = torch.empty((2, nb, R * T), dtype=torch.uint8, device=gpu)
    for i in range(2):
        rq.encode_batch(src[i], K, T, esis, ref[i])
    torch.cuda.synchronize()
    out = torch.zeros_like(ref)
    streams = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    for rep in range(3):
        for i, s in enumerate(streams):
            rq.encode_batch(src[i], K, T, esis, out[i], stream=s)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_decode_async_back_to_back(gpu, rq):
    """rq_decode_batch_async: three batches queued back to back on one stream without a host sync
    (double-buffered descriptors, copy-stream upload) give the synchronous call's statuses and bytes."""
    K, T, N, nb = 256, 1200, 282, 16
    esis = list(range(K, N))
    rng = np.random.default_rng(77)
    src, out = _batch_encode(rq, gpu, K, T, nb, esis, 3)
    runs = []
    for it in range(3):
        er, rl, rows = [], [], []
        for b in range(nb):
            lost = set(rng.choice(N, 14 + it, replace=False).tolist())
            er.append(sorted(i for i in lost if i < K))
            rl.append([e for e in esis if e not in lost])
            rows.extend((b, e - K) for e in rl[-1])
        rep = out.view(nb, N - K, T)[torch.tensor([b for b, _ in rows], device=gpu),
                                     torch.tensor([r for _, r in rows], device=gpu)].contiguous()
        data = src.clone()
        for b in range(nb):
            for i in er[b]:
                data[b, i * T:(i + 1) * T] = 0x5A
        runs.append((rq.DecodeBatch(K, T, er, rl), data, rep))
    stream = torch.cuda.current_stream(gpu)
    sts = [db.run_async(data, rep, stream=stream) for db, data, rep in runs]
    torch.cuda.synchronize()
    for (db, data, rep), st in zip(runs, sts):
        assert (st == 1).all(), st
        assert torch.equal(data, src)
    # the same batch synchronously: identical statuses
    db, data, rep = runs[0]
    assert np.array_equal(db.run(data, rep), sts[0])
    # the async call refuses pageable status memory
    d = db._desc(data, rep, np.zeros(nb, np.int32), None)
    assert rq.lib().rq_decode_batch_async(d) == rq.RQ_ERR_BAD_ARG


class _StagedBlock:
    """Python mirror of go/fecquic/rq_stage.go + rq_batchdec.go for one block: ingest copies each symbol
    once into the block's pinned staging (source ESI e at row e, repairs appended from row K), the
    bookkeeping is the rq_tracker (AddSymbol's bool without the bytes), and the decode hands the staged
    rows to rq_decode_blocks_host where they lie (a gather only when a row is missing below the repairs)."""

    def __init__(self, rq, size, N, K, T):
        import ctypes
        self.rq, self.N, self.K, self.T, self.size = rq, N, K, T, size
        self.ptr = rq.lib().rq_host_alloc(N * T)
        assert self.ptr
        self.buf = np.ctypeslib.as_array((ctypes.c_uint8 * (N * T)).from_address(self.ptr))
        self.buf[:] = 0xA5  # stale bytes of a reused buffer
        self.row_of = {}
        self.n_rep = 0
        self.tracker = rq.NewRaptorQTracker(size, T)
        self.haveU = 0

    def ingest(self, esi, sym):
        if esi in self.row_of:
            return None  # a duplicate: dropped at ingest
        row = esi if esi < self.K else self.K + self.n_rep
        self.n_rep += esi >= self.K
        self.buf[row * self.T:(row + 1) * self.T] = np.frombuffer(sym, np.uint8)
        self.row_of[esi] = row
        inc = self.tracker.AddSymbol(esi, sym)
        self.haveU += inc
        return inc

    def decode_args(self):
        kl = self.tracker.K
        reps = sorted((e for e in self.row_of if e >= kl), key=lambda e: self.row_of[e])
        data = self.buf[:kl * self.T]
        if all(self.row_of[e] == kl + j for j, e in enumerate(reps)):
            rows = self.buf[kl * self.T:(kl + len(reps)) * self.T].reshape(-1, self.T)
            gathered = False
        else:
            rows = np.stack([self.buf[self.row_of[e] * self.T:(self.row_of[e] + 1) * self.T] for e in reps]) \
                if reps else np.zeros((0, self.T), np.uint8)
            gathered = True
        erased = [e for e in range(kl) if e not in self.row_of]
        return data, erased, reps, rows, gathered

    def free(self):
        self.rq.lib().rq_host_free(self.ptr)


@pytest.mark.parametrize("K,T,N,loss,seed,short", [(64, 1200, 80, 0.10, 1, False), (26, 1500, 32, 0.15, 2, False),
                                                   (256, 64, 282, 0.05, 3, False), (5, 1100, 8, 0.3, 4, False),
                                                   (64, 1200, 80, 0.10, 6, True)])
def test_staged_receiver_matches_oracle(gpu, rq, oracle, K, T, N, loss, seed, short):
    """The Go receiver's staged path on the shapes of test_decoder_matches_oracle: the
    tracker's bools equal the oracle decoder's, symbol by symbol, in arrival order with duplicates; the
    staged rows decode through rq_decode_blocks_host (all ready blocks of a trial in one call) to the
    oracle's (ok, bytes).  short: last blocks of a file (library K < the wrapper K, so ESIs between them
    are repairs staged at source rows)."""
    rng = np.random.default_rng(seed)
    ready, gathered = [], 0
    for trial in range(6):
        size = (K * T - int(rng.integers(0, T))) if not short else (int(rng.integers(K // 3, K - 3)) * T - 11)
        data = rand_bytes(rng, size)
        ref_enc = oracle.OracleEncoder(data, T)
        syms = [ref_enc.gen_symbol(i).tobytes() for i in range(N)]
        keep = [i for i in range(N) if rng.random() >= loss]
        arrival = list(rng.permutation(keep)) + [int(x) for x in rng.choice(keep, 3)]
        sb = _StagedBlock(rq, size, N, K, T)
        rdec = oracle.OracleDecoder(size, T)
        for e in arrival:
            e = int(e)
            want = rdec.add_symbol(e, syms[e])
            got = sb.ingest(e, syms[e])
            assert got is None or got == want, (trial, e)
        try:
            ref = rdec.decode()
        except RuntimeError:
            assert sb.haveU == 0 or sb.tracker.Held() < sb.tracker.K
            sb.free()
            continue
        ready.append((sb, ref, data))
    try:
        assert ready
        args = [sb.decode_args() for sb, _, _ in ready]
        gathered = sum(a[4] for a in args)
        kl = ready[0][0].tracker.K
        same_k = [i for i, (sb, _, _) in enumerate(ready) if sb.tracker.K == kl]
        st = rq.decode_blocks_host(kl, T, [args[i][:4] for i in same_k])
        for j, i in enumerate(same_k):
            sb, ref, data = ready[i]
            assert (st[j] == 1) == ref[0], (i, st[j])
            if ref[0]:
                assert bytes(sb.buf[:sb.size]) == ref[1] == data
        for i in set(range(len(ready))) - set(same_k):  # other library K (short blocks): one call each
            sb, ref, data = ready[i]
            st = rq.decode_blocks_host(sb.tracker.K, T, [args[i][:4]])
            assert (st[0] == 1) == ref[0]
            if ref[0]:
                assert bytes(sb.buf[:sb.size]) == ref[1] == data
        if not short:
            assert gathered == 0  # full blocks: every decode used the staged rows as they lie
    finally:
        for sb, _, _ in ready:
            sb.free()
