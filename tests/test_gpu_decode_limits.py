"""GPU decode beyond the fast solvers: many received repairs, heavy source loss (the general solver
with its basis in LDS and in global memory), rank-deficient batches, and the second pass that
re-solves a block on all its received repairs when the first e + margin are rank-deficient.

The reference decodes any erasure pattern whose system has full rank, from every held symbol
(go/fec/raptorq_wrap.go:72-74 -> RQ/decoder.go:64-134; receiver call site go/fecquic/rxbuf.go:351).
Every case is checked against the oracle (ok flag and bytes)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle_symbols(oracle, data, T, esis):
    enc = oracle.OracleEncoder(data, T)
    return {e: enc.gen_symbol(e).tobytes() for e in esis}


def _oracle_decode(oracle, data, T, held):
    d = oracle.OracleDecoder(len(data), T)
    for e, s in held.items():
        d.add_symbol(e, s)
    return d.decode()


def _batch(rq, gpu, K, T, blocks, mode):
    """blocks: list of (data bytes, {esi: symbol}) with len(data) == K*T.  Decodes them in one batch
    through rq_decode_batch (mode 'sync') or rq_decode_batch_async ('async'); returns (status, data)."""
    nb = len(blocks)
    er, rl, rows = [], [], []
    dat = np.zeros((nb, K * T), np.uint8)
    for b, (data, held) in enumerate(blocks):
        src = np.frombuffer(data, np.uint8)
        er.append([i for i in range(K) if i not in held])
        rl.append(sorted(e for e in held if e >= K))
        rows.extend(held[e] for e in rl[-1])
        dat[b] = src
        for i in er[-1]:
            dat[b, i * T:(i + 1) * T] = 0xA5
    d_data = torch.from_numpy(dat).to(gpu)
    rep = np.frombuffer(b"".join(rows) or bytes(T), np.uint8).reshape(-1, T)
    d_rep = torch.from_numpy(rep.copy()).to(gpu)
    db = rq.DecodeBatch(K, T, er, rl)
    if mode == "sync":
        st = db.run(d_data, d_rep).copy()
    else:
        st = db.run_async(d_data, d_rep, stream=torch.cuda.current_stream(gpu))
        torch.cuda.synchronize()
        st = st.copy()
    return st, d_data.cpu().numpy()


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_many_received_repairs(gpu, rq, oracle, mode):
    """K=1024, N=1400, 5 % loss: ~357 received repairs per block (beyond the old 255 limit)."""
    K, T, N = 1024, 64, 1400
    rng = np.random.default_rng(31)
    blocks = []
    for b in range(3):
        data = rng.integers(0, 256, K * T, dtype=np.uint8).tobytes()
        syms = _oracle_symbols(oracle, data, T, range(N))
        lost = set(rng.choice(N, 70, replace=False).tolist())
        blocks.append((data, {e: s for e, s in syms.items() if e not in lost}))
    assert min(sum(e >= K for e in h) for _, h in blocks) > 300
    st, out = _batch(rq, gpu, K, T, blocks, mode)
    for b, (data, held) in enumerate(blocks):
        ok, ref = _oracle_decode(oracle, data, T, held)
        assert ok and st[b] == 1, (b, st[b])
        assert out[b].tobytes() == ref == data


@pytest.mark.parametrize("n_lost", [200, 307])
def test_heavy_source_loss(gpu, rq, oracle, n_lost):
    """30 % of the sources lost at K=1024 (e = 307: the general solver's basis in global memory)
    and e = 200 (basis in LDS), through the batch path and the per-object decoder."""
    K, T = 1024, 64
    rng = np.random.default_rng(n_lost)
    data = rng.integers(0, 256, K * T, dtype=np.uint8).tobytes()
    N = K + n_lost + 40
    syms = _oracle_symbols(oracle, data, T, range(N))
    lost = set(rng.choice(K, n_lost, replace=False).tolist()) | set(rng.choice(range(K, N), 20, replace=False).tolist())
    held = {e: s for e, s in syms.items() if e not in lost}
    ok, ref = _oracle_decode(oracle, data, T, held)
    assert ok and ref == data
    st, out = _batch(rq, gpu, K, T, [(data, held)], "sync")
    assert st[0] == 1 and out[0].tobytes() == data
    dec = rq.NewRaptorQDecoder(len(data), T)
    for e in sorted(held):
        dec.AddSymbol(e, held[e])
    assert dec.Decode() == (True, data)


def _rank_deficient(oracle, K, T, seed, want=2):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, K * T, dtype=np.uint8).tobytes()
    N = K + K // 2
    syms = _oracle_symbols(oracle, data, T, range(N + 16))
    found = []
    for _ in range(4000):
        ids = sorted(rng.choice(N, K, replace=False).tolist())
        if not _oracle_decode(oracle, data, T, {i: syms[i] for i in ids})[0]:
            found.append(ids)
            if len(found) >= want:
                break
    return data, syms, N, found


def test_rank_deficient_batch_and_second_pass(gpu, rq, oracle):
    """Received = K rank-deficient patterns through the batch path (sync and async: status 0, as
    the reference's (false, nil, nil)); then three more repairs with ESIs above all received ones
    and the subset margin forced to 0, so the first pass (first e repairs) is rank-deficient and
    the second pass (all repairs) decodes: ok/bytes as the oracle."""
    K, T = 64, 16
    data, syms, N, found = _rank_deficient(oracle, K, T, 17)
    assert found, "no rank-deficient pattern found"
    blocks = [(data, {i: syms[i] for i in ids}) for ids in found]
    for mode in ("sync", "async"):
        st, _ = _batch(rq, gpu, K, T, blocks, mode)
        assert list(st) == [0] * len(found), (mode, st)
    more = [(data, {**h, **{e: syms[e] for e in range(N, N + 3)}}) for _, h in blocks]
    old = rq.lib().rq_debug_decode_margin(0)
    try:
        # sync: the host's second pass; async: every received repair in one call, so the first solver
        # finishes the block itself on all of them (inline_general)
        res = {mode: _batch(rq, gpu, K, T, more, mode) for mode in ("sync", "async")}
    finally:
        rq.lib().rq_debug_decode_margin(old)
    for mode, (st, out) in res.items():
        for b, (_, held) in enumerate(more):
            ok, ref = _oracle_decode(oracle, data, T, held)
            assert (st[b] == 1) == ok, (mode, b)
            if ok:
                assert out[b].tobytes() == ref == data, (mode, b)


def test_first_solver_finishes_rank_deficient_rows_inline(gpu, rq, oracle):
    """One erased source (e = 1) whose coefficient is zero in the first e + margin received repairs (the
    first solver's rows are rank-deficient by construction) and nonzero in a later one: the block is
    recovered in one call.  Round 6: with no block beyond e = 64 the first solver runs the general
    algorithm on every received repair itself (SolveArgs::inline_general, general_block) instead of
    deferring to a k_solve launch, and writes the async call's status; a block whose received repairs
    all have a zero coefficient stays undecodable (status 0, as the oracle)."""
    K, T, c = 32, 16, 5
    rng = np.random.default_rng(41)
    unit = np.zeros(K * T, np.uint8)
    unit[c * T:(c + 1) * T] = 1
    coef = oracle.OracleEncoder(unit.tobytes(), T)
    margin = rq.lib().rq_debug_decode_margin(8)  # (returns the current margin; restored below)
    rq.lib().rq_debug_decode_margin(margin)
    zeros, esi = [], K  # the received list is sorted: its first e + margin rows are these
    while len(zeros) < margin + 1:
        if coef.gen_symbol(esi)[0] == 0:
            zeros.append(esi)
        esi += 1
        assert esi < K + 40000, "not enough zero-coefficient repairs"
    while coef.gen_symbol(esi)[0] == 0:
        esi += 1
    data = rng.integers(0, 256, K * T, dtype=np.uint8).tobytes()
    syms = _oracle_symbols(oracle, data, T, list(range(K)) + zeros + [esi])
    src = {i: syms[i] for i in range(K) if i != c}
    solvable = {**src, **{e: syms[e] for e in zeros + [esi]}}
    hopeless = {**src, **{e: syms[e] for e in zeros}}
    assert _oracle_decode(oracle, data, T, solvable) == (True, data)
    assert not _oracle_decode(oracle, data, T, hopeless)[0]
    for mode in ("async", "sync"):
        st, out = _batch(rq, gpu, K, T, [(data, solvable), (data, hopeless), (data, solvable)], mode)
        assert list(st) == [1, 0, 1], (mode, st)
        assert out[0].tobytes() == data and out[2].tobytes() == data, mode
