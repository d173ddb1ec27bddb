"""GPU parity of the host-memory batch API (rq_encode_batch_host / rq_decode_batch_host): the path a
cgo caller without device memory takes (fecquic sender windows and receiver workers, SURVEY.md
sec. 8f rank 1).  Results must equal the device-resident batch API's bit for bit, across several
pipeline chunks, strided and pageable or pinned host buffers."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _device_encode(rq, gpu, src_h, K, T, esis):
    src = torch.from_numpy(np.ascontiguousarray(src_h[:, :K * T])).to(gpu)
    out = torch.empty((src.shape[0], len(esis) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_host_encode_matches_device_batch(gpu, rq):
    # 1000 blocks at T=1200: three pipeline chunks (>= 410 blocks each) on the two internal streams
    K, T, R, nb = 64, 1200, 16, 1000
    esis = list(range(K, K + R))
    rng = np.random.default_rng(31)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)            # pageable
    ref = _device_encode(rq, gpu, src, K, T, esis)
    out = torch.zeros((nb, R * T), dtype=torch.uint8).pin_memory()    # pinned
    rq.encode_batch_host(src, K, T, esis, out)
    assert np.array_equal(out.numpy(), ref)
    # strided source rows (a wider host buffer) and strided repair rows: per-block copies
    wide = np.zeros((nb, K * T + 64), np.uint8)
    wide[:, :K * T] = src
    out2 = np.full((nb, R * T + 128), 7, np.uint8)
    rq.encode_batch_host(wide, K, T, esis, out2[:, :])
    assert np.array_equal(out2[:, :R * T], ref)
    assert (out2[:, R * T:] == 7).all()


def test_host_encode_bench_shape(gpu, rq):
    # the bench block shape (K=1024, T=1200, 76 repairs) on a small batch
    K, T, R, nb = 1024, 1200, 76, 8
    esis = list(range(K, K + R))
    src = np.random.default_rng(5).integers(0, 256, (nb, K * T), dtype=np.uint8)
    out = np.zeros((nb, R * T), np.uint8)
    rq.encode_batch_host(src, K, T, esis, out, device_mask=1)
    assert np.array_equal(out, _device_encode(rq, gpu, src, K, T, esis))


@pytest.mark.parametrize("K,T,N,nb,n_erase", [(64, 1200, 80, 1000, 8), (1024, 1200, 1100, 12, 55),
                                               (128, 256, 148, 40, 7)])
def test_host_decode_round_trip(gpu, rq, K, T, N, nb, n_erase):
    R = N - K
    esis = list(range(K, N))
    rng = np.random.default_rng(K * 7 + nb)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    rep_all = _device_encode(rq, gpu, src, K, T, esis).reshape(nb, R, T)
    er, rl, rows = [], [], []
    for b in range(nb):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
        rows.extend(rep_all[b, e - K] for e in rl[-1])
    # one block with too few symbols: status RQ_ERR_NOT_ENOUGH, its rows untouched
    er[1] = list(range(R + 1))
    rl[1] = esis
    rows = [rep_all[b, e - K] for b in range(nb) for e in rl[b]]
    repair = torch.from_numpy(np.stack(rows)).pin_memory()
    data = torch.from_numpy(src.copy()).pin_memory()
    d3 = data.numpy().reshape(nb, K, T)
    for b in range(nb):
        d3[b, er[b]] = 0xA5
    before = data.numpy().copy()
    db = rq.DecodeBatch(K, T, er, rl)
    st = rq.decode_batch_host(db, data, repair).copy()
    assert st[1] == rq.RQ_ERR_NOT_ENOUGH
    assert np.array_equal(data.numpy()[1], before[1])
    ok = st == 1
    assert ok.sum() >= nb - 2 - nb // 20
    assert np.array_equal(data.numpy()[ok], src[ok])
    assert np.array_equal(data.numpy()[~ok], before[~ok])
    # same statuses as the device-resident batch
    dd = torch.from_numpy(before).to(gpu)
    db2 = rq.DecodeBatch(K, T, er, rl)
    st2 = db2.run(dd, repair.to(gpu))
    torch.cuda.synchronize()
    assert np.array_equal(st, st2)


def test_host_batch_bad_device_mask(gpu, rq):
    K, T = 64, 64
    src = np.zeros((1, K * T), np.uint8)
    out = np.zeros((1, T), np.uint8)
    with pytest.raises(rq.RaptorQError) as ei:
        rq.encode_batch_host(src, K, T, [K], out, device_mask=1 << 31)
    assert ei.value.code == rq.RQ_ERR_BAD_ARG


@pytest.mark.parametrize("K,T,N", [(64, 1201, 80), (26, 1499, 32), (10, 3, 16)])
def test_host_api_any_symbol_size(gpu, rq, oracle, K, T, N):
    """T not a multiple of 4 through the host-memory API (rows padded in device staging): repairs
    and recovered payloads equal the oracle's."""
    nb = 5
    esis = list(range(K, N))
    rng = np.random.default_rng(T)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    out = np.zeros((nb, len(esis) * T), np.uint8)
    rq.encode_batch_host(src, K, T, esis, out)
    for b in (0, nb - 1):
        ref = oracle.OracleEncoder(src[b].tobytes(), T)
        for r, e in enumerate(esis):
            assert np.array_equal(out[b, r * T:(r + 1) * T], ref.gen_symbol(e)), (b, e)
    er, rl, rows = [], [], []
    for b in range(nb):
        lost = set(rng.choice(N, 3, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
        rows += [out[b, (e - K) * T:(e - K + 1) * T] for e in rl[-1]]
    data = src.copy()
    for b in range(nb):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0
    db = rq.DecodeBatch(K, T, er, rl)
    st = rq.decode_batch_host(db, data, np.stack(rows))
    assert (st == 1).all() and np.array_equal(data, src)


def test_decode_blocks_host_matches_batch(gpu, rq):
    """rq_decode_blocks_host (per-block buffers: a receiver's staging) decodes like
    rq_decode_batch_host; blocks may sit anywhere in host memory, pinned or not."""
    K, T, N, nb = 128, 1200, 148, 9
    esis = list(range(K, N))
    rng = np.random.default_rng(77)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    rep = _device_encode(rq, gpu, src, K, T, esis).reshape(nb, N - K, T)
    blocks = []
    for b in range(nb):
        lost = set(rng.choice(N, 7, replace=False).tolist())
        er = sorted(i for i in lost if i < K)
        rl = [e for e in esis if e not in lost]
        buf = (torch.from_numpy(src[b].copy()).pin_memory() if b % 2 else src[b].copy())
        view = buf.numpy() if hasattr(buf, "numpy") else buf
        for i in er:
            view[i * T:(i + 1) * T] = 0x33
        blocks.append((buf, er, rl, np.stack([rep[b, e - K] for e in rl])))
    st = rq.decode_blocks_host(K, T, blocks)
    assert st == [1] * nb
    for b, (buf, *_rest) in enumerate(blocks):
        view = buf.numpy() if hasattr(buf, "numpy") else buf
        assert np.array_equal(view, src[b])


def test_host_batch_virtual_shards(gpu, rq):
    """The per-device host threads of the host-memory batch calls (run_sharded), driven on one GPU by
    splitting its blocks over 3 threads: the same repairs and decoded payloads as one thread."""
    K, T, N, nb = 64, 1200, 80, 7
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    esis = list(range(K, N))
    ref = np.zeros((nb, (N - K) * T), np.uint8)
    rq.encode_batch_host(src, K, T, esis, ref)
    old = rq.lib().rq_debug_virtual_shards(3)
    try:
        out = np.zeros_like(ref)
        rq.encode_batch_host(src, K, T, esis, out)
        assert np.array_equal(out, ref)
        er = [sorted(rng.choice(K, 5, replace=False).tolist()) for _ in range(nb)]
        rl = [esis[:12] for _ in range(nb)]
        data = src.copy()
        for b in range(nb):
            for i in er[b]:
                data[b, i * T:(i + 1) * T] = 0
        repair = np.concatenate([ref[b].reshape(N - K, T)[:12] for b in range(nb)])  # [n_rows, T]
        db = rq.DecodeBatch(K, T, er, rl)
        st = rq.decode_batch_host(db, data, repair)
        assert (st == 1).all() and np.array_equal(data, src)
    finally:
        rq.lib().rq_debug_virtual_shards(old)


def test_host_decode_forced_retry_multi_chunk(gpu, rq):
    """Host-memory decode over several pipeline chunks (1 000 blocks of 76.8 KB) with the subset
    margin forced to 0: each block's first pass solves on exactly e repairs, so some are rank-
    deficient and take the all-repairs pass inside the chunk's collect step (after the first pass's
    rows were scattered).  Every block decodes to its source, with the device batch's statuses."""
    K, T, N, nb, n_erase = 64, 1200, 80, 1000, 8
    esis = list(range(K, N))
    rng = np.random.default_rng(31)
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    rep_all = _device_encode(rq, gpu, src, K, T, esis).reshape(nb, N - K, T)
    er, rl = [], []
    for b in range(nb):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
    repair = torch.from_numpy(np.stack([rep_all[b, e - K] for b in range(nb) for e in rl[b]])).pin_memory()
    data = torch.from_numpy(src.copy()).pin_memory()
    d3 = data.numpy().reshape(nb, K, T)
    for b in range(nb):
        d3[b, er[b]] = 0x3C
    before = data.numpy().copy()
    old = rq.lib().rq_debug_decode_margin(0)
    try:
        st = rq.decode_batch_host(rq.DecodeBatch(K, T, er, rl), data, repair).copy()
        dd = torch.from_numpy(before).to(gpu)
        st2 = rq.DecodeBatch(K, T, er, rl).run(dd, repair.to(gpu))
        torch.cuda.synchronize()
    finally:
        rq.lib().rq_debug_decode_margin(old)
    assert (st == 1).all() and np.array_equal(st, st2)
    assert np.array_equal(data.numpy(), src)
    assert np.array_equal(dd.cpu().numpy(), src)
