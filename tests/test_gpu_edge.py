"""GPU edge cases of the batch path: sparse repair ESIs (the decode union is then the exact sorted
set, not a dense range), descriptor lists in arbitrary order, large K (allocator under extreme
register pressure: thousands of scratch slots), and the largest symbol ids the 24-bit ESI space
allows.  Bytes against the oracle where it is fast enough, else against the CPU port (held to the
oracle by tests/test_cpu_baseline.py)."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqcpu  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)


def _src(gpu, nb, K, T, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    return torch.randint(0, 256, (nb, K * T), dtype=torch.uint8, device=gpu, generator=g)


def test_sparse_repair_esis_decode(gpu, rq, oracle):
    """Received repairs at scattered ESIs up to ~2^20, a different set per block: the engine compiles
    the exact union (binary-searched union indices) and every block decodes to the oracle's bytes."""
    K, T, nb = 64, 256, 6
    rng = np.random.default_rng(5)
    src = _src(gpu, nb, K, T, 5)
    src_h = src.cpu().numpy()
    er, rl, rows = [], [], []
    for b in range(nb):
        e = sorted(rng.choice(K, 4 + b, replace=False).tolist())
        esis = sorted(set((K + rng.integers(0, 1 << 20, 12 + b)).tolist()))
        ref = oracle.OracleEncoder(src_h[b].tobytes(), T)
        er.append(e)
        rl.append(esis)
        rows.extend(ref.gen_symbol(x) for x in esis)
    rep = torch.from_numpy(np.stack(rows)).to(gpu)
    data = src.clone()
    for b in range(nb):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0x5A
    st = rq.DecodeBatch(K, T, er, rl).run(data, rep)
    torch.cuda.synchronize()
    assert (st == 1).all()
    assert torch.equal(data, src)


def test_unsorted_descriptor_lists(gpu, rq, oracle):
    """Erased and repair lists in arbitrary order (the receiver's arrival order): same bytes."""
    K, T, N, nb = 128, 1200, 148, 4
    rng = np.random.default_rng(9)
    src = _src(gpu, nb, K, T, 9)
    esis = list(range(K, N))
    out = torch.empty((nb, (N - K) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    er, rl, rows = [], [], []
    for b in range(nb):
        e = rng.choice(K, 9, replace=False).tolist()           # unsorted
        r = rng.permutation(np.arange(K, N))[:14].tolist()     # unsorted
        er.append(e)
        rl.append(r)
        rows.extend(out[b].view(N - K, T)[x - K] for x in r)
    rep = torch.stack(rows)
    data = src.clone()
    for b in range(nb):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0
    st = rq.DecodeBatch(K, T, er, rl).run(data, rep)
    torch.cuda.synchronize()
    assert (st == 1).all() and torch.equal(data, src)


@pytest.mark.parametrize("K,R", [(4096, 40), (8192, 24)])
def test_large_k_encode(gpu, rq, K, R):
    """K = 4096 / 8192: programs with 5 000 / 13 600 scratch spills per item (and slots past the
    preloaded soffset bases).  Repairs of every block against the CPU port; one block's repairs at
    the top of the 24-bit ESI space too."""
    T, nb = 64, 16
    src = _src(gpu, nb, K, T, K)
    for esis in (list(range(K, K + R)), list(range((1 << 24) - R, 1 << 24))):
        out = torch.empty((nb, R * T), dtype=torch.uint8, device=gpu)
        rq.encode_batch(src, K, T, esis, out)
        torch.cuda.synchronize()
        ref = rqcpu.encode(src.cpu().numpy(), K, T, esis, THREADS)
        assert np.array_equal(out.cpu().numpy(), ref)


def test_large_k_decode_round_trip(gpu, rq):
    """K = 4096, 2 % of N erased: every block decodes back to its source."""
    K, T, nb = 4096, 64, 8
    N = K + K // 20
    rng = np.random.default_rng(17)
    src = _src(gpu, nb, K, T, 17)
    esis = list(range(K, N))
    out = torch.empty((nb, (N - K) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    er, rl, rows = [], [], []
    for b in range(nb):
        lost = set(rng.choice(N, N // 50, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
        rows.extend(out[b].view(N - K, T)[e - K] for e in rl[-1])
    rep = torch.stack(rows)
    data = src.clone()
    for b in range(nb):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0xFF
    st = rq.DecodeBatch(K, T, er, rl).run(data, rep)
    torch.cuda.synchronize()
    assert (st == 1).all() and torch.equal(data, src)


def _sparse_case(gpu, oracle, K, T, nb, seed, lo, hi, skip_block=None):
    """Blocks with scattered received repair ESIs in [lo, hi); block `skip_block` loses nothing (its
    status is decided on the host, so it is not solved)."""
    rng = np.random.default_rng(seed)
    src = _src(gpu, nb, K, T, seed)
    src_h = src.cpu().numpy()
    er, rl, rows = [], [], []
    for b in range(nb):
        e = [] if b == skip_block else sorted(rng.choice(K, 3 + b, replace=False).tolist())
        esis = sorted(set(rng.integers(lo, hi, 10 + b).tolist()))
        ref = oracle.OracleEncoder(src_h[b].tobytes(), T)
        er.append(e)
        rl.append(esis)
        rows.extend(ref.gen_symbol(x) for x in esis)
    rep = torch.from_numpy(np.stack(rows)).to(gpu)
    data = src.clone()
    for b in range(nb):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0xC3
    return src, data, rep, er, rl


def test_sparse_repair_esis_decode_async(gpu, rq, oracle):
    """The async path over a sparse union (every block offers all its received repairs, so the host
    plan bounds the union by the argument check's maximum; the union is the exact sorted set)."""
    K, T, nb = 64, 256, 5
    src, data, rep, er, rl = _sparse_case(gpu, oracle, K, T, nb, 21, K, K + (1 << 18))
    db = rq.DecodeBatch(K, T, er, rl)
    st = db.run_async(data, rep)
    torch.cuda.synchronize()
    assert (st == 1).all()
    assert torch.equal(data, src)


def test_far_repair_esis_decode_unmapped_union(gpu, rq, oracle):
    """Received repairs near the top of the 24-bit ESI space (more than 2^22 past K: the host plan
    builds the union by sorting, union indices by binary search), one block with nothing lost
    (not solved: its status comes from the host), sync and async."""
    K, T, nb = 64, 256, 4
    for run in ("run", "run_async"):
        src, data, rep, er, rl = _sparse_case(gpu, oracle, K, T, nb, 33, (1 << 24) - 4096, 1 << 24, skip_block=1)
        st = getattr(rq.DecodeBatch(K, T, er, rl), run)(data, rep)
        torch.cuda.synchronize()
        assert (st == 1).all(), (run, st)
        assert torch.equal(data, src), run
