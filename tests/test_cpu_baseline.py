"""librqcpu.so (the CPU baseline bench.py times: this engine's column-program algorithm on host cores)
against the oracle: repair symbols and decoded payloads bit for bit, rank-deficient and
not-enough-symbols statuses, several threads."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "rl-quic-raptor_amd"))
import rqcpu  # noqa: E402


@pytest.mark.parametrize("K,T,R", [(64, 1200, 16), (256, 1201, 26), (10, 16, 8), (1024, 64, 76), (2048, 40, 20)])
def test_cpu_encode_matches_oracle(oracle, K, T, R):
    rng = np.random.default_rng(K + T)
    src = rng.integers(0, 256, (3, K * T), dtype=np.uint8)
    esis = list(range(K, K + R)) + [K + 5000]
    out = rqcpu.encode(src, K, T, esis, threads=2)
    ref = oracle.OracleEncoder(src[1].tobytes(), T)
    for r, e in enumerate(esis):
        assert np.array_equal(out[1, r * T:(r + 1) * T], ref.gen_symbol(e)), e


@pytest.mark.parametrize("K,T,N,n_erase", [(64, 1200, 80, 8), (256, 64, 282, 14), (1024, 32, 1100, 55),
                                           (128, 16, 400, 30)])
def test_cpu_decode_matches_oracle(oracle, K, T, N, n_erase):
    rng = np.random.default_rng(N)
    nb = 4
    src = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    esis = list(range(K, N))
    rep = rqcpu.encode(src, K, T, esis)
    er, rl, rows = [], [], []
    data = src.copy()
    for b in range(nb):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
        rows += [rep[b, (e - K) * T:(e - K + 1) * T] for e in rl[-1]]
        for i in er[-1]:
            data[b, i * T:(i + 1) * T] = 0x5A
    st = rqcpu.decode(data, K, T, er, rl, np.stack(rows), threads=3)
    for b in range(nb):
        d = oracle.OracleDecoder(K * T, T)
        for i in range(K):
            if i not in er[b]:
                d.add_symbol(i, src[b, i * T:(i + 1) * T].tobytes())
        for r, e in enumerate(rl[b]):
            d.add_symbol(e, rep[b, (e - K) * T:(e - K + 1) * T].tobytes())
        ok, out = d.decode()
        assert (st[b] == 1) == ok
        if ok:
            assert data[b].tobytes() == out == src[b].tobytes()


def test_cpu_decode_statuses(oracle):
    """Not enough symbols (-3), nothing erased (1), and a rank-deficient received = K pattern (0)."""
    K, T = 64, 16
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    N = K + K // 2
    enc = oracle.OracleEncoder(data.tobytes(), T)
    syms = {i: enc.gen_symbol(i) for i in range(N)}
    bad = None
    for _ in range(4000):
        ids = sorted(rng.choice(N, K, replace=False).tolist())
        d = oracle.OracleDecoder(K * T, T)
        for i in ids:
            d.add_symbol(i, syms[i].tobytes())
        if not d.decode()[0]:
            bad = ids
            break
    assert bad is not None
    blocks = [(list(range(5)), [K, K + 1]), ([], []), ([i for i in range(K) if i not in bad], [e for e in bad if e >= K])]
    buf = np.stack([data] * 3).copy()
    rows = [syms[e] for _, rl in blocks for e in rl]
    st = rqcpu.decode(buf, K, T, [b[0] for b in blocks], [b[1] for b in blocks], np.stack(rows))
    assert list(st) == [-3, 1, 0]
