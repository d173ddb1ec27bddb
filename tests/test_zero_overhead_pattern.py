"""CPU: config 3's zero-overhead reception pattern (tests/test_gpu_configs.py, seed 61: 55 of 1 100
symbols lost per block, exactly K received) against the oracle decoder.  Whether a block decodes depends
only on its received ESIs, so small symbols (T=16) give the same verdicts as the GPU test's T=1200: the
three blocks the GPU reports rank-deficient fail in the oracle, their neighbours decode."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

DEFICIENT = [433, 567, 868]  # tests/test_gpu_configs.py ZERO_OVERHEAD_DEFICIENT


def _pattern(K=1024, N=1100, nb=1024):
    rng = np.random.default_rng(61)
    er, rl = [], []
    for _ in range(nb):
        lost = set(rng.choice(N, 55, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in range(K, N) if e not in lost][:len(er[-1])])
    return er, rl


def test_zero_overhead_verdicts_match_oracle():
    K, T = 1024, 16
    er, rl = _pattern()
    for b in DEFICIENT + [432, 434, 868 - 1]:
        src = np.random.default_rng(b).integers(0, 256, K * T, dtype=np.uint8)
        enc = O.OracleEncoder(src.tobytes(), T)
        dec = O.OracleDecoder(K * T, T)
        lost = set(er[b])
        for i in range(K):
            if i not in lost:
                dec.add_symbol(i, src[i * T:(i + 1) * T].tobytes())
        for e in rl[b]:
            dec.add_symbol(e, enc.gen_symbol(e).tobytes())
        ok, payload = dec.decode()
        assert ok == (b not in DEFICIENT), b
        if ok:
            assert payload == src.tobytes(), b
