"""Experiments library only (RQHIP_LIB=.../build_exp/librqhip.so): k_solve_ip (rows of e bytes, in-place
Gauss-Jordan) and the shipped k_solve_pq<1, 4> give the same statuses and bytes; e > 64 takes the wide /
general solvers either way.  Run by tests/test_gpu_experimental_programs.py in its own process (the
release library has no k_solve_ip).  Prints one "ok <case>" line per case; exits non-zero on a mismatch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "rl-quic-raptor_amd"))
import rqhip as rq  # noqa: E402

CASES = [
    (1024, 1200, 76, [55, 1, 16, 17, 33, 48, 49, 64, 2, 3, 0, 63], 8),
    (256, 256, 80, [64, 70, 5, 1, 32], 8),
    (64, 8, 20, [20, 19, 1, 6], 8),
    (128, 256, 40, [40, 30, 20, 39, 8, 16], 0),  # no row margin: rank-deficient first passes
]


def case(gpu, K, T, R, erase_counts, seed):
    g = torch.Generator().manual_seed(seed)
    n = len(erase_counts)
    src = torch.randint(0, 256, (n, K * T), dtype=torch.uint8, generator=g).to(gpu)
    out = torch.empty((n, R * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, list(range(K, K + R)), out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    erased = [sorted(rng.choice(K, ne, replace=False).tolist()) if ne else [] for ne in erase_counts]
    reps = [list(range(K, K + R)) for _ in erase_counts]
    data = src.clone()
    for b, er in enumerate(erased):
        for i in er:
            data[b, i * T:(i + 1) * T] = (b * 31 + i) & 0xFF
    return src, data, erased, reps, out.view(n * R, T).contiguous()


def main():
    gpu = torch.device("cuda:0")
    assert "build_exp" in str(rq.LIB_PATH), rq.LIB_PATH
    for K, T, R, ec, margin in CASES:
        src, data, erased, reps, rep = case(gpu, K, T, R, ec, 3 * K + T)
        old_m = rq.lib().rq_debug_decode_margin(margin)
        res = []
        try:
            for mode in (0, 1):
                d = data.clone()
                old = rq.solve_mode(mode)
                try:
                    st = np.array(rq.DecodeBatch(K, T, erased, reps).run(d, rep))
                    torch.cuda.synchronize()
                finally:
                    rq.solve_mode(old)
                res.append((d, st))
        finally:
            rq.lib().rq_debug_decode_margin(old_m)
        (d0, st0), (d1, st1) = res
        assert np.array_equal(st0, st1), (K, st0, st1)
        for b in range(len(ec)):
            assert torch.equal(d0[b], d1[b]), (K, b)
            if st1[b] == 1:
                assert torch.equal(d1[b], src[b]), (K, b)
        print("ok", K, T, R, ec, margin, flush=True)


if __name__ == "__main__":
    main()
