"""One config-5 shape through the host-memory batch API, for a kernel + memory-copy trace: encode
once, then decode_batch_host `reps` times, each timed on the host.
usage: python tools/hostdec_trace.py K T [reps]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402
from bench import erasure_pattern  # noqa: E402


def main():
    K, T = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    N = K + K // 10 + 8
    R, n_erase = N - K, round(0.05 * N)
    B = max(8, int(128 * 2 ** 20 // (K * T)))
    rng = np.random.default_rng(5)
    src = torch.from_numpy(rng.integers(0, 256, (B, K * T), dtype=np.uint8)).pin_memory()
    rep = torch.empty((B, R * T), dtype=torch.uint8).pin_memory()
    er, rl = erasure_pattern(K, N, B, n_erase, 11)
    rqhip.encode_batch_host(src, K, T, list(range(K, N)), rep)
    rv = rep.view(B, R, T)
    repair = torch.cat([rv[b, [e - K for e in rl[b]]] for b in range(B)]).pin_memory()
    data = src.clone().pin_memory()
    db = rqhip.DecodeBatch(K, T, er, rl)
    for i in range(reps):
        t0 = time.perf_counter()
        rqhip.decode_batch_host(db, data, repair)
        dt = time.perf_counter() - t0
        print("decode %d: %.3f ms  %.1f GB/s (H2D bytes %.1f MB)" % (i, dt * 1e3, B * K * T / dt / 1e9,
              (B * K * T + repair.numel()) / 1e6), flush=True)
    assert torch.equal(data, src)


if __name__ == "__main__":
    main()
