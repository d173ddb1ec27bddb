"""Launches profiled by tools/gpu_profile.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes).

1. Calibration: the column program with outputs = the K=10 source rows themselves (ESIs 0..9) is a
   pure copy in the encode kernel's own access pattern (4-byte-per-lane buffer loads and stores of
   256-B row segments).  At T=1024 every segment is whole 128-B lines that no other wave touches, so
   it reads and writes exactly blocks*10*T bytes and FETCH_SIZE / WRITE_SIZE of that launch calibrate
   the counters for this access width (rq_colprog_K10_n10).
2. The bench workload's encode launch: K=1024 T=1200 N=1100, 1024 blocks (rq_colprog_K1024_n76).
3. BASELINE config 2's encode launch: K=256 T=1200, 26 repairs, 1024 blocks (rq_colprog_K256_n26).
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    Tc, Bc = 1024, 65536
    src = torch.randint(0, 256, (Bc, 10 * Tc), dtype=torch.uint8, device=dev)
    out = torch.empty_like(src)
    for _ in range(3):
        rqhip.encode_batch(src, 10, Tc, list(range(10)), out)
    torch.cuda.synchronize()
    assert torch.equal(src, out)
    del src, out
    T = 1200
    K, N, B = 1024, 1100, 1024
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev)
    rep = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
    for _ in range(3):
        rqhip.encode_batch(src, K, T, list(range(K, N)), rep)
    torch.cuda.synchronize()
    del src, rep
    # 3. BASELINE config 2's encode launch: K=256 T=1200, 26 repairs, 1024 blocks (rq_colprog_K256_n26)
    K2, R2 = 256, 26
    src = torch.randint(0, 256, (B, K2 * T), dtype=torch.uint8, device=dev)
    rep = torch.empty((B, R2 * T), dtype=torch.uint8, device=dev)
    for _ in range(3):
        rqhip.encode_batch(src, K2, T, list(range(K2, K2 + R2)), rep)
    torch.cuda.synchronize()
    print("calibration bytes per launch", Bc * 10 * Tc, "encode source bytes per launch", B * K * T, "config 2",
          B * K2 * T)


if __name__ == "__main__":
    main()
