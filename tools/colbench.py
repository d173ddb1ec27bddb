"""Column-program encode: parity spot check + timing at a batch config (GPU).

usage: python tools/colbench.py [K] [T] [N] [blocks] [iters]
RQBENCH_PAD=bytes pads the source block stride (a view into a wider buffer).
"""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402

if os.environ.get("RQHIP_LIB"):  # an alternative build (e.g. tools/build_experiments.sh)
    rqhip.LIB_PATH = Path(os.environ["RQHIP_LIB"])


def main():
    K, T, N, B, iters = (int(x) for x in (sys.argv[1:6] + ["1024", "1200", "1100", "1024", "10"][len(sys.argv) - 1:]))
    dev = torch.device("cuda:0")
    esis = list(range(K, N))
    g = torch.Generator(device=dev).manual_seed(5)
    pad = int(os.environ.get("RQBENCH_PAD", "0"))
    src = torch.randint(0, 256, (B, K * T + pad), dtype=torch.uint8, device=dev, generator=g)[:, :K * T]
    out = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
    t0 = time.time()
    rqhip.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    print("first call (compile + run) %.3f s" % (time.time() - t0), flush=True)
    from oracle import oracle as O
    for b in (0, B - 1):
        ref = O.OracleEncoder(src[b].cpu().numpy().tobytes(), T)
        got = out[b].cpu().numpy().reshape(N - K, T)
        bad = [r for r in range(N - K) if not np.array_equal(got[r], ref.gen_symbol(K + r))]
        print("block", b, "mismatching repairs:", bad[:10], len(bad), flush=True)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        rqhip.encode_batch(src, K, T, esis, out)
    e0.record(s)
    for _ in range(iters):
        rqhip.encode_batch(src, K, T, esis, out)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print("encode K=%d T=%d N=%d blocks=%d: %.4f ms/launch, %.1f GB/s source" % (K, T, N, B, ms, B * K * T / ms / 1e6),
          flush=True)


if __name__ == "__main__":
    main()
