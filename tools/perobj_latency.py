"""Per-object API latency (GPU) at raptorq_eval / fecquic block shapes: CreateEncoder, GenSymbol per
id, AddSymbol, Decode -- the calls go/fec/raptorq_wrap.go makes per block (cmd/raptorq_eval/main.go:
199-223, fecquic/transfer.go:180, rxbuf.go:351).  Payloads are seeded random; each shape runs a
warm-up block first (program build or disk-cache load), then `blocks` timed blocks.

usage: python tools/perobj_latency.py [blocks] > profiles/<round>_perobj_latency.json
"""
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402

SHAPES = [  # (K, L, N, erasure fraction): fecquic client default, raptorq_eval exp B K=64
    (26, 1500, 32, 0.10),
    (64, 1200, 80, 0.10),
    (256, 1200, 282, 0.05),
]


def one_block(K, L, N, p, rng):
    data = rng.integers(0, 256, K * L, dtype=np.uint8).tobytes()
    t = {}
    t0 = time.perf_counter()
    enc = rqhip.NewRaptorQEncoder(data, K, L)
    t["create_encoder_ms"] = (time.perf_counter() - t0) * 1e3
    syms = {}
    t0 = time.perf_counter()
    for i in range(N):
        syms[i] = enc.GenSymbol(i)
    t["gensymbol_total_ms"] = (time.perf_counter() - t0) * 1e3
    keep = [i for i in range(N) if rng.random() >= p]
    if len(keep) < K:
        keep = list(range(N))[:K + 2]
    dec = rqhip.NewRaptorQDecoder(K * L, L)
    t0 = time.perf_counter()
    for i in keep:
        dec.AddSymbol(i, syms[i])
    t["addsymbol_total_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    ok, out = dec.Decode()
    t["decode_ms"] = (time.perf_counter() - t0) * 1e3
    t["ok"] = bool(ok) and bytes(out) == data
    t["n_add"] = len(keep)
    t["erased_source"] = sum(1 for i in range(K) if i not in set(keep))
    return t


def main():
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rng = np.random.default_rng(1337)
    res = []
    for K, L, N, p in SHAPES:
        one_block(K, L, N, p, rng)  # warm-up: program build / disk-cache load, module load
        runs = [one_block(K, L, N, p, rng) for _ in range(blocks)]
        med = {k: round(statistics.median(r[k] for r in runs), 4)
               for k in ("create_encoder_ms", "gensymbol_total_ms", "addsymbol_total_ms", "decode_ms")}
        med["gensymbol_per_call_us"] = round(med["gensymbol_total_ms"] * 1e3 / N, 2)
        res.append({"K": K, "L": L, "N": N, "erasure": p, "blocks": blocks,
                    "ok_rate": sum(r["ok"] for r in runs) / blocks,
                    "median": med,
                    "reference_go_1core_ms": {"create_encoder": 0.38, "decode": 0.42} if K == 64 else None})
        print(json.dumps(res[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"tool": "perobj_latency", "shapes": res}))


if __name__ == "__main__":
    main()
