"""BASELINE.json config 5 through the library's host-memory batch path: for each K in {128, 512, 2048}
x T in {256, 1200} (N = K + K/10 + 8, 5 % of N erased), rq_encode_batch_host then
rq_decode_batch_host on pinned buffers, payloads checked bit-exactly; per-shape and combined
end-to-end GB/s of source.  usage: python tools/mixed_host_api.py [MB per shape] [iters]"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402


def shape(K, T, mb, iters, rng):
    N = K + K // 10 + 8
    R, n_erase = N - K, round(0.05 * N)
    B = max(8, int(mb * 2 ** 20 // (K * T)))
    esis = list(range(K, N))
    src = torch.from_numpy(rng.integers(0, 256, (B, K * T), dtype=np.uint8)).pin_memory()
    rep = torch.empty((B, R * T), dtype=torch.uint8).pin_memory()
    rqhip.encode_batch_host(src, K, T, esis, rep)
    t0 = time.perf_counter()
    for _ in range(iters):
        rqhip.encode_batch_host(src, K, T, esis, rep)
    t_enc = (time.perf_counter() - t0) / iters
    er, rl = [], []
    for b in range(B):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
    rv = rep.view(B, R, T)
    repair = torch.cat([rv[b, [e - K for e in rl[b]]] for b in range(B)]).pin_memory()
    data = src.clone().pin_memory()
    d3 = data.view(B, K, T)
    db = rqhip.DecodeBatch(K, T, er, rl)
    times = []
    for _ in range(iters + 1):
        for b in range(B):
            d3[b, er[b]] = 0
        t0 = time.perf_counter()
        st = rqhip.decode_batch_host(db, data, repair)
        times.append(time.perf_counter() - t0)
    ok = torch.from_numpy(st == 1)
    assert torch.equal(data[ok], src[ok]), (K, T)
    t_dec = float(np.mean(times[1:]))
    gb = B * K * T / 1e9
    return {"K": K, "T": T, "N": N, "blocks": B, "encode_GBps": round(gb / t_enc, 2),
            "decode_GBps": round(gb / t_dec, 2), "ok_fraction": float(ok.float().mean()),
            "source_GB": gb, "t_enc": t_enc, "t_dec": t_dec}


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rng = np.random.default_rng(5)
    res = [shape(K, T, mb, iters, rng) for K in (128, 512, 2048) for T in (256, 1200)]
    tot_gb = sum(r["source_GB"] for r in res)
    tot_t = sum(r["t_enc"] + r["t_dec"] for r in res)
    print(json.dumps({"what": "config 5 via rq_encode_batch_host / rq_decode_batch_host (pinned host buffers, "
                      "one GPU); GB/s of source end to end", "shapes": res,
                      "combined_encode_plus_decode_GBps": round(tot_gb / tot_t, 2)}), flush=True)


if __name__ == "__main__":
    main()
