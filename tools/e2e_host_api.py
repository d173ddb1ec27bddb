"""End-to-end rate of the library's own host-memory batch path (rq_encode_batch_host /
rq_decode_batch_host): what a cgo caller gets.  Payloads, repairs and recovered rows live in pinned
host memory; the library stages through the device in chunks on two internal streams.  Decode
uploads each data block once and downloads only the recovered rows.

usage: python tools/e2e_host_api.py [blocks] [iters] [device_mask]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mask = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    K, T, N, n_erase = 1024, 1200, 1100, 55
    R = N - K
    esis = list(range(K, N))
    rng = np.random.default_rng(3)
    src = torch.from_numpy(rng.integers(0, 256, (B, K * T), dtype=np.uint8)).pin_memory()
    rep = torch.empty((B, R * T), dtype=torch.uint8).pin_memory()
    rqhip.encode_batch_host(src, K, T, esis, rep, mask)  # warm-up: program compile, staging buffers
    t0 = time.perf_counter()
    for _ in range(iters):
        rqhip.encode_batch_host(src, K, T, esis, rep, mask)
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
    for it in range(iters + 1):
        for b in range(B):
            d3[b, er[b]] = 0
        t0 = time.perf_counter()
        st = rqhip.decode_batch_host(db, data, repair, mask)
        times.append(time.perf_counter() - t0)
    ok = st == 1
    assert torch.equal(data[torch.from_numpy(ok)], src[torch.from_numpy(ok)]), "decode mismatch"
    t_dec = float(np.mean(times[1:]))
    src_gb = B * K * T / 1e9
    res = {
        "what": "rq_encode_batch_host / rq_decode_batch_host, pinned host buffers, K=%d T=%d N=%d, %d blocks, "
                "erase %d of N, device_mask=%d" % (K, T, N, B, n_erase, mask),
        "encode_ms": round(t_enc * 1e3, 2), "encode_GBps": round(src_gb / t_enc, 2),
        "encode_pcie_bytes": B * (K + R) * T,
        "decode_ms": round(t_dec * 1e3, 2), "decode_GBps": round(src_gb / t_dec, 2),
        "decode_pcie_bytes": int(B * K * T + repair.numel() + sum(len(e) for e in er) * T),
        "encode_plus_decode_GBps": round(src_gb / (t_enc + t_dec), 2),
        "decode_ok_fraction": float(ok.mean()),
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
