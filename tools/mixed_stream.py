"""BASELINE.json config 5 on one GPU: a round-robin stream of K in {128, 512, 2048} x T in {256, 1200}
blocks at 5 % loss (the go/fecquic loopback shape, N = K + K/10 + 8), end to end including pinned
H2D/D2H: per shape, source -> H2D -> encode -> D2H repairs, then received rows + repairs -> H2D ->
decode -> D2H payload, chunks pipelined on two streams.  Every payload is checked bit-exactly.
Each rank of a multi-GPU run would take its own share of the stream (blocks are independent).

usage: python tools/mixed_stream.py [MB per shape] [iters]
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


def run_shape(K, T, mb, iters, rng, dev, streams):
    N = K + K // 10 + 8
    R = N - K
    n_erase = round(0.05 * N)
    B = max(8, int(mb * 2 ** 20 // (K * T)))
    CH = max(1, B // 8)
    host_src = torch.from_numpy(rng.integers(0, 256, (B, K * T), dtype=np.uint8)).pin_memory()
    host_rep = torch.empty((B, R * T), dtype=torch.uint8).pin_memory()
    esis = list(range(K, N))
    d_src = [torch.empty((CH, K * T), dtype=torch.uint8, device=dev) for _ in streams]
    d_rep = [torch.empty((CH, R * T), dtype=torch.uint8, device=dev) for _ in streams]

    def enc():
        for i, c0 in enumerate(range(0, B, CH)):
            s, nb = streams[i % 2], min(CH, B - c0)
            with torch.cuda.stream(s):
                d_src[i % 2][:nb].copy_(host_src[c0:c0 + nb], non_blocking=True)
                rqhip.encode_batch(d_src[i % 2][:nb], K, T, esis, d_rep[i % 2][:nb], stream=s)
                host_rep[c0:c0 + nb].copy_(d_rep[i % 2][:nb], non_blocking=True)
        torch.cuda.synchronize()

    enc()
    t0 = time.perf_counter()
    for _ in range(iters):
        enc()
    t_enc = (time.perf_counter() - t0) / iters
    er, rl = [], []
    for b in range(B):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in range(K, N) if e not in lost])
    host_data = host_src.clone()
    for b in range(B):
        for i in er[b]:
            host_data[b, i * T:(i + 1) * T] = 0
    host_data = host_data.pin_memory()
    hrv = host_rep.view(B, R, T)
    chunks = []
    for c0 in range(0, B, CH):
        nb = min(CH, B - c0)
        rows = torch.cat([hrv[c0 + b, [e - K for e in rl[c0 + b]]] for b in range(nb)]).pin_memory()
        chunks.append((c0, nb, rows, rqhip.DecodeBatch(K, T, er[c0:c0 + nb], rl[c0:c0 + nb])))
    d_data = [torch.empty((CH, K * T), dtype=torch.uint8, device=dev) for _ in streams]
    d_recv = [torch.empty((CH * R, T), dtype=torch.uint8, device=dev) for _ in streams]
    host_out = torch.empty((B, K * T), dtype=torch.uint8).pin_memory()

    def dec():
        ok = 0
        for i, (c0, nb, rows, db) in enumerate(chunks):
            s = streams[i % 2]
            with torch.cuda.stream(s):
                d_data[i % 2][:nb].copy_(host_data[c0:c0 + nb], non_blocking=True)
                d_recv[i % 2][:len(rows)].copy_(rows, non_blocking=True)
                st = db.run(d_data[i % 2][:nb], d_recv[i % 2][:len(rows)], stream=s)
                host_out[c0:c0 + nb].copy_(d_data[i % 2][:nb], non_blocking=True)
                ok += int((st == 1).sum())
        torch.cuda.synchronize()
        return ok

    ok = dec()
    good = torch.equal(host_out, host_src) if ok == B else None
    t0 = time.perf_counter()
    for _ in range(iters):
        dec()
    t_dec = (time.perf_counter() - t0) / iters
    src_bytes = B * K * T
    return {"K": K, "T": T, "N": N, "blocks": B, "decoded": ok, "bit_exact": good,
            "encode_GBps": round(src_bytes / t_enc / 1e9, 2), "decode_GBps": round(src_bytes / t_dec / 1e9, 2),
            "t_enc": t_enc, "t_dec": t_dec, "bytes": src_bytes}


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 128
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    rng = np.random.default_rng(5)
    res = [run_shape(K, T, mb, iters, rng, dev, streams) for K in (128, 512, 2048) for T in (256, 1200)]
    tot_b = sum(r["bytes"] for r in res)
    tot_t = sum(r["t_enc"] + r["t_dec"] for r in res)
    for r in res:
        r.pop("t_enc"), r.pop("t_dec"), r.pop("bytes")
    print(json.dumps({"what": "mixed K x T stream, 5% loss, end-to-end incl. pinned H2D/D2H, 1 GPU",
                      "shapes": res, "encode_plus_decode_GBps": round(tot_b / tot_t / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
