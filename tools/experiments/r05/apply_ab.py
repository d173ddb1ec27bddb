"""A/B of the decode's apply kernels on config 3 (1 024 blocks K=1024 T=1200, 55 of 1 100 symbols erased):
decode_ms of rq_decode_batch_async with rq_debug_apply_mode 0 (k_apply) and 1 (register-table apply),
interleaved, and a bytes check of both against the source.  Usage: python apply_ab.py [reps] [apply|solve]
("solve": rq_debug_solve_mode 0 = k_solve_pq, 1 = in-place k_solve_ip instead)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "rl-quic-raptor_amd"))
import rqhip as rq  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    setm = rq.solve_mode if len(sys.argv) > 2 and sys.argv[2] == "solve" else rq.apply_mode
    K, T, N, B, ne = 1024, 1200, 1100, 1024, 55
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, generator=g).to(dev)
    esis = list(range(K, N))
    out = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
    rq.encode_batch(src, K, T, esis, out)
    rng = np.random.default_rng(5)
    erased, rl, rows = [], [], []
    for b in range(B):
        lost = set(rng.choice(N, ne, replace=False).tolist())
        erased.append(sorted(i for i in lost if i < K))
        r = [e for e in esis if e not in lost]
        rl.append(r)
        rows.extend((b, e - K) for e in r)
    rep = out.view(B, N - K, T)[torch.tensor([b for b, _ in rows], device=dev),
                                torch.tensor([r for _, r in rows], device=dev)].contiguous()
    db = rq.DecodeBatch(K, T, erased, rl)
    data = src.clone()
    res = {0: [], 1: []}
    for mode in (0, 1):
        setm(mode)
        d = src.clone()
        st = db.run(d, rep)
        torch.cuda.synchronize()
        ok = int((np.array(st) == 1).sum())
        same = all(torch.equal(d[b], src[b]) for b in range(B) if st[b] == 1)
        print(f"mode {mode}: solved {ok}/{B}, bytes equal source: {same}", flush=True)
    s = torch.cuda.current_stream()
    for it in range(reps):
        for mode in (0, 1):
            setm(mode)
            for _ in range(2):
                db.run_async(data, rep, stream=s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                db.run_async(data, rep, stream=s)
            e1.record(s)
            torch.cuda.synchronize()
            res[mode].append(e0.elapsed_time(e1) / 5)
    for mode in (0, 1):
        a = np.array(res[mode])
        print(f"mode {mode}: decode_ms median {np.median(a):.4f} min {a.min():.4f} max {a.max():.4f}", flush=True)


if __name__ == "__main__":
    main()
