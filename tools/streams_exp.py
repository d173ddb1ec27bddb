"""Encode+decode of the bench workload (1 024 blocks K=1024 T=1200, 55 of 1 100 erased) split into S
equal parts on S streams of one process, against S = 1: whole-step time per S.  (Two processes sharing
one GPU ran the step 8 % faster per block than one, profiles/r02x: this checks whether streams in one
process get the same overlap.)

usage: python tools/streams_exp.py [steps]
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


def part(dev, K, T, N, B, n_erase, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev, generator=g)
    esis = list(range(K, N))
    rep = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
    rqhip.encode_batch(src, K, T, esis, rep)
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    er, rl = [], []
    for _ in range(B):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in range(K, N) if e not in lost])
    bi = torch.tensor([b for b in range(B) for _ in rl[b]], device=dev)
    ri = torch.tensor([e - K for b in range(B) for e in rl[b]], device=dev)
    recv = rep.view(B, N - K, T)[bi, ri].contiguous()
    data = src.clone()
    db = rqhip.DecodeBatch(K, T, er, rl)
    st = db.run(data, recv)
    torch.cuda.synchronize()
    assert (st == 1).all() and torch.equal(data, src)
    return dict(src=src, rep=rep, recv=recv, data=data, db=db, esis=esis)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    K, T, N, B, n_erase = 1024, 1200, 1100, 1024, 55
    res = {}
    for S in (1, 2, 4):
        parts = [part(dev, K, T, N, B // S, n_erase, 100 + s) for s in range(S)]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        for _ in range(3):
            for p, st in zip(parts, streams):
                rqhip.encode_batch(p["src"], K, T, p["esis"], p["rep"], stream=st)
                p["db"].run_async(p["data"], p["recv"], stream=st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            for p, st in zip(parts, streams):
                rqhip.encode_batch(p["src"], K, T, p["esis"], p["rep"], stream=st)
                p["db"].run_async(p["data"], p["recv"], stream=st)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        res[S] = {"ms_per_step": round(dt * 1e3, 4), "GBps": round(B * K * T / dt / 1e9, 1)}
        print(S, res[S], flush=True)
        del parts
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
