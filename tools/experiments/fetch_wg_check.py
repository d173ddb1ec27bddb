"""Experiments library, RQHIP_WG=4 RQHIP_FETCH_LOG=1 (tests/test_gpu_experimental_programs.py): a config-3
decode (1 024 blocks K=1024 T=1200, 55 of 1 100 symbols erased per block) whose syndrome launch runs
four-wave workgroups and carries the descriptor fetch (the launch logs its shape on stderr); every block
must decode back to its source, sync and async.  Prints "ok" at the end."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "rl-quic-raptor_amd"))
import rqhip as rq  # noqa: E402


def main():
    gpu = torch.device("cuda:0")
    K, T, N, nb, ne = 1024, 1200, 1100, 1024, 55
    g = torch.Generator().manual_seed(77)
    src = torch.randint(0, 256, (nb, K * T), dtype=torch.uint8, generator=g).to(gpu)
    esis = list(range(K, N))
    out = torch.empty((nb, (N - K) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(77)
    er, rl, rows = [], [], []
    for b in range(nb):
        lost = set(rng.choice(N, ne, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in esis if e not in lost])
        rows.extend((b, e - K) for e in rl[-1])
    rep = out.view(nb, N - K, T)[torch.tensor([b for b, _ in rows], device=gpu),
                                 torch.tensor([r for _, r in rows], device=gpu)].contiguous()
    for mode in ("sync", "async"):
        data = src.clone()
        eb = torch.tensor([b for b in range(nb) for _ in er[b]], device=gpu, dtype=torch.long)
        ei = torch.tensor([i for b in range(nb) for i in er[b]], device=gpu, dtype=torch.long)
        data.view(nb, K, T)[eb, ei] = 0x5A
        db = rq.DecodeBatch(K, T, er, rl)
        st = db.run(data, rep) if mode == "sync" else db.run_async(data, rep)
        torch.cuda.synchronize()
        st = np.array(st)
        assert (st == 1).all(), (mode, np.unique(st))
        assert torch.equal(data, src), mode
        print(mode, "ok", flush=True)
    print("ok")


if __name__ == "__main__":
    main()
