"""Decode probe: small batches through rq.DecodeBatch, printing how recovered rows differ from the
source (which rows, which dword columns, XOR pattern).  A debugging aid for k_apply changes."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "rl-quic-raptor_amd"))
import rqhip as rq  # noqa: E402

gpu = torch.device("cuda", 0)
for K, T, N, nb, ne in [(5, 1100, 8, 4, 1), (5, 1100, 8, 4, 2), (10, 1200, 16, 4, 3), (100, 1200, 118, 4, 9),
                        (1024, 1200, 1100, 8, 55)]:
    g = torch.Generator(device=gpu).manual_seed(K)
    src = torch.randint(0, 256, (nb, K * T), dtype=torch.uint8, device=gpu, generator=g)
    esis = list(range(K, N))
    out = torch.empty((nb, len(esis) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    rng = np.random.default_rng(K)
    er, rl = [], []
    for _ in range(nb):
        lost = sorted(rng.choice(K, ne, replace=False).tolist())
        er.append(lost)
        rl.append(esis)
    R = N - K
    rep = out.view(nb, R, T).reshape(nb * R, T).contiguous()
    data = src.clone()
    d3 = data.view(nb, K, T)
    for b in range(nb):
        for i in er[b]:
            d3[b, i] = 0xA5
    st = rq.DecodeBatch(K, T, er, rl).run(data, rep)
    torch.cuda.synchronize()
    a = data.view(nb, K, T).cpu().numpy()
    s = src.view(nb, K, T).cpu().numpy()
    print("K=%d T=%d N=%d e=%d status=%s" % (K, T, N, ne, list(st)[:nb]))
    for b in range(nb):
        for i in er[b]:
            d = np.nonzero((a[b, i] != s[b, i]).reshape(-1, 4).any(1))[0]
            if len(d):
                x = a[b, i].view(np.uint32) ^ s[b, i].view(np.uint32)
                print("  block %d row %d: %d bad dwords, first %s last %d; xor[0:4]=%s" %
                      (b, i, len(d), d[:8].tolist(), d[-1], [hex(v) for v in x[d[:4]]]))
            else:
                print("  block %d row %d ok" % (b, i))
