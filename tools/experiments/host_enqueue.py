"""Config-3 step cost of the timing events and the host enqueue: wall ms per step of the bench's timed
loop with its three timing events per step, with one, and with none; and the pure host time of one
encode_batch / DecodeBatch.run_async call on an idle device (synchronized before each call, so the
staging double buffer never waits)."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402
import bench  # noqa: E402

K, T, N, B, S = 1024, 1200, 1100, 1024, 30
dev = torch.device("cuda", 0)
src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev)
rep = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
er, rl = bench.erasure_pattern(K, N, B, 55, 7)
rb = torch.tensor([b for b in range(B) for _ in rl[b]], device=dev, dtype=torch.long)
rr = torch.tensor([e - K for b in range(B) for e in rl[b]], device=dev, dtype=torch.long)
data = src.clone()
db = rqhip.DecodeBatch(K, T, er, rl)
esis = list(range(K, N))
stream = torch.cuda.current_stream(dev)
rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
recv = rep.view(B, N - K, T)[rb, rr].contiguous()


def loop(n_ev):
    for _ in range(3):
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        db.run_async(data, recv, stream=stream)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(S)]
    t0 = time.perf_counter()
    for s in range(S):
        if n_ev >= 1:
            ev[s][0].record(stream)
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        if n_ev >= 3:
            ev[s][1].record(stream)
        db.run_async(data, recv, stream=stream)
        if n_ev >= 3:
            ev[s][2].record(stream)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / S


for n_ev in (3, 0, 1, 3, 0):
    print("events per step %d: %.4f ms per step" % (n_ev, loop(n_ev)), flush=True)
he, hd = [], []
for _ in range(10):
    torch.cuda.synchronize()
    a = time.perf_counter()
    rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    db.run_async(data, recv, stream=stream)
    d = time.perf_counter()
    he.append(b - a)
    hd.append(d - c)
print("host ms per call on an idle device: encode %.3f, decode %.3f (min %.3f)" %
      (1e3 * sum(he) / 10, 1e3 * sum(hd) / 10, 1e3 * min(hd)))
