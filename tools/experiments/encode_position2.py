"""Follow-up of encode_position.py: the bench's step shape [encode(src -> rep), decode(data)] repeated,
then the same with the encode writing two alternating output buffers, then with the encode reading the
decode's data buffer, 12 steps each, so a kernel trace compares the encode launch across the three."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402
import bench  # noqa: E402

K, T, N, B = 1024, 1200, 1100, 1024
dev = torch.device("cuda", 0)
src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev)
rep = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
rep2 = torch.empty_like(rep)
er, rl = bench.erasure_pattern(K, N, B, 55, 7)
rb = torch.tensor([b for b in range(B) for _ in rl[b]], device=dev, dtype=torch.long)
rr = torch.tensor([e - K for b in range(B) for e in rl[b]], device=dev, dtype=torch.long)
data = src.clone()
db = rqhip.DecodeBatch(K, T, er, rl)
esis = list(range(K, N))
s = torch.cuda.current_stream(dev)
rqhip.encode_batch(src, K, T, esis, rep, stream=s)
recv = rep.view(B, N - K, T)[rb, rr].contiguous()
for mode in range(3):
    for i in range(12):
        a = data if mode == 2 else src
        o = (rep2 if i % 2 else rep) if mode == 1 else rep
        rqhip.encode_batch(a, K, T, esis, o, stream=s)
        db.run_async(data, recv, stream=s)
    torch.cuda.synchronize()
print("done")
