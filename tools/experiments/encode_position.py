"""Why the encode launch of the config-3 step takes ~4 % longer than the decode's syndrome launch of the
same program: a step of encode(src), encode(src), encode(data), decode(data), repeated, so a kernel trace
shows the program's time by position (after the apply, after itself) and by source buffer (src, or the
decode's data buffer that the apply just wrote)."""
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
for _ in range(12):
    rqhip.encode_batch(src, K, T, esis, rep, stream=s)
    rqhip.encode_batch(src, K, T, esis, rep, stream=s)
    rqhip.encode_batch(data, K, T, esis, rep2, stream=s)
    db.run_async(data, recv, stream=s)
torch.cuda.synchronize()
print("done")
