"""Encode-kernel phase ablation (timing only; outputs are wrong for dbg != 0).
Runs k_encode on B blocks with RQHIP_DBG bits given on the command line (set before import)."""
import os, sys, time, json
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import torch, rqhip
K, T, N = int(os.environ.get("K", 1024)), int(os.environ.get("T", 1200)), int(os.environ.get("N", 1100))
B = int(os.environ.get("B", 1024))
dev = torch.device("cuda:0")
src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev)
esis = list(range(K, N))
out = torch.empty((B, len(esis) * T), dtype=torch.uint8, device=dev)
for _ in range(2):
    rqhip.encode_batch(src, K, T, esis, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    rqhip.encode_batch(src, K, T, esis, out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(json.dumps({"dbg": os.environ.get("RQHIP_DBG", "0"), "K": K, "B": B, "ms": round(ms, 3),
                  "GBps": round(B * K * T / ms / 1e6, 1)}))
