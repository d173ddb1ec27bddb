"""Cross-item prefetch diagnosis: encode one K=1024 T=64 block (552 repairs) and the e=512 decode of
tests/test_gpu_apply.py::test_apply_stream_bound_falls_back, under RQHIP_CIP (experiments library)."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip as rq  # noqa: E402

if os.environ.get("RQHIP_LIB"):
    rq.LIB_PATH = Path(os.environ["RQHIP_LIB"])
from oracle import oracle as O  # noqa: E402

gpu = torch.device("cuda:0")
K, T = 1024, 64
for R, nb in ((552, 1), (552, 1), (552, 2), (600, 1), (76, 1), (300, 1), (1100, 1)):
    g = torch.Generator().manual_seed(R + nb)
    src = torch.randint(0, 256, (nb, K * T), dtype=torch.uint8, generator=g).to(gpu)
    out = torch.empty((nb, R * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, list(range(K, K + R)), out)
    torch.cuda.synchronize()
    for b in range(nb):
        enc = O.OracleEncoder(src[b].cpu().numpy().tobytes(), T)
        got = out[b].cpu().numpy().reshape(R, T)
        bad = [r for r in range(R) if not np.array_equal(got[r], enc.gen_symbol(K + r))]
        print("encode R=%d blocks=%d block %d: %d bad rows %s" % (R, nb, b, len(bad), bad[:8]), flush=True)
