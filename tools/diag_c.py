"""Diagnostics: the device's intermediate symbols C (encode_batch c_out) against the oracle, row by
row; prints per K the mismatching C rows (column index c of C) and which strip dwords differ."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import numpy as np, torch, rqhip, oracle

for K, T in [(5, 64), (26, 120), (64, 1200), (256, 1200), (1024, 1200)]:
    rng = np.random.default_rng(K)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    p = rqhip.params(len(data), T)
    ref = oracle.encode_C(data, T)
    src = torch.from_numpy(data.reshape(1, -1).copy()).cuda()
    cout = torch.zeros((1, p["L"] * T), dtype=torch.uint8, device="cuda")
    rqhip.encode_batch(src, K, T, [], None, c_out=cout)
    got = cout.cpu().numpy().reshape(p["L"], T)
    bad = np.nonzero((got != ref).any(axis=1))[0]
    W, S, H = p["W"], p["S"], p["H"]
    print(f"K={K} T={T} L={p['L']} W={W} S={S} H={H}: {len(bad)} bad rows", bad[:40].tolist())
    if len(bad):
        r = bad[0]
        dw = np.nonzero((got[r].view(np.uint32) != ref[r].view(np.uint32)))[0]
        print("   first bad row dwords:", dw[:64].tolist())
