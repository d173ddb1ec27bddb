"""Cost of stream event records between back-to-back column-program launches (K=1024 encode, 1024
blocks): wall time of 20 launches with no events, torch timing events, and HIP events created with
hipEventDisableSystemFence (ctypes)."""
import ctypes
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
K, T, N, B, n = 1024, 1200, 1100, 1024, 20
dev = torch.device("cuda:0")
src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev)
out = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
esis = list(range(K, N))
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)


def hip_events(flags, count):
    evs = []
    for _ in range(count):
        e = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)) == 0
        evs.append(e)
    return evs


def run(mode, per):
    evs = hip_events(0 if mode == "hip" else 0x20000000, per * n) if mode in ("hip", "hipnofence") else None
    tev = [torch.cuda.Event(enable_timing=True) for _ in range(per * n)] if mode == "torch" else None
    for _ in range(3):
        rqhip.encode_batch(src, K, T, esis, out, stream=st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        for j in range(per):
            if tev:
                tev[i * per + j].record(st)
            elif evs:
                hip.hipEventRecord(evs[i * per + j], sp)
        rqhip.encode_batch(src, K, T, esis, out, stream=st)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for mode, per in (("none", 0), ("torch", 1), ("torch", 3), ("hip", 1), ("hip", 3), ("hipnofence", 1), ("hipnofence", 3),
                  ("none", 0)):
    print("%-11s events/launch %d: %.4f ms per launch" % (mode, per, run(mode, per)), flush=True)
