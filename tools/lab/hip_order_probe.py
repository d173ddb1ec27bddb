"""Probe (GPU box): which libamdhip64 a process maps and whether librqhip.so sees the device, when the
library is loaded before torch (raw ctypes) or after it.  python tools/lab/hip_order_probe.py raw|torch"""
import ctypes
import sys
from pathlib import Path

LIB = Path(__file__).resolve().parents[2] / "rl-quic-raptor_amd" / "build" / "librqhip.so"
if sys.argv[1] == "raw":
    L = ctypes.CDLL(str(LIB))
    import torch
    print("raw order: torch", torch.cuda.is_available(), "librqhip devices", L.rq_device_count(), flush=True)
else:
    import torch
    L = ctypes.CDLL(str(LIB))
    print("torch first: torch", torch.cuda.is_available(), "librqhip devices", L.rq_device_count(), flush=True)
maps = open("/proc/self/maps").read()
print(sorted(set(ln.split()[-1] for ln in maps.splitlines() if "amdhip64" in ln)))
