"""Interpreter micro-benchmark: k_encode on synthetic wave programs (K=1024 geometry).
Each level gives every wave `ops` XOR ops of `nsrc` sources (independent slots); reports
cycles per level at 2.4 GHz from the kernel time of n_blocks blocks (10 strips each)."""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import numpy as np, rqhip

PAGE = 64
SD = 30  # strip width (dwords) k_encode picks for K=1024, T=1200; stream slot fields are slot*SD

NWAVES = int(os.environ.get("RQHIP_WAVES", 8))

def build(levels, ops, nsrc, nwaves=NWAVES, ty=0):
    streams = []
    for w in range(nwaves):
        segs = []
        for lv in range(levels):
            seg = [0]
            for o in range(ops):
                dA, dB = ((w * 64 + o * 2) % 900) * SD, ((w * 64 + o * 2 + 1) % 900) * SD
                op = [ty | 8 | 16 | (nsrc << 16), dA | (dB << 16)]
                for k in range(nsrc):
                    op.append((((lv * 7 + k * 13 + w) % 900 + 100) * SD) | ((((lv * 5 + k * 11 + w) % 900 + 100) * SD) << 16))
                    if ty == 1:
                        op.append(0x0203)
                if len(seg) + len(op) + 1 > PAGE:
                    seg.append(0); segs.append(seg); seg = [0]
                seg.extend(op); seg[0] += 1
            seg.append(1); segs.append(seg)
        s = []; prev = None
        for sg in segs:
            used = len(s) % PAGE
            if used and used + len(sg) > PAGE:
                s.extend([0] * (PAGE - used)); s[prev] |= 2
            s.extend(sg); prev = len(s) - 1
            if len(s) % PAGE == 0: s[prev] |= 2
        s.extend([0] * ((-len(s)) % PAGE))
        streams.append(s)
    off = []; words = []
    for s in streams:
        off.append(len(words)); words.extend(s)
    return np.array(words, np.uint32), np.array(off, np.uint32)

def run(levels, ops, nsrc, ty=0, blocks=256):
    w, o = build(levels, ops, nsrc, ty=ty)
    ms = ctypes.c_float(0)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    rqhip._check(rqhip.lib().rq_debug_run_wave_program(1024, 1200, P(w), len(w), P(o), levels, blocks, 5, ctypes.byref(ms)))
    rounds = blocks * 10 / 256
    cyc = ms.value * 1e-3 * 2.4e9 / rounds / max(levels, 1)
    return ms.value, cyc

if __name__ == "__main__":
    base = run(0, 0, 0)[0]
    print("empty program: %.3f ms" % base)
    cases = [(200, 0, 0, 0), (200, 1, 1, 0), (200, 2, 1, 0), (200, 1, 4, 0), (200, 1, 8, 0), (200, 2, 4, 0),
             (200, 4, 4, 0), (200, 1, 16, 0), (200, 1, 32, 0), (200, 4, 16, 0), (100, 1, 50, 0), (200, 1, 2, 1), (100, 1, 16, 1)]
    for (lv, ops, ns, ty) in cases:
        ms, cyc = run(lv, ops, ns, ty)
        print("levels=%d ops/wave=%d nsrc=%d type=%d: %.3f ms  ~%.0f cycles/level (net %.0f)" % (lv, ops, ns, ty, ms, cyc, (ms - base) * 1e-3 * 2.4e9 / (2560 / 256) / lv))
