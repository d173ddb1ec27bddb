"""Interpreter micro-benchmark: k_encode on synthetic wave programs (K=1024 geometry, sd=30).
Each level gives every wave `ops` XOR ops (statement pairs) of `nsrc` sources on independent
slots, in the stream format of rq_wave_format.hpp; reports cycles per level at 2.4 GHz from the
kernel time of n_blocks blocks (10 strips each, one workgroup per CU)."""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import numpy as np, rqhip

SD = 30  # strip width (dwords) k_encode picks for K=1024, T=1200
RB = SD * 4  # slot row bytes
NWAVES = int(os.environ.get("RQHIP_WAVES", 16))
OP_XOR, OP_END, BARRIER, ADVANCE = 0, 7, 1 << 8, 1 << 9
NO = 0xFFFFFFFF


def build(levels, ops, nsrc, nwaves=NWAVES):
    streams = []
    for w in range(nwaves):
        s = []  # groups

        def place(piece):
            if len(s) % 8 + len(piece) + 1 > 8:
                s.append([OP_END | ADVANCE, 0, 0, 0] * 2)
                while len(s) % 8:
                    s.append([0] * 8)
            s.extend(piece)
        for lv in range(levels):
            for o in range(ops):
                dA, dB = ((w * 64 + o * 2) % 900) * RB, ((w * 64 + o * 2 + 1) % 900) * RB
                ng = max(1, (nsrc + 3) // 4)
                hdr = OP_XOR | (ng << 16)
                piece = [[hdr, dA, NO, 0, hdr, dB, NO, 0]]
                for q in range(ng):
                    g = []
                    for half in (0, 1):
                        for j in range(4):
                            k = 4 * q + j
                            slot = ((lv * 7 + k * 13 + w + half * 5) % 900 + 100) if k < nsrc else 1000
                            g.append(slot * RB)
                    piece.append(g)
                place(piece)
            last = len(s) % 8 == 7
            s.append([OP_END | BARRIER | (ADVANCE if last else 0), 0, 0, 0] * 2)
        while len(s) % 8:
            s.append([0] * 8)
        streams.append([x for g in s for x in g])
    off, words = [], []
    for st in streams:
        off.append(len(words))
        words.extend(st)
    words.extend([0] * 192)
    return np.array(words, np.uint32), np.array(off, np.uint32)


def run(levels, ops, nsrc, blocks=256):
    w, o = build(levels, ops, nsrc)
    ms = ctypes.c_float(0)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    rqhip._check(rqhip.lib().rq_debug_run_wave_program(1024, 1200, P(w), len(w), P(o), levels, blocks, 5, ctypes.byref(ms)))
    return ms.value


if __name__ == "__main__":
    base = run(0, 0, 0)
    rounds = 256 * 10 / 256
    print("empty program: %.3f ms" % base)
    cases = [(200, 0, 0), (200, 1, 1), (200, 2, 1), (200, 1, 4), (200, 1, 8), (200, 2, 4), (200, 4, 4),
             (200, 1, 16), (200, 1, 24), (200, 4, 16), (100, 2, 24)]
    for (lv, ops, ns) in cases:
        ms = run(lv, ops, ns)
        net = (ms - base) * 1e-3 * 2.4e9 / rounds / lv
        print("levels=%d ops/wave=%d nsrc=%d: %.3f ms  net %.0f cycles/level" % (lv, ops, ns, ms, net))
