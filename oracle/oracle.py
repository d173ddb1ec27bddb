"""ctypes binding of the oracle (oracle/rq_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Never on the product path.  See rq_oracle.c for the parity status
("parity unpinned": no golden vectors exist in the reference).

The class `OracleDecoder` mirrors xssnick/raptorq's Decoder state machine
(RQ/decoder.go:23-134): AddSymbol's size check, de-duplication and its bool
("K <= unique symbols held", RQ/decoder.go:47,57), and Decode's three outcomes.
"""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = _HERE / "build" / "liboracle.so"
_lib = None

PARAM_NAMES = ("K", "Kp", "J", "S", "H", "W", "L", "P", "P1", "U", "B")


def build():
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not _LIB.exists():
            build()
        L = ctypes.CDLL(str(_LIB))
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.rqo_params.argtypes = [ctypes.c_uint64, ctypes.c_uint32, u32p]
        L.rqo_rand.argtypes = [ctypes.c_uint32] * 3
        L.rqo_rand.restype = ctypes.c_uint32
        L.rqo_tuple.argtypes = [u32p, ctypes.c_uint32, u32p]
        L.rqo_lt_cols.argtypes = [u32p, ctypes.c_uint32, u32p]
        L.rqo_solve.argtypes = [u32p, ctypes.c_uint32, ctypes.c_uint32, u32p, u8p, u8p]
        L.rqo_encode_C.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p]
        L.rqo_gen_symbol.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_uint32, u8p]
        L.rqo_lt_symbol.argtypes = [u32p, ctypes.c_uint32, u8p, ctypes.c_uint32, u8p]
        L.rqo_decode.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u32p, u8p, u8p]
        L.rqo_constraint_rows.argtypes = [u32p, u8p, u8p]
        L.rqo_gf_exp.argtypes = [ctypes.c_int]
        L.rqo_gf_exp.restype = ctypes.c_uint8
        L.rqo_gf_log.argtypes = [ctypes.c_int]
        L.rqo_gf_log.restype = ctypes.c_uint8
        L.rqo_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.rqo_gf_mul.restype = ctypes.c_uint8
        _lib = L
    return _lib


def _u8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _u32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def params(size, T):
    out = np.zeros(11, np.uint32)
    rc = lib().rqo_params(size, T, _u32(out))
    if rc == -1:
        raise ValueError("symbol size cannot be zero")
    if rc == -2:
        raise ValueError("k is too big")
    return dict(zip(PARAM_NAMES, (int(x) for x in out))), out


def rand(y, i, m):
    return lib().rqo_rand(y, i, m)


def tuple_(pvec, X):
    out = np.zeros(6, np.uint32)
    lib().rqo_tuple(_u32(pvec), X, _u32(out))
    return tuple(int(x) for x in out)


def lt_cols(pvec, X):
    out = np.zeros(64, np.uint32)
    n = lib().rqo_lt_cols(_u32(pvec), X, _u32(out))
    return [int(x) for x in out[:n]]


def solve(pvec, T, isis, syms):
    isis = np.ascontiguousarray(isis, np.uint32)
    syms = np.ascontiguousarray(syms, np.uint8)
    L = int(pvec[6])
    C = np.zeros((L, T), np.uint8)
    rc = lib().rqo_solve(_u32(pvec), T, len(isis), _u32(isis), _u8(syms), _u8(C))
    return (C if rc == 0 else None)


def encode_C(data, T):
    """Intermediate symbols C (L x T) of CreateEncoder(data)."""
    data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data, np.uint8)
    p, pvec = params(len(data), T)
    C = np.zeros((p["L"], T), np.uint8)
    buf = data if len(data) else np.zeros(1, np.uint8)
    rc = lib().rqo_encode_C(_u8(buf), len(data), T, _u8(C))
    if rc != 0:
        raise RuntimeError("oracle encode failed rc=%d" % rc)
    return C


def lt_symbol(pvec, T, C, isi):
    out = np.zeros(T, np.uint8)
    lib().rqo_lt_symbol(_u32(pvec), T, _u8(np.ascontiguousarray(C)), isi, _u8(out))
    return out


class OracleEncoder:
    """xssnick Encoder: CreateEncoder + GenSymbol (RQ/encoder.go:15-41)."""

    def __init__(self, data, T):
        self.data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        self.T = T
        self.p, self.pvec = params(len(self.data), T)
        self.C = encode_C(self.data, T)

    def gen_symbol(self, esi):
        K, Kp = self.p["K"], self.p["Kp"]
        if esi < K:
            out = np.zeros(self.T, np.uint8)
            chunk = self.data[esi * self.T:(esi + 1) * self.T]
            out[:len(chunk)] = chunk
            return out
        return lt_symbol(self.pvec, self.T, self.C, esi + Kp - K)


class OracleDecoder:
    """xssnick Decoder (RQ/decoder.go:23-134)."""

    def __init__(self, data_size, T):
        self.size = data_size
        self.T = T
        self.p, self.pvec = params(data_size, T)
        self.syms = {}

    def add_symbol(self, esi, data):
        if len(data) != self.T:
            raise ValueError("incorrect symbol size %d, should be %d" % (len(data), self.T))
        if esi not in self.syms:
            self.syms[esi] = np.frombuffer(bytes(data), np.uint8).copy()
        return self.p["K"] <= len(self.syms)

    def decode(self):
        """Returns (ok, bytes|None); raises on 'not enough symbols to decode'."""
        esis = np.array(sorted(self.syms), np.uint32)
        syms = (np.stack([self.syms[int(e)] for e in esis]) if len(esis)
                else np.zeros((1, self.T), np.uint8))
        out = np.zeros(max(self.size, 1), np.uint8)
        rc = lib().rqo_decode(self.size, self.T, len(esis), _u32(esis), _u8(syms), _u8(out))
        if rc == -3:
            raise RuntimeError("not enough symbols to decode")
        if rc == 1:
            return False, None
        if rc != 0:
            raise RuntimeError("oracle decode rc=%d" % rc)
        return True, out[:self.size].tobytes()


def constraint_rows(pvec):
    S, H, L = int(pvec[3]), int(pvec[4]), int(pvec[6])
    ldpc = np.zeros((S, L), np.uint8)
    hdpc = np.zeros((H, L), np.uint8)
    lib().rqo_constraint_rows(_u32(pvec), _u8(ldpc), _u8(hdpc))
    return ldpc, hdpc


def gf_tables():
    L_ = lib()
    return (np.array([L_.rqo_gf_exp(i) for i in range(512)], np.uint8),
            np.array([L_.rqo_gf_log(i) for i in range(256)], np.uint8))
