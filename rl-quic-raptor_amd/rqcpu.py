"""ctypes binding of librqcpu.so: the CPU baseline (the engine's column-program algorithm on host
cores, csrc/rq_cpu.cpp).  Loaded by bench.py's cpu_baseline leg and the tests only; the product
(librqhip.so / rqhip.py) never calls it."""
import ctypes
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "build" / "librqcpu.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            subprocess.run(["make", "-s", "-C", str(_HERE), "-j8", "build/librqcpu.so"], check=True)
        L = ctypes.CDLL(str(LIB_PATH))
        u32p = ctypes.POINTER(ctypes.c_uint32)
        vp = ctypes.c_void_p
        L.rqc_encode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_uint64, u32p,
                                 ctypes.c_uint32, vp, ctypes.c_uint64, ctypes.c_int]
        L.rqc_decode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_uint64, u32p, u32p,
                                 u32p, u32p, vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        L.rqc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _p32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def encode(src, K, T, esis, threads=1):
    """src: uint8 [n_blocks, K*T] -> repairs uint8 [n_blocks, len(esis)*T]."""
    src = np.ascontiguousarray(src, np.uint8)
    e = np.asarray(esis, np.uint32)
    out = np.empty((src.shape[0], len(e) * T), np.uint8)
    rc = lib().rqc_encode(K, T, src.shape[0], src.ctypes.data, src.strides[0], _p32(e), len(e), out.ctypes.data,
                          out.strides[0], threads)
    if rc:
        raise RuntimeError("rqc_encode %d: %s" % (rc, lib().rqc_last_error().decode()))
    return out


def decode(data, K, T, erased_lists, repair_lists, repair_rows, threads=1):
    """In-place decode of data [n_blocks, K*T] (erased rows overwritten); repair_rows [n, T] in
    repair_lists order.  Returns the per-block status (1 ok, 0 rank-deficient, -3 not enough)."""
    assert data.dtype == np.uint8 and data.flags.c_contiguous
    nb = data.shape[0]
    ne = np.array([len(x) for x in erased_lists], np.uint32)
    er = np.concatenate([np.asarray(x, np.uint32) for x in erased_lists] + [np.zeros(1, np.uint32)])
    nr = np.array([len(x) for x in repair_lists], np.uint32)
    re_ = np.concatenate([np.asarray(x, np.uint32) for x in repair_lists] + [np.zeros(1, np.uint32)])
    rep = np.ascontiguousarray(repair_rows, np.uint8)
    st = np.zeros(nb, np.int32)
    rc = lib().rqc_decode(K, T, nb, data.ctypes.data, data.strides[0], _p32(ne), _p32(er), _p32(nr), _p32(re_),
                          rep.ctypes.data, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), threads)
    if rc:
        raise RuntimeError("rqc_decode %d: %s" % (rc, lib().rqc_last_error().decode()))
    return st
