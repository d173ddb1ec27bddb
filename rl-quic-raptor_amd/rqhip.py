"""Python binding of librqhip.so (ctypes), mirroring go/fec/raptorq_wrap.go.

The reference API (go/fec/raptorq_wrap.go:13-124) is reproduced name for name so the parity
tests read like the reference's own usage (go/cmd/raptorq_eval/main.go:199-222,
go/integrationtests/fec/raptorq_experiments_test.go:142-172):

    NewRaptorQEncoder(data, K, L) -> RaptorQEncoder   .GenSymbol(id) .BaseSymbolsNum()
    NewRaptorQDecoder(dataSize, L) -> RaptorQDecoder  .AddSymbol(id, data) .Decode()
    RaptorQEncodeBlock(data, N, K, L) -> [Packet]
    RaptorQDecodeBytes(recv, N, K, L, dataSize) -> (bytes, ok)

Go's (value, error) returns become Python exceptions (RaptorQError) carrying the same message.
The batch functions take torch CUDA tensors (device pointers) and drive the device-resident
hot path.  All compute happens in the HIP kernels of librqhip.so: if the library or a gfx950
device is missing the calls fail loudly -- there is no CPU fallback.
"""
import ctypes
import os
import subprocess
from dataclasses import dataclass
from pathlib import Path

_HERE = Path(__file__).resolve().parent
# RQHIP_LIB names an alternative build of the same library (tools/build_experiments.sh) for tuning runs
LIB_PATH = Path(os.environ["RQHIP_LIB"]).resolve() if os.environ.get("RQHIP_LIB") else _HERE / "build" / "librqhip.so"
# the experiments variant (RQHIP_* knobs; the pair and four-row-staging programs, the unshipped solvers)
EXP_LIB_PATH = _HERE / "build_exp" / "librqhip.so"
_lib = None
_exp_lib = None

RQ_OK = 0
RQ_ERR_SYMBOL_SIZE_ZERO = -1
RQ_ERR_K_TOO_BIG = -2
RQ_ERR_NOT_ENOUGH = -3
RQ_ERR_SYMBOL_SIZE = -4
RQ_ERR_BAD_ARG = -5
RQ_ERR_DEVICE = -6
RQ_ERR_UNSUPPORTED = -7
RQ_ERR_PLAN = -8

EXPORTED = (
    "rq_strerror", "rq_last_error", "rq_params", "rq_encoder_create", "rq_encoder_k",
    "rq_encoder_symbol_size", "rq_encoder_symbol", "rq_encoder_symbols", "rq_encoder_free",
    "rq_decoder_create", "rq_decoder_k", "rq_decoder_add", "rq_decoder_decode", "rq_decoder_free",
    "rq_encode_batch", "rq_decode_batch", "rq_decode_batch_async", "rq_encode_batch_host", "rq_decode_batch_host", "rq_device_count", "rq_set_device",
    "rq_debug_colprog_eval", "rq_debug_colprog_emulate", "rq_debug_colprog_assemble", "rq_debug_decode_margin",
    "rq_debug_apply_mode", "rq_debug_apply_sx", "rq_debug_apply_gi_asm", "rq_debug_solve_mode",
    "rq_decode_blocks_host", "rq_host_alloc", "rq_host_free", "rq_debug_colprog_passes",
    "rq_debug_shard_plan", "rq_debug_virtual_shards", "rq_debug_tuple", "rq_stream_release", "rq_shutdown",
    "rq_launch_timing", "rq_launch_time", "rq_debug_pair_emulate", "rq_debug_dma4_emulate", "rq_debug_decode_plan",
    "rq_debug_assemble", "rq_debug_colprog_bound", "rq_debug_cache_roundtrip", "rq_debug_gi_fits",
    "rq_debug_apply_gi_check", "rq_debug_gi_stream",
    "rq_tracker_create", "rq_tracker_k", "rq_tracker_add", "rq_tracker_held", "rq_tracker_free",
)


class RaptorQError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class EncodeDesc(ctypes.Structure):
    _fields_ = [("T", ctypes.c_uint32), ("K", ctypes.c_uint32), ("n_blocks", ctypes.c_uint32),
                ("src", ctypes.c_void_p), ("src_stride", ctypes.c_uint64), ("n_esi", ctypes.c_uint32),
                ("esi", ctypes.POINTER(ctypes.c_uint32)), ("out", ctypes.c_void_p),
                ("out_stride", ctypes.c_uint64), ("c_out", ctypes.c_void_p), ("c_stride", ctypes.c_uint64),
                ("stream", ctypes.c_void_p)]


class DecodeDesc(ctypes.Structure):
    _fields_ = [("T", ctypes.c_uint32), ("K", ctypes.c_uint32), ("n_blocks", ctypes.c_uint32),
                ("data", ctypes.c_void_p), ("data_stride", ctypes.c_uint64),
                ("n_erased", ctypes.POINTER(ctypes.c_uint32)), ("erased", ctypes.POINTER(ctypes.c_uint32)),
                ("n_repair", ctypes.POINTER(ctypes.c_uint32)), ("repair_esi", ctypes.POINTER(ctypes.c_uint32)),
                ("repair", ctypes.c_void_p), ("status", ctypes.POINTER(ctypes.c_int32)),
                ("stream", ctypes.c_void_p)]


class BlockIO(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("repair", ctypes.c_void_p), ("n_erased", ctypes.c_uint32),
                ("erased", ctypes.POINTER(ctypes.c_uint32)), ("n_repair", ctypes.c_uint32),
                ("repair_esi", ctypes.POINTER(ctypes.c_uint32)), ("status", ctypes.c_int32)]


def build():
    # RQHIP_BUILD_CMD replaces the make invocation (a test hook: tests/test_multi_rank.py counts builds)
    cmd = os.environ.get("RQHIP_BUILD_CMD")
    if cmd:
        subprocess.run(cmd, shell=True, check=True)
    else:
        subprocess.run(["make", "-s", "-C", str(_HERE), "-j8"], check=True)


def ensure_built():
    """Build librqhip.so if it is missing, under an exclusive file lock, without loading it (no GPU call).
    Returns True if this process ran the build.  Several processes that start at once (bench.py's ranks)
    then run one build between them, and none of them can dlopen a half-written library: the others wait
    on the lock and find the finished file."""
    if LIB_PATH.exists():
        return False
    import fcntl
    LIB_PATH.parent.mkdir(parents=True, exist_ok=True)
    with open(str(LIB_PATH) + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if LIB_PATH.exists():
                return False
            # hipcc cross-compiles gfx950 without a device; a failed build raises -- there is no CPU
            # fallback behind this library
            try:
                build()
            except (OSError, subprocess.CalledProcessError) as ex:
                raise RaptorQError(RQ_ERR_DEVICE, "librqhip.so could not be built: %s" % ex) from ex
            if not LIB_PATH.exists():
                raise RaptorQError(RQ_ERR_DEVICE, "librqhip.so not built (run `make -C rl-quic-raptor_amd`)")
            return True
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def lib():
    global _lib
    if _lib is None:
        ensure_built()
        _lib = _load(LIB_PATH)
    return _lib


def exp_lib():
    """The experiments library (tools/build_experiments.sh), built on first use; its own ctypes handle
    beside the release library's.  The pair / four-row-staging debug entry points work only here."""
    global _exp_lib
    if _exp_lib is None:
        if EXP_LIB_PATH == LIB_PATH:
            _exp_lib = lib()
            return _exp_lib
        if not EXP_LIB_PATH.exists():
            try:
                subprocess.run(["bash", str(_HERE.parent / "tools" / "build_experiments.sh")], check=True)
            except (OSError, subprocess.CalledProcessError) as ex:
                raise RaptorQError(RQ_ERR_DEVICE, "experiments library could not be built: %s" % ex) from ex
        _exp_lib = _load(EXP_LIB_PATH)
    return _exp_lib


def _load(path):
    """dlopen one build of librqhip.so and set its ctypes signatures."""
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7 (same soname as
    # /opt/rocm's).  Loaded first, torch's copy also serves librqhip.so's NEEDED entry; loaded after
    # librqhip.so, a second runtime initialises the device beside the first and the library's
    # hipGetDeviceCount then fails (seen on the GPU box, r03h).  The Python mirror exchanges device
    # tensors and streams with torch, so it loads torch's runtime first when torch is present.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(str(path))
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u16p = ctypes.POINTER(ctypes.c_uint16)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    ip = ctypes.POINTER(ctypes.c_int)
    vp = ctypes.c_void_p
    sig = {
        "rq_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "rq_last_error": ([], ctypes.c_char_p),
        "rq_params": ([ctypes.c_uint64, ctypes.c_uint32, u32p], ctypes.c_int),
        "rq_encoder_create": ([u8p, ctypes.c_size_t, ctypes.c_uint32, ip], vp),
        "rq_encoder_k": ([vp], ctypes.c_uint32),
        "rq_encoder_symbol_size": ([vp], ctypes.c_uint32),
        "rq_encoder_symbol": ([vp, ctypes.c_uint32, u8p], ctypes.c_int),
        "rq_encoder_symbols": ([vp, ctypes.c_uint32, ctypes.c_uint32, u8p], ctypes.c_int),
        "rq_encoder_free": ([vp], None),
        "rq_decoder_create": ([ctypes.c_uint64, ctypes.c_uint32, ip], vp),
        "rq_decoder_k": ([vp], ctypes.c_uint32),
        "rq_decoder_add": ([vp, ctypes.c_uint32, u8p, ctypes.c_size_t, ip], ctypes.c_int),
        "rq_decoder_decode": ([vp, u8p, ip], ctypes.c_int),
        "rq_decoder_free": ([vp], None),
        "rq_tracker_create": ([ctypes.c_uint64, ctypes.c_uint32, ip], vp),
        "rq_tracker_k": ([vp], ctypes.c_uint32),
        "rq_tracker_add": ([vp, ctypes.c_uint32, ctypes.c_size_t, ip], ctypes.c_int),
        "rq_tracker_held": ([vp], ctypes.c_uint32),
        "rq_tracker_free": ([vp], None),
        "rq_encode_batch": ([ctypes.POINTER(EncodeDesc)], ctypes.c_int),
        "rq_decode_batch": ([ctypes.POINTER(DecodeDesc)], ctypes.c_int),
        "rq_decode_batch_async": ([ctypes.POINTER(DecodeDesc)], ctypes.c_int),
        "rq_encode_batch_host": ([ctypes.POINTER(EncodeDesc), ctypes.c_uint32], ctypes.c_int),
        "rq_decode_batch_host": ([ctypes.POINTER(DecodeDesc), ctypes.c_uint32], ctypes.c_int),
        "rq_device_count": ([], ctypes.c_int),
        "rq_set_device": ([ctypes.c_int], ctypes.c_int),
        "rq_debug_colprog_eval": ([ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, vp, vp, u32p],
                                  ctypes.c_int),
        "rq_debug_colprog_emulate": ([ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, vp, vp, u32p, u32p,
                                      ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)],
                                     ctypes.c_int),
        "rq_debug_colprog_assemble": ([ctypes.c_uint32, u32p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)],
                                      ctypes.c_int),
        "rq_debug_decode_margin": ([ctypes.c_uint32], ctypes.c_uint32),
        "rq_debug_apply_mode": ([ctypes.c_uint32], ctypes.c_uint32),
        "rq_debug_apply_sx": ([ctypes.c_uint32], ctypes.c_uint32),
        "rq_debug_solve_mode": ([ctypes.c_uint32], ctypes.c_uint32),
        "rq_debug_gi_fits": ([ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
        "rq_debug_gi_stream": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_size_t, u32p], ctypes.c_int),
        "rq_debug_apply_gi_check": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p],
                                    ctypes.c_int),
        "rq_debug_apply_gi_asm": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p,
                                   ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rq_decode_blocks_host": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(BlockIO), ctypes.c_uint32,
                                   ctypes.c_uint32], ctypes.c_int),
        "rq_host_alloc": ([ctypes.c_size_t], vp),
        "rq_host_free": ([vp], None),
        "rq_debug_colprog_passes": ([ctypes.c_int], ctypes.c_int),
        "rq_debug_shard_plan": ([ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ip, u32p, u32p,
                                 ctypes.c_uint32], ctypes.c_int),
        "rq_debug_virtual_shards": ([ctypes.c_uint32], ctypes.c_uint32),
        "rq_debug_tuple": ([ctypes.c_uint32, ctypes.c_uint32, u32p], ctypes.c_int),
        "rq_stream_release": ([vp], ctypes.c_int),
        "rq_shutdown": ([], ctypes.c_int),
        "rq_launch_timing": ([ctypes.c_int], ctypes.c_int),
        "rq_launch_time": ([ctypes.POINTER(ctypes.c_double), u32p, ctypes.c_int], ctypes.c_int),
        "rq_debug_pair_emulate": ([ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, vp, vp, u32p, u32p,
                                   ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rq_debug_decode_plan": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p, u32p, ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_double), u32p], ctypes.c_int),
        "rq_debug_dma4_emulate": ([ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, vp, vp, ctypes.c_uint32,
                                   ctypes.c_uint32, u32p, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rq_debug_assemble": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rq_debug_cache_roundtrip": ([ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
        "rq_debug_colprog_bound": ([ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, vp, vp, ctypes.c_uint64,
                                    u32p], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


def launch_timing(enable):
    """rq_launch_timing: column-program launches of the current device record their own start/stop
    events (the dispatch's, no stream markers) while enabled."""
    _check(lib().rq_launch_timing(1 if enable else 0))


def launch_time(reset=True):
    """rq_launch_time: (summed kernel milliseconds, launch count) timed since the last reset."""
    ms = ctypes.c_double(0)
    n = ctypes.c_uint32(0)
    _check(lib().rq_launch_time(ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0))
    return ms.value, n.value


def _check(rc, L=None):
    if rc != RQ_OK:
        L = L or lib()
        detail = L.rq_last_error().decode() or L.rq_strerror(rc).decode()
        raise RaptorQError(rc, detail)
    return rc


def _buf(data):
    b = bytes(data)
    return b, (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")


# ------------------------------------------------------------------ parameters / column programs
PARAM_NAMES = ("K", "Kp", "J", "S", "H", "W", "L", "P", "P1", "U", "B")


def params(size, T):
    out = (ctypes.c_uint32 * 11)()
    _check(lib().rq_params(size, T, out))
    return dict(zip(PARAM_NAMES, list(out)))


COLPROG_STAT_NAMES = ("instructions", "valu", "src_loads", "out_stores", "spill_stores", "spill_loads", "accw",
                      "accr", "waits", "nops", "sync_reloads", "scratch_slots", "ir_nodes", "xtimes", "lds_stores",
                      "lds_loads", "lgkm_waits", "lds_slots")


def colprog_stats(K, esis=None, opts=None):
    """Host-only statistics of the column program for (K, output ESIs) (None: all L symbols)."""
    import numpy as np
    st = np.zeros(18, np.uint32)
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    e = np.asarray(esis if esis is not None else [0], np.uint32)
    o = np.asarray(list(opts or []) + [0] * (9 - len(opts or [])), np.uint32)
    _check(lib().rq_debug_colprog_emulate(K, 4, P32(e) if esis is not None else None, len(e), None, None, P32(o),
                                          P32(st), None, 0, None))
    return dict(zip(COLPROG_STAT_NAMES, (int(x) for x in st[:18])))


def colprog_emulate(K, T, esis, src, opts=None):
    """Run the allocated machine program on the host for one block (test infrastructure).  opts: up to 9
    allocation options (include/rqhip_debug.h), the rest 0 = default."""
    import numpy as np
    src = np.ascontiguousarray(src, np.uint8)
    e = np.asarray(esis, np.uint32)
    out = np.zeros((len(e), T), np.uint8)
    o = np.asarray(list(opts or []) + [0] * (9 - len(opts or [])), np.uint32)
    st = np.zeros(18, np.uint32)
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(lib().rq_debug_colprog_emulate(K, T, P32(e), len(e), src.ctypes.data, out.ctypes.data, P32(o), P32(st),
                                          None, 0, None))
    return out, dict(zip(COLPROG_STAT_NAMES, (int(x) for x in st[:18])))


def colprog_eval(K, T, esis, src):
    """Evaluate the column program's IR on the host for one block (test infrastructure)."""
    import numpy as np
    src = np.ascontiguousarray(src, np.uint8)
    e = np.asarray(esis, np.uint32)
    out = np.zeros((len(e), T), np.uint8)
    st = np.zeros(12, np.uint32)
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(lib().rq_debug_colprog_eval(K, T, P32(e), len(e), src.ctypes.data, out.ctypes.data, P32(st)))
    return out


def colprog_asm(K, esis, opts=None):
    """gfx950 assembly text of the column program for (K, output ESIs) (opts as colprog_emulate)."""
    import numpy as np
    e = np.asarray(esis, np.uint32)
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    o = np.asarray(list(opts or []) + [0] * (9 - len(opts or [])), np.uint32)
    n = ctypes.c_size_t(0)
    _check(lib().rq_debug_colprog_emulate(K, 4, P32(e), len(e), None, None, P32(o), None, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    _check(lib().rq_debug_colprog_emulate(K, 4, P32(e), len(e), None, None, P32(o), None, buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value].decode()


PAIR_STATS = ("a_ins", "a_valu", "a_loads", "a_agpr_moves", "a_ring_stores", "a_barriers", "b_ins", "b_valu",
              "b_ring_loads", "b_stores", "ring", "transfers", "handed", "lds_bytes", "a_dma4", "sched_4r")


def pair_emulate(K, T, esis, src=None, cfg=(0, 0, 0, 0, 0), assemble=False, L=None):
    """rq_debug_pair_emulate: the two-wave split of the (K, esis) program, run on the host over two items
    of one block (src: K*T bytes, or None for statistics only).  Returns (outputs or None, stats dict).
    The pair programs live in the experiments library (L defaults to exp_lib())."""
    L = L or exp_lib()
    import numpy as np
    e = np.asarray(esis, np.uint32)
    c = np.asarray(tuple(cfg) + (0,) * (5 - len(cfg)), np.uint32)
    st = np.zeros(16, np.uint32)
    out = None
    sp = op = None
    if src is not None:
        s = np.ascontiguousarray(np.frombuffer(bytes(src), np.uint8))
        out = np.zeros(len(esis) * T, np.uint8)
        sp, op = s.ctypes.data, out.ctypes.data
    n = ctypes.c_size_t(0)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(L.rq_debug_pair_emulate(K, T, P(e), len(e), sp, op, P(c), P(st), ctypes.byref(n) if assemble else None), L)
    d = dict(zip(PAIR_STATS, (int(x) for x in st)))
    d["code_bytes"] = n.value
    return (out.reshape(len(esis), T) if out is not None else None), d


DMA4_STATS = ("ins", "valu", "dma4", "scratch_slots", "tbl_slots", "lds_slots", "ins_plain", "sched_4r")


def dma4_emulate(K, T, esis, src=None, quads=8, la=0, assemble=False, L=None):
    """rq_debug_dma4_emulate: the single-wave program with four-row staging, run on the host over one
    item (src: K*T bytes, or None for statistics only).  Returns (outputs or None, stats dict).
    Four-row staging lives in the experiments library (L defaults to exp_lib())."""
    L = L or exp_lib()
    import numpy as np
    e = np.asarray(esis, np.uint32)
    st = np.zeros(8, np.uint32)
    out = None
    sp = op = None
    if src is not None:
        s = np.ascontiguousarray(np.frombuffer(bytes(src), np.uint8))
        out = np.zeros(len(esis) * T, np.uint8)
        sp, op = s.ctypes.data, out.ctypes.data
    n = ctypes.c_size_t(0)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(L.rq_debug_dma4_emulate(K, T, P(e), len(e), sp, op, quads, la, P(st), ctypes.byref(n) if assemble else None), L)
    d = dict(zip(DMA4_STATS, (int(x) for x in st)))
    d["code_bytes"] = n.value
    return (out.reshape(len(esis), T) if out is not None else None), d


def colprog_assemble(K, esis):
    """Assemble the column program in process (amd_comgr); returns the code object size."""
    import numpy as np
    e = np.asarray(esis, np.uint32)
    n = ctypes.c_size_t(0)
    _check(lib().rq_debug_colprog_assemble(K, e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(e),
                                           ctypes.byref(n)))
    return n.value


def assemble(text):
    """rq_debug_assemble: gfx950 assembly text through the engine's register check and amd_comgr;
    returns the code object size (RaptorQError with the check's message otherwise)."""
    b = text.encode()
    n = ctypes.c_size_t(0)
    _check(lib().rq_debug_assemble(b, len(b), ctypes.byref(n)))
    return n.value


def apply_gi_asm(kc=8, g=5, pdg=2, cpl=1, pack=0, assemble=True, sx=0):
    """rq_debug_apply_gi_asm: (assembly text, code object size or None) of the register-table apply kernel
    (sx = 1: the shape that reads precomputed syndromes)."""
    n = ctypes.c_size_t(0)
    cpl |= pack << 8 | sx << 9
    _check(lib().rq_debug_apply_gi_asm(kc, g, pdg, cpl, None, 0, ctypes.byref(n), None))
    buf = ctypes.create_string_buffer(n.value + 1)
    co = ctypes.c_size_t(0)
    _check(lib().rq_debug_apply_gi_asm(kc, g, pdg, cpl, buf, n.value + 1, None, ctypes.byref(co) if assemble else None))
    return buf.value.decode(), (co.value if assemble else None)


def solve_mode(mode):
    """rq_debug_solve_mode: 1 = in-place first solve (k_solve_ip), 0 = k_solve_pq; returns the previous mode."""
    return lib().rq_debug_solve_mode(mode)


def apply_mode(mode):
    """rq_debug_apply_mode: 1 = register-table apply, 0 = v_perm k_apply; returns the previous mode."""
    return lib().rq_debug_apply_mode(mode)


def apply_sx(on):
    """rq_debug_apply_sx: 1 = syndromes precomputed beside the first solver (the default), 0 = the apply
    XORs the received and r0 rows itself; returns the previous setting."""
    return lib().rq_debug_apply_sx(on)


def colprog_bound(K, T, esis, src, src_bytes):
    """rq_debug_colprog_bound: the (K, esis) program emulated on one block with its source buffer resource
    bounded at src_bytes; returns (outputs, row_end)."""
    import numpy as np
    src = np.ascontiguousarray(src, np.uint8)
    e = np.asarray(esis, np.uint32)
    out = np.zeros((len(e), T), np.uint8)
    re_ = ctypes.c_uint32(0)
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(lib().rq_debug_colprog_bound(K, T, P32(e), len(e), src.ctypes.data, out.ctypes.data, src_bytes,
                                        ctypes.byref(re_)))
    return out, re_.value


def shard_plan(device_mask, n_devices, n_blocks, virtual_shards=0):
    """[(device, first block, end block)] of a host-memory batch call (rq_debug_shard_plan)."""
    cap = 64
    dev = (ctypes.c_int * cap)()
    b0 = (ctypes.c_uint32 * cap)()
    b1 = (ctypes.c_uint32 * cap)()
    n = lib().rq_debug_shard_plan(device_mask, n_devices, n_blocks, virtual_shards, dev, b0, b1, cap)
    _check(min(n, 0))
    return [(dev[i], b0[i], b1[i]) for i in range(n)]


def device_count():
    return lib().rq_device_count()


# ------------------------------------------------------------------ go/fec mirror
@dataclass
class Packet:
    """fec.Packet (go/fec/packet_polar.go:87-90)."""
    Index: int
    Data: bytes


class RaptorQEncoder:
    """go/fec RaptorQEncoder (raptorq_wrap.go:13-18, 29-49)."""

    def __init__(self, handle, K, L):
        self._h = handle
        self.K = K
        self.L = L

    def GenSymbol(self, id):
        T = lib().rq_encoder_symbol_size(self._h)
        out = (ctypes.c_uint8 * T)()
        _check(lib().rq_encoder_symbol(self._h, id, out))
        return bytes(out)

    def GenSymbols(self, first, count):
        """Batch extension: symbols first..first+count-1 in one device launch."""
        T = lib().rq_encoder_symbol_size(self._h)
        out = (ctypes.c_uint8 * max(T * count, 1))()
        _check(lib().rq_encoder_symbols(self._h, first, count, out))
        b = bytes(out)
        return [b[i * T:(i + 1) * T] for i in range(count)]

    def BaseSymbolsNum(self):
        return lib().rq_encoder_k(self._h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rq_encoder_free(self._h)
            self._h = None


def NewRaptorQEncoder(data, K, L):
    if K <= 0 or L <= 0:
        raise RaptorQError(RQ_ERR_BAD_ARG, "bad K or L")
    b, arr = _buf(data)
    err = ctypes.c_int(0)
    h = lib().rq_encoder_create(arr, len(b), L, ctypes.byref(err))
    if not h:
        _check(err.value)
    return RaptorQEncoder(h, K, L)


class RaptorQDecoder:
    """go/fec RaptorQDecoder (raptorq_wrap.go:20-25, 52-74)."""

    def __init__(self, handle, K, L, size):
        self._h = handle
        self.K = K
        self.L = L
        self._size = size

    def AddSymbol(self, id, data):
        b, arr = _buf(data)
        can = ctypes.c_int(0)
        _check(lib().rq_decoder_add(self._h, id, arr, len(b), ctypes.byref(can)))
        return bool(can.value)

    def Decode(self):
        """(ok, bytes|None); raises RaptorQError('not enough symbols to decode')."""
        out = (ctypes.c_uint8 * max(self._size, 1))()
        ok = ctypes.c_int(0)
        _check(lib().rq_decoder_decode(self._h, out, ctypes.byref(ok)))
        if not ok.value:
            return False, None
        return True, bytes(out)[:self._size]

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rq_decoder_free(self._h)
            self._h = None


def NewRaptorQDecoder(dataSize, L):
    if dataSize < 0 or L <= 0:
        raise RaptorQError(RQ_ERR_BAD_ARG, "bad dataSize or L")
    err = ctypes.c_int(0)
    h = lib().rq_decoder_create(dataSize, L, ctypes.byref(err))
    if not h:
        _check(err.value)
    return RaptorQDecoder(h, lib().rq_decoder_k(h), L, dataSize)


class RaptorQTracker:
    """The shim's RaptorQTracker (go/fec/raptorq_rqhip.go): RaptorQDecoder.AddSymbol's bookkeeping and
    bool without the symbol bytes (rq_tracker_*), for a receiver that stages symbols itself."""

    def __init__(self, handle, K, L):
        self._h = handle
        self.K = K
        self.L = L

    def AddSymbol(self, id, data):
        can = ctypes.c_int(0)
        _check(lib().rq_tracker_add(self._h, id, len(data), ctypes.byref(can)))
        return bool(can.value)

    def Held(self):
        return lib().rq_tracker_held(self._h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rq_tracker_free(self._h)
            self._h = None


def NewRaptorQTracker(dataSize, L):
    if dataSize < 0 or L <= 0:
        raise RaptorQError(RQ_ERR_BAD_ARG, "bad dataSize or L")
    err = ctypes.c_int(0)
    h = lib().rq_tracker_create(dataSize, L, ctypes.byref(err))
    if not h:
        _check(err.value)
    return RaptorQTracker(h, lib().rq_tracker_k(h), L)


def RaptorQEncodeBlock(data, N, K, L):
    """raptorq_wrap.go:81-99 (GenSymbol 0..N-1; repairs generated in one launch)."""
    if N <= 0 or K <= 0 or L <= 0 or K > N:
        raise RaptorQError(RQ_ERR_BAD_ARG, "bad N/K/L")
    data = bytes(data)[:K * L]
    enc = NewRaptorQEncoder(data, K, L)
    return [Packet(i, s) for i, s in enumerate(enc.GenSymbols(0, N))]


def RaptorQDecodeBytes(recv, N, K, L, dataSize):
    """raptorq_wrap.go:103-124: ignores out-of-range indices and AddSymbol errors."""
    if K <= 0 or L <= 0 or dataSize < 0:
        return None, False
    try:
        dec = NewRaptorQDecoder(dataSize, L)
    except RaptorQError:
        return None, False
    for p in recv:
        if p.Index < 0 or p.Index >= N:
            continue
        try:
            dec.AddSymbol(p.Index, p.Data)
        except RaptorQError:
            pass
    try:
        ok, out = dec.Decode()
    except RaptorQError:
        return None, False
    if not ok:
        return None, False
    return out, True


# ------------------------------------------------------------------ device-resident batch API
def _stream_ptr(stream):
    if stream is None:
        return None
    return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


_esi_cache = {}


def _esi_array(esis):
    key = tuple(esis)
    arr = _esi_cache.get(key)
    if arr is None:
        if len(_esi_cache) > 64:
            _esi_cache.clear()
        arr = _esi_cache[key] = (ctypes.c_uint32 * max(len(esis), 1))(*esis)
    return arr


def encode_batch(src, K, T, esis, out, c_out=None, stream=None):
    """src: uint8 CUDA tensor [n_blocks, K*T] (contiguous rows); out: [n_blocks, len(esis)*T]."""
    d = EncodeDesc(T=T, K=K, n_blocks=src.shape[0], src=src.data_ptr(), src_stride=src.stride(0),
                   n_esi=len(esis), esi=_esi_array(esis), out=out.data_ptr() if out is not None else None,
                   out_stride=out.stride(0) if out is not None else 0,
                   c_out=c_out.data_ptr() if c_out is not None else None,
                   c_stride=c_out.stride(0) if c_out is not None else 0, stream=_stream_ptr(stream))
    _check(lib().rq_encode_batch(ctypes.byref(d)))


class DecodeBatch:
    """Host-side descriptor arrays for decode_batch, prepared once per erasure pattern."""

    def __init__(self, K, T, erased_lists, repair_lists):
        import numpy as np
        self.K, self.T = K, T
        self.n_blocks = len(erased_lists)
        self.n_erased = np.array([len(e) for e in erased_lists], np.uint32)
        self.erased = np.concatenate([np.asarray(e, np.uint32) for e in erased_lists] + [np.zeros(1, np.uint32)])
        self.n_repair = np.array([len(r) for r in repair_lists], np.uint32)
        self.repair_esi = np.concatenate([np.asarray(r, np.uint32) for r in repair_lists] + [np.zeros(1, np.uint32)])
        self.status = np.zeros(self.n_blocks, np.int32)
        self._pinned = None
        P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        self._ptrs = (P32(self.n_erased), P32(self.erased), P32(self.n_repair), P32(self.repair_esi))

    def _desc(self, data, repair, status, stream):
        ne, er, nr, re_ = self._ptrs
        return DecodeDesc(T=self.T, K=self.K, n_blocks=self.n_blocks, data=data.data_ptr(),
                          data_stride=data.stride(0), n_erased=ne, erased=er, n_repair=nr, repair_esi=re_,
                          repair=repair.data_ptr(), status=status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          stream=_stream_ptr(stream))

    def host_plan_us(self, iters=20):
        """rq_debug_decode_plan: mean host time (us) of one async call's host side on these arrays (no
        device work); returns (us, descriptor words)."""
        us = ctypes.c_double(0)
        n = ctypes.c_uint32(0)
        ne, er, nr, re_ = self._ptrs
        _check(lib().rq_debug_decode_plan(self.T, self.K, self.n_blocks, ne, er, nr, re_, iters, ctypes.byref(us),
                                          ctypes.byref(n)))
        return us.value, n.value

    def run(self, data, repair, stream=None):
        """rq_decode_batch: synchronous, returns the status array."""
        _check(lib().rq_decode_batch(ctypes.byref(self._desc(data, repair, self.status, stream))))
        return self.status

    def run_async(self, data, repair, stream=None):
        """rq_decode_batch_async: queues the decode and returns its pinned status array, valid once
        the stream has completed the work."""
        if self._pinned is None:
            import torch
            self._pinned = torch.zeros(self.n_blocks, dtype=torch.int32).pin_memory()
        st = self._pinned.numpy()
        _check(lib().rq_decode_batch_async(ctypes.byref(self._desc(data, repair, st, stream))))
        return st


# ------------------------------------------------------------------ host-memory batch API
def _host_rows(a):
    """(pointer, bytes between rows) of a 2-D uint8 host buffer: numpy array or CPU torch tensor
    (pinned with .pin_memory() for full PCIe rate)."""
    if hasattr(a, "data_ptr"):
        assert not a.is_cuda and a.element_size() == 1 and a.stride(1) == 1
        return a.data_ptr(), a.stride(0)
    assert a.dtype.itemsize == 1 and a.strides[1] == 1
    return a.ctypes.data, a.strides[0]


def encode_batch_host(src, K, T, esis, out, device_mask=0):
    """rq_encode_batch_host: src [n_blocks, >=K*T] and out [n_blocks, >=len(esis)*T] in host memory;
    blocks are split over the devices of device_mask (0: the current device).  Synchronous."""
    sp, ss = _host_rows(src)
    op, os_ = _host_rows(out)
    esi_arr = (ctypes.c_uint32 * max(len(esis), 1))(*esis)
    d = EncodeDesc(T=T, K=K, n_blocks=src.shape[0], src=sp, src_stride=ss, n_esi=len(esis), esi=esi_arr,
                   out=op, out_stride=os_, c_out=None, c_stride=0, stream=None)
    _check(lib().rq_encode_batch_host(ctypes.byref(d), ctypes.c_uint32(device_mask)))


def decode_batch_host(db, data, repair, device_mask=0):
    """rq_decode_batch_host with the descriptor arrays of a DecodeBatch: data [n_blocks, >=K*T] (host;
    recovered rows written in place), repair [n_rows, T] (host, repair_esi order).  Returns status."""
    P32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    dp, ds = _host_rows(data)
    rp, _ = _host_rows(repair)
    d = DecodeDesc(T=db.T, K=db.K, n_blocks=db.n_blocks, data=dp, data_stride=ds, n_erased=P32(db.n_erased),
                   erased=P32(db.erased), n_repair=P32(db.n_repair), repair_esi=P32(db.repair_esi), repair=rp,
                   status=db.status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), stream=None)
    _check(lib().rq_decode_batch_host(ctypes.byref(d), ctypes.c_uint32(device_mask)))
    return db.status


def decode_blocks_host(K, T, blocks, device_mask=0):
    """rq_decode_blocks_host: blocks = [(data, erased, repair_esi, repair_rows)] with data a writable
    host uint8 buffer of K*T bytes (received source rows in place) and repair_rows [n, T] (host,
    contiguous).  Recovered rows are written into each data buffer.  Returns the statuses."""
    import numpy as np
    arr = (BlockIO * max(len(blocks), 1))()
    keep = []
    for i, (data, erased, resi, rows) in enumerate(blocks):
        dp, _ = _host_rows(data.reshape(1, -1) if hasattr(data, "reshape") else data)
        er = np.asarray(erased, np.uint32)
        re_ = np.asarray(resi, np.uint32)
        rows = np.ascontiguousarray(rows, np.uint8) if not hasattr(rows, "data_ptr") else rows
        rp = rows.data_ptr() if hasattr(rows, "data_ptr") else rows.ctypes.data
        keep += [er, re_, rows]
        arr[i].data = dp
        arr[i].repair = rp
        arr[i].n_erased = len(er)
        arr[i].erased = er.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        arr[i].n_repair = len(re_)
        arr[i].repair_esi = re_.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _check(lib().rq_decode_blocks_host(K, T, arr, len(blocks), ctypes.c_uint32(device_mask)))
    return [arr[i].status for i in range(len(blocks))]
