"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol declared in
include/rqhip.h (the product ABI) and include/rqhip_debug.h (test-only diagnostics), reports parameters
and the reference's error strings, and fails loudly (no CPU fallback) when no device is present."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def header_functions(name="rqhip.h"):
    txt = (ROOT / "include" / name).read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rq_\w+)\s*\(", txt)))


def test_header_symbols_exported(rq):
    names = sorted(set(header_functions()) | set(header_functions("rqhip_debug.h")))
    assert len(names) >= 20
    L = rq.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(rq.EXPORTED) == names


def test_product_header_has_only_product_entries():
    """include/rqhip.h is what the cgo shim binds: the reference's replacements, the batch paths, device
    control and the bench's launch timing.  The diagnostics live in the test-only rqhip_debug.h."""
    prod, dbg = header_functions(), header_functions("rqhip_debug.h")
    assert not [n for n in prod if n.startswith("rq_debug_")], prod
    assert dbg and all(n.startswith("rq_debug_") for n in dbg), dbg
    assert not set(prod) & set(dbg)


def test_params_and_errors(rq):
    p = rq.params(1024 * 1200, 1200)
    assert (p["K"], p["Kp"], p["L"], p["P1"]) == (1024, 1032, 1101, 53)
    with pytest.raises(rq.RaptorQError, match="symbol size cannot be zero") as ei:
        rq.params(10, 0)
    assert ei.value.code == rq.RQ_ERR_SYMBOL_SIZE_ZERO
    with pytest.raises(rq.RaptorQError, match="k is too big"):
        rq.params(56404 * 8, 8)
    assert rq.lib().rq_strerror(rq.RQ_ERR_NOT_ENOUGH).decode() == "not enough symbols to decode"


def test_wrapper_argument_errors(rq):
    with pytest.raises(rq.RaptorQError, match="bad K or L"):
        rq.NewRaptorQEncoder(b"abc", 0, 10)
    with pytest.raises(rq.RaptorQError, match="bad dataSize or L"):
        rq.NewRaptorQDecoder(10, 0)
    with pytest.raises(rq.RaptorQError, match="bad N/K/L"):
        rq.RaptorQEncodeBlock(b"abc", 2, 3, 10)
    assert rq.RaptorQDecodeBytes([], 4, 0, 10, 5) == (None, False)


def test_decoder_host_state_without_device(rq):
    """AddSymbol bookkeeping is host-side (RQ/decoder.go:39-57): size check and the bool."""
    dec = rq.NewRaptorQDecoder(26 * 16, 16)
    assert dec.K == 26
    res = [dec.AddSymbol(i, bytes(16)) for i in range(30)]
    assert res == [False] * 25 + [True] * 5
    with pytest.raises(rq.RaptorQError, match="incorrect symbol size 15, should be 16"):
        dec.AddSymbol(31, bytes(15))
    dec2 = rq.NewRaptorQDecoder(26 * 16, 16)
    dec2.AddSymbol(0, bytes(16))
    with pytest.raises(rq.RaptorQError, match="not enough symbols to decode"):
        dec2.Decode()


def test_fast_path_needs_no_device(rq):
    """All K source symbols held: Decode returns them without a solve (RQ/decoder.go:69,134)."""
    data = bytes((i * 7) % 256 for i in range(5 * 20 - 3))
    dec = rq.NewRaptorQDecoder(len(data), 20)
    for i in range(5):
        chunk = data[i * 20:(i + 1) * 20]
        dec.AddSymbol(i, chunk + bytes(20 - len(chunk)))
    assert dec.Decode() == (True, data)


def test_device_paths_fail_loudly_without_gpu(rq):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; covered by the gpu tests")
    with pytest.raises(rq.RaptorQError) as ei:
        rq.NewRaptorQEncoder(b"x" * 100, 1, 10)
    assert ei.value.code == rq.RQ_ERR_DEVICE
    # the host-memory batch path has no CPU fallback either
    import numpy as np
    src, out = np.zeros((2, 64 * 64), np.uint8), np.zeros((2, 64), np.uint8)
    with pytest.raises(rq.RaptorQError) as ei:
        rq.encode_batch_host(src, 64, 64, [64], out)
    assert ei.value.code == rq.RQ_ERR_DEVICE
    db = rq.DecodeBatch(64, 64, [[1], [2]], [[64], [64]])
    with pytest.raises(rq.RaptorQError) as ei:
        rq.decode_batch_host(db, np.zeros((2, 64 * 64), np.uint8), np.zeros((2, 64), np.uint8))
    assert ei.value.code == rq.RQ_ERR_DEVICE


def _config3_batch(rq, n_blocks=1024, seed=1):
    K, N = 1024, 1100
    rng = np.random.default_rng(seed)
    el, rl = [], []
    for _ in range(n_blocks):
        lost = set(rng.choice(N, 55, replace=False).tolist())
        el.append(sorted(x for x in lost if x < K))
        rl.append([x for x in range(K, N) if x not in lost])
    return rq.DecodeBatch(K, 1200, el, rl)


def test_decode_host_plan_is_bounded(rq):
    """The host side of one async decode call on the config-3 descriptors (1 024 blocks, 55 of 1 100
    symbols lost each): argument checks, the union of the candidate repairs and the
    descriptor words, with nothing cached across calls.  The word count is the layout's; the time bound
    is loose here (a shared container CPU: ~90 us measured) -- the GPU box's figure is in DESIGN.md."""
    db = _config3_batch(rq)
    us, words = db.host_plan_us(20)
    nb = db.n_blocks
    n_er, n_rep = int(db.n_erased.sum()), int(db.n_repair.sum())
    assert words == nb + 2 * (nb + 1) + nb + n_er + n_rep + nb + 2 * nb
    assert 0 < us < 2000, us


def test_decode_host_plan_argument_errors(rq):
    """Out-of-range ESIs fail before any status is written (checked over the whole arrays at once)."""
    db = _config3_batch(rq, n_blocks=4)
    db.repair_esi[3] = 5  # a repair ESI below K
    with pytest.raises(rq.RaptorQError):
        db.host_plan_us(1)
    db = _config3_batch(rq, n_blocks=4)
    db.erased[0] = 1024  # an erased ESI at K
    with pytest.raises(rq.RaptorQError):
        db.host_plan_us(1)


def test_tracker_bookkeeping_matches_the_decoder(rq, oracle):
    """rq_tracker_* (the receiver's AddSymbol bookkeeping without the bytes) returns the
    bool the oracle decoder's add_symbol returns (RQ/decoder.go:47,57: K <= unique symbols held) on the same
    ESI sequence -- sources and repairs in random order with duplicates -- and refuses a wrong size with
    the decoder's message."""
    rng = np.random.default_rng(5)
    for K, T, N, loss in ((26, 16, 32, 0.15), (64, 40, 80, 0.10), (256, 8, 282, 0.05), (5, 12, 8, 0.3)):
        size = K * T - int(rng.integers(0, T))
        data = bytes(rng.integers(0, 256, size, dtype=np.uint8))
        enc = oracle.OracleEncoder(data, T)
        keep = [i for i in range(N) if rng.random() >= loss]
        seq = list(rng.permutation(keep)) + [int(x) for x in rng.choice(keep, 5)]  # + duplicates
        tr = rq.NewRaptorQTracker(size, T)
        dec = oracle.OracleDecoder(size, T)
        assert tr.K == (size + T - 1) // T
        got = [tr.AddSymbol(int(e), bytes(T)) for e in seq]
        want = [dec.add_symbol(int(e), enc.gen_symbol(int(e)).tobytes()) for e in seq]
        assert got == want, (K, seq)
        assert tr.Held() == len(set(int(e) for e in seq))
        with pytest.raises(rq.RaptorQError, match="incorrect symbol size %d, should be %d" % (T - 1, T)):
            tr.AddSymbol(0, bytes(T - 1))
    import ctypes
    err = ctypes.c_int(0)
    assert not rq.lib().rq_tracker_create(100, 0, ctypes.byref(err)) and err.value == rq.RQ_ERR_SYMBOL_SIZE_ZERO
    assert "symbol size cannot be zero" in rq.lib().rq_last_error().decode()
