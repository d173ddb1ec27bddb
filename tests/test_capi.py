"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol declared in
include/rqhip.h, reports parameters and the reference's error strings, and fails loudly (no
CPU fallback) when no device is present."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def header_functions():
    txt = (ROOT / "include/rqhip.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rq_[a-z_]+)\s*\(", txt)))


def test_header_symbols_exported(rq):
    names = header_functions()
    assert len(names) >= 20
    L = rq.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(rq.EXPORTED) == names


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
