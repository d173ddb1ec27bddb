"""fecquic harness pieces that need no GPU (libfecquic.so): the symbol header v1 (byte layout of
go/internal/fecwire/header.go:15-59) and v2 (wide N/K/SymID/BlockID), the file header
(go/fecquic/fileheader.go), and the receiver behaviour go/fecquic/rxbuf_test.go:9-100 pins (the
ingress ring never blocks, ingest stays fast when it is full, budget pressure drops repairs only),
plus the reference's readiness rule (rxbuf.go:472-486, :344-348)."""
import ctypes
import hashlib
import struct
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "rl-quic-raptor_amd" / "build" / "libfecquic.so"


@pytest.fixture(scope="module")
def fq(rq):  # rq: builds the package (librqhip.so and friends) on demand
    import subprocess
    if not LIB.exists():
        subprocess.run(["make", "-s", "-C", str(LIB.parent.parent), "-j8"], check=True)
    L = ctypes.CDLL(str(LIB))
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.fq_header_marshal.argtypes = [u32p, ctypes.c_char_p]
    L.fq_header_marshal.restype = ctypes.c_uint32
    L.fq_header_unmarshal.argtypes = [ctypes.c_char_p, ctypes.c_uint32, u32p]
    L.fq_header_unmarshal.restype = ctypes.c_uint32
    L.fq_file_header_unmarshal.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.c_char_p, u32p]
    L.fq_test_ring.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    L.fq_test_ingest_full.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    L.fq_test_budget.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64)]
    L.fq_test_ready.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
    L.fq_test_guards.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
    return L


def marshal(fq, fields):
    f = (ctypes.c_uint32 * 9)(*fields)
    out = ctypes.create_string_buffer(24)
    n = fq.fq_header_marshal(f, out)
    return out.raw[:n]


def unmarshal(fq, b):
    f = (ctypes.c_uint32 * 9)()
    n = fq.fq_header_unmarshal(b, len(b), f)
    return n, list(f)


def test_header_v1_layout(fq):
    """Version 1 is the reference's 16 bytes, little endian (header.go:29-43)."""
    b = marshal(fq, [1, 3, 0, 0x1234, 32, 26, 7, 1200, 0xDEADBEEF])
    assert b == struct.pack("<BBHBBBBII", 1, 3, 0x1234, 32, 26, 7, 0, 1200, 0xDEADBEEF)
    n, f = unmarshal(fq, b)
    assert n == 16 and f == [1, 3, 0, 0x1234, 32, 26, 7, 1200, 0xDEADBEEF]
    assert unmarshal(fq, b[:15])[0] == 0  # short (header.go:46)
    # fields that do not fit v1 are refused when v1 is forced
    assert marshal(fq, [1, 3, 0, 1, 300, 256, 0, 1200, 0]) == b""


def test_header_v2_wide_fields(fq):
    """Version 2 carries K > 255, N and SymID > 255 and a 32-bit block counter; version 0 = auto
    picks v1 whenever the block fits it, and a v2 parser still reads v1."""
    b = marshal(fq, [2, 3, 0, 70000, 2260, 2048, 2259, 1200, 0])
    assert len(b) == 24 and b[0] == 2
    assert unmarshal(fq, b) == (24, [2, 3, 0, 70000, 2260, 2048, 2259, 1200, 0])
    assert marshal(fq, [0, 3, 0, 5, 32, 26, 31, 1500, 0])[0] == 1
    big = marshal(fq, [0, 3, 0, 5, 1100, 1024, 1099, 1200, 0])
    assert big[0] == 2 and unmarshal(fq, big)[1][4:7] == [1100, 1024, 1099]
    assert unmarshal(fq, big[:23])[0] == 0


def test_file_header(fq):
    sha = hashlib.sha256(b"payload").digest()
    b = b"QFEC" + struct.pack("<HQ", 1, 123456789) + sha + struct.pack("<I", 1200) + bytes(8)
    size, chunk = ctypes.c_uint64(), ctypes.c_uint32()
    out = ctypes.create_string_buffer(32)
    assert fq.fq_file_header_unmarshal(b, len(b), ctypes.byref(size), out, ctypes.byref(chunk)) == 0
    assert (size.value, out.raw, chunk.value) == (123456789, sha, 1200)
    assert fq.fq_file_header_unmarshal(b[:57], 57, ctypes.byref(size), out, ctypes.byref(chunk)) == -1
    assert fq.fq_file_header_unmarshal(b"QFEX" + b[4:], 58, ctypes.byref(size), out, ctypes.byref(chunk)) == -2
    bad = b[:4] + struct.pack("<H", 2) + b[6:]
    assert fq.fq_file_header_unmarshal(bad, 58, ctypes.byref(size), out, ctypes.byref(chunk)) == -3


def test_ring_never_blocks(fq):
    """TestMPSCRingTryPushNonBlocking: pushes on a full ring fail at once; the consumer then sees
    the items in order."""
    ns = ctypes.c_uint64()
    assert fq.fq_test_ring(8, 2000, ctypes.byref(ns)) == 0
    assert ns.value < 200_000


def test_ingest_fast_when_ring_full(fq, tmp_path):
    """TestRXIngestNonBlockingWhenRingFull: with no consumer, ingests past the ring's 8 slots are
    dropped quickly."""
    assert fq.fq_test_ingest_full(str(tmp_path).encode(), 500) <= 50


def test_budget_drops_repairs_only(fq, tmp_path):
    """TestRXBudgetDropsRepairs: 3 KiB budget, 6 systematic symbols then 2000 repairs -- some repairs
    dropped, no systematic symbol.  Then the same flood in bursts the classifier keeps up with, so
    the drops come from the budget rule itself (rxbuf.go:425-431)."""
    out = (ctypes.c_int64 * 3)()
    assert fq.fq_test_budget(str(tmp_path).encode(), 0, out) == 0
    assert out[0] > 0 and out[1] == 0
    assert fq.fq_test_budget(str(tmp_path).encode(), 100, out) == 0
    assert out[0] > 0 and out[2] > 0 and out[1] == 0


def test_readiness_rules(fq, tmp_path):
    """K=26, N=32 with every symbol delivered: AddSymbol returns true only from the 26th unique
    symbol on (RQ/decoder.go:47,57), so the reference's haveU reaches 7 < K -- the block is never
    decoded, DDL or not (rxbuf.go:344-348).  The held rule decodes it at once (all sources present:
    the fast path, no device work)."""
    out = (ctypes.c_int64 * 4)()
    assert fq.fq_test_ready(str(tmp_path).encode(), 0, 120, out) == 0
    assert out[0] == 0 and out[1] >= 2 and out[2] == 32 and out[3] == 0
    assert fq.fq_test_ready(str(tmp_path).encode(), 1, 60, out) == 0
    assert out[0] == 1 and out[2] >= 26 and out[3] == 1


def test_ingest_guards(fq, tmp_path):
    """Untrusted headers: a block whose header claims more source rows than the staging slot holds
    (slots are sized from the first header), or N < K, is dropped before anything is copied; a late
    symbol of a block already written is dropped rather than re-creating the block in a fresh slot."""
    out = (ctypes.c_int64 * 4)()
    assert fq.fq_test_guards(str(tmp_path).encode(), out) == 0
    assert out[0] == 0 and out[1] == 1   # late repair of the written block: dropped, counted
    assert out[2] >= 2 and out[3] == 0   # oversized and short-N headers: dropped at staging
