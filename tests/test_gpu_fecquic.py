"""GPU: the fecquic-shaped loopback transfer (rl-quic-raptor_amd/fecquic, `fecquic loopback`) --
sender windows through rq_encode_batch_host, datagrams with the v1/v2 symbol header, receiver
ingest into pinned per-block staging, AddSymbol-bool bookkeeping, DDL, batched GPU decode through
rq_decode_blocks_host, offset writes and the SHA-256 check (go/fecquic/transfer.go:42-479,
rxbuf.go:279-567).  SURVEY.md sec. 8(f) ranks 1-3; BASELINE.json config 5's K x T stream shape."""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "rl-quic-raptor_amd" / "build" / "fecquic"


def run(tmp_path, size, *args, timeout=120):
    src = tmp_path / "in.bin"
    rng = np.random.default_rng(size)
    src.write_bytes(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
    out = tmp_path / "out.bin"
    cmd = [str(BIN), "loopback", "--file", str(src), "--out", str(out), "--timeout-s", "90"] + [str(a) for a in args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
    res = json.loads(line)
    assert r.returncode == 0 and res["ok"], (r.stdout[-2000:], r.stderr[-2000:])
    assert out.read_bytes() == src.read_bytes()
    return res


@pytest.mark.parametrize("K,T,mb", [(128, 1200, 6), (512, 256, 4), (512, 1200, 8), (2048, 1200, 20)])
def test_mixed_k_stream_5pct(gpu, rq, tmp_path, K, T, mb):
    """Config 5 shapes (N = K + K/10 + 8, 5 % sender loss): K > 255 travels in v2 headers; every
    block decodes on the GPU (held readiness: decode once K unique symbols are held).  The receive
    budget is raised from the reference's 10 MiB default (rxbuf.go:24-26), which a window of
    K=2048 blocks (2.5 MB each) exceeds: its repairs would be dropped and the blocks never decode."""
    N = K + K // 10 + 8
    res = run(tmp_path, mb * 2 ** 20 + 777, "--K", K, "--N", N, "--L", T, "--drop", 0.05, "--seed", K + T,
              "--ready", "held", "--max-blocks", 32 if K >= 2048 else 128, "--budget", 256 << 20)
    assert res["tx"]["dropped"] > 0 and res["rx"]["gpu_calls"] >= 1
    assert res["rx"]["dec_blocks"] == res["tx"]["blocks"]


def test_reference_readiness_over_udp(gpu, rq, tmp_path):
    """The reference's readiness rule (haveU counts AddSymbol true returns; decode at haveU >= K) over
    UDP on 127.0.0.1 with the file header on a TCP stream; N >= 2K - 1 so blocks become ready."""
    res = run(tmp_path, 3 * 2 ** 20 + 5, "--K", 26, "--N", 60, "--L", 1200, "--drop", 0.05, "--transport", "udp",
              "--ready", "ref", "--window", 16)
    assert res["rx"]["queued_ready"] >= res["tx"]["blocks"] - res["rx"]["queued_ddl"]
    assert res["tx"]["blocks"] == res["rx"]["dec_blocks"]


def test_v1_header_forced_default_shape(gpu, rq, tmp_path):
    """quicfec-client's default shape (K=26, N=32, L=1200) with v1 headers, as the reference sends."""
    res = run(tmp_path, 2 * 2 ** 20 + 3, "--K", 26, "--N", 32, "--L", 1200, "--drop", 0.03, "--header-version", 1,
              "--ready", "held")
    assert res["rx"]["dec_blocks"] == res["tx"]["blocks"]


EVAL = ROOT / "rl-quic-raptor_amd" / "build" / "raptorq_eval"


def test_raptorq_eval_experiment_b(gpu, rq, tmp_path):
    """raptorq_eval -exp B through the per-object C-ABI (GenSymbol timed too) and the batched host
    API: every generation decodes at p=0 (main.go:182-228 / raptorq_wrap.go calls)."""
    csv = tmp_path / "b.csv"
    r = subprocess.run([str(EVAL), "-exp", "B", "-schemes", "raptorq,raptorq-batch", "-N", "80", "-K", "64", "-L",
                        "1200", "-objMB", "1", "-trials", "2", "-p", "0,0.05", "-seed", "7", "-csv", str(csv)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("scheme=")]
    assert len(lines) == 4
    for ln in lines:
        if "p=0.0000" in ln:
            assert "ok=1.0000" in ln, ln
    rows = csv.read_text().strip().splitlines()
    assert rows[0].startswith("scheme,p,trials,ok_rate") and len(rows) == 5


def test_raptorq_eval_experiment_a(gpu, rq, tmp_path):
    data = tmp_path / "train.txt"
    data.write_bytes(np.random.default_rng(3).integers(0, 256, 200_003, dtype=np.uint8).tobytes())
    r = subprocess.run([str(EVAL), "-exp", "A", "-data", str(data), "-K", "26", "-L", "1500", "-repeats", "3"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("Experiment A: RaptorQ p=0"), (r.stdout, r.stderr)


def test_wire_symbols_match_oracle(gpu, rq, oracle, tmp_path):
    """The symbols the sender puts on the wire are the library's: every datagram of a small transfer
    (three K=26 blocks and a short final block, v1 headers, N=32, L=1200, 10 % sender loss) is parsed
    (16-byte FECHeader, go/internal/fecwire/header.go:15-59) and its payload compared with the oracle's
    GenSymbol(SymID) of that block's source bytes (RQ/encoder.go:36-41; the short block with the
    library K = ceil(bytes / L), raptorq_wrap.go:81-99).  The receiver's decode of those datagrams is
    checked by the SHA-256 of the transfer as in the other tests."""
    import struct
    K, N, L = 26, 32, 1200
    size = 3 * K * L + 5 * L + 17
    dump = tmp_path / "wire.bin"
    run(tmp_path, size, "--K", K, "--N", N, "--L", L, "--drop", 0.1, "--seed", 4, "--header-version", 1,
        "--ready", "held", "--dump", dump)
    src = (tmp_path / "in.bin").read_bytes()
    raw = dump.read_bytes()
    pos, seen, enc = 0, 0, {}
    while pos < len(raw):
        (n,) = struct.unpack_from("<I", raw, pos)
        dg = raw[pos + 4:pos + 4 + n]
        pos += 4 + n
        ver, scheme, bid, n_, k_, sym, flags, plen, _ = struct.unpack_from("<BBHBBBBII", dg, 0)
        assert ver == 1 and (n_, k_, plen) == (N, K, L)
        payload = dg[16:16 + plen]
        if bid not in enc:
            block = src[bid * K * L:(bid + 1) * K * L]
            enc[bid] = oracle.OracleEncoder(block, L)
        assert payload == enc[bid].gen_symbol(sym).tobytes(), (bid, sym)
        seen += 1
    assert len(enc) == 4 and seen > 0.8 * 4 * N
