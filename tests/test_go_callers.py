"""The Go-side fecquic callers of the batch API.

go/fecquic/rq_window.go (sender: one fec.EncodeWindow call per window of blocks) and rq_batchdec.go
(receiver: the decode workers batch ready blocks into fec.DecodeBlocks with fec.HostAlloc staging),
plus transfer.go.patch / rxbuf.go.patch that point the reference's sender loop
(go/fecquic/transfer.go:166-181) and decode workers (rxbuf.go:336-377) at them.  No Go toolchain exists
here or on the GPU box, so nothing is compiled; these checks keep the callers tied to the shim:
every fec.* call resolves to an exported function of go/fec/raptorq_rqhip.go with the same arity, the
patches apply to the reference files and keep its AddSymbol bookkeeping and DDL scheduler, and the
rxManager / rxBlock members the new code touches exist in the reference receiver.  CPU only; the
reference-file checks skip where /root/reference is absent."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SHIM = (ROOT / "go" / "fec" / "raptorq_rqhip.go").read_text()
NEW = {p.name: p.read_text() for p in (ROOT / "go" / "fecquic").glob("*.go")}
# the same sources without // comments (the call and type checks look at code only)
CODE = {n: re.sub(r"//[^\n]*", "", s) for n, s in NEW.items()}
PATCHES = {p.name: p.read_text() for p in (ROOT / "go" / "fecquic").glob("*.patch")}
REF = Path("/root/reference/go/fecquic")


def _args(src, start):
    """Top-level argument list text of the call whose '(' is at src[start - 1]."""
    i, depth = start, 1
    while depth:
        depth += {"(": 1, ")": -1}.get(src[i], 0)
        i += 1
    inner = src[start:i - 1]
    out, d, cur = [], 0, ""
    for ch in inner:
        d += {"(": 1, "[": 1, "{": 1, ")": -1, "]": -1, "}": -1}.get(ch, 0)
        if ch == "," and d == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def shim_funcs():
    """exported package-level function name -> parameter count (Go groups `a, b int` as two)."""
    funcs = {}
    for m in re.finditer(r"^func ([A-Z]\w*)\(", SHIM, flags=re.M):
        params = _args(SHIM, m.end())
        funcs[m.group(1)] = len(params)
    return funcs


def test_new_files_are_fecquic_sources():
    assert set(NEW) == {"rq_window.go", "rq_batchdec.go"}
    for name, src in NEW.items():
        assert "\npackage fecquic\n" in src, name
        assert '"github.com/quic-go/quic-go/fec"' in src, name


def test_every_fec_call_resolves_to_the_shim():
    funcs = shim_funcs()
    for need in ("EncodeWindow", "DecodeBlocks", "HostAlloc", "HostFree", "RaptorQEncodeBlock"):
        assert need in funcs, need
    seen = set()
    for name, src in CODE.items():
        for m in re.finditer(r"\bfec\.([A-Z]\w*)\(", src):
            fn = m.group(1)
            assert fn in funcs, "%s calls fec.%s, which raptorq_rqhip.go does not export" % (name, fn)
            n = len(_args(src, m.end()))
            assert n == funcs[fn], "%s: fec.%s with %d arguments, the shim takes %d" % (name, fn, n, funcs[fn])
            seen.add(fn)
        # the only fec type they name is the reference's Packet (packet_polar.go:87-90), by its two fields
        for t in re.findall(r"\bfec\.([A-Z]\w*)\b(?!\()", src):
            assert t == "Packet", t
        for lit in re.findall(r"fec\.Packet\{(.*?)\}", src):
            assert set(re.findall(r"(\w+):", lit)) <= {"Index", "Data"}, lit
    assert {"EncodeWindow", "DecodeBlocks", "HostAlloc", "HostFree", "RaptorQEncodeBlock"} <= seen


def test_patched_calls_match_the_new_functions():
    added = "\n".join(l[1:] for p in PATCHES.values() for l in p.splitlines() if l.startswith("+") and not l.startswith("+++"))
    m = re.search(r"newWindowReader\(", added)
    assert m and len(_args(added, m.end())) == 5
    assert re.search(r"^func newWindowReader\(r io.Reader, N, K, L int, deviceMask uint32\) \*windowReader", NEW["rq_window.go"], re.M)
    assert re.search(r"pkts, n, encErr := win\.next\(\)", added)
    assert re.search(r"^func \(w \*windowReader\) next\(\) \(\[\]fec\.Packet, int, error\)", NEW["rq_window.go"], re.M)
    assert "m.batchDecodeWorker()" in added
    assert re.search(r"^func \(m \*rxManager\) batchDecodeWorker\(\)", NEW["rq_batchdec.go"], re.M)


def test_patches_keep_the_receiver_bookkeeping():
    """The receiver patch only swaps the worker body: the classifier's AddSymbol bool bookkeeping (haveU,
    readiness at haveU >= K, rxbuf.go:406-493), the 50 ms DDL scheduler (:381-404) and the budget stay."""
    removed = "\n".join(l for l in PATCHES["rxbuf.go.patch"].splitlines() if l.startswith("-") and not l.startswith("---"))
    for keep in ("AddSymbol", "m.ddl", "haveU++", "budget"):
        assert keep not in removed, keep
    assert "b.dec.Decode()" in removed  # the per-object Decode is what the batch call replaces


@pytest.mark.skipif(not REF.exists() or shutil.which("patch") is None, reason="reference tree or patch(1) absent")
def test_patches_apply_to_the_reference(tmp_path):
    for f in ("transfer.go", "rxbuf.go"):
        shutil.copy(REF / f, tmp_path / f)
        text = PATCHES[f + ".patch"].replace("go/fecquic/", "")
        r = subprocess.run(["patch", "-p1", "-s", "-d", str(tmp_path)], input=text, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    assert "fec." not in (tmp_path / "transfer.go").read_text()  # the patch also drops the now-unused import


@pytest.mark.skipif(not REF.exists(), reason="reference tree absent")
def test_receiver_members_exist_in_the_reference():
    ref = (REF / "rxbuf.go").read_text()
    src = NEW["rq_batchdec.go"]
    for member in set(re.findall(r"\bm\.(\w+)", src)) - {"batchDecodeWorker", "decodeBatch", "decodeGroup"}:
        assert re.search(r"^\s+%s\s" % member, ref, re.M), "rxManager has no %s" % member
    for field in set(re.findall(r"\bb\.(\w+)", src)):
        assert re.search(r"^\s+(\w+, )*%s\b" % field, ref, re.M), "rxBlock has no %s" % field
    for field in set(re.findall(r"\bs\.(\w+)", src)):
        assert field in ("b", "n"), field  # slab{b []byte; n int}
    assert re.search(r"type writeTask struct \{\s*off\s+int64\s*data\s+\[\]byte", ref)
