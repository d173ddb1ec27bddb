"""The Go-side fecquic callers of the batch API.

go/fecquic/rq_window.go (sender: one fec.EncodeWindow call per window of blocks), rq_stage.go (ingest
copies each symbol once, into its block's pinned staging; the classifier's AddSymbol is the
bookkeeping-only fec.RaptorQTracker) and rq_batchdec.go (the decode workers batch ready blocks into
fec.DecodeBlocks on the staged rows), plus transfer.go.patch / rxbuf.go.patch that point the reference's
sender loop (go/fecquic/transfer.go:166-268), receive loops (:380-456), classifier, ingest
(rxbuf.go:406-538) and decode workers (:336-377) at them, and go/internal/fecwire/header.go.patch (the
24-byte version-2 symbol header, K >= 256).  No Go toolchain exists
here or on the GPU box, so nothing is compiled; these checks keep the callers tied to the shim:
every fec.* call resolves to an exported function of go/fec/raptorq_rqhip.go with the same arity, the
patches apply to the reference files and keep its AddSymbol bookkeeping and DDL scheduler, and the
rxManager / rxBlock members the new code touches exist in the reference receiver.  CPU only; the
reference-file checks skip where /root/reference is absent."""
import ctypes
import json
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
HDR_PATCH = (ROOT / "go" / "internal" / "fecwire" / "header.go.patch").read_text()
REF = Path("/root/reference/go/fecquic")
REF_HDR = Path("/root/reference/go/internal/fecwire/header.go")


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
    assert set(NEW) == {"rq_window.go", "rq_batchdec.go", "rq_stage.go"}
    for name, src in NEW.items():
        assert "\npackage fecquic\n" in src, name
        assert '"github.com/quic-go/quic-go/fec"' in src, name


def test_every_fec_call_resolves_to_the_shim():
    funcs = shim_funcs()
    for need in ("EncodeWindow", "DecodeBlocks", "HostAlloc", "HostFree", "RaptorQEncodeBlock", "NewRaptorQTracker"):
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


def _patched(tmp_path):
    """The reference's transfer.go, rxbuf.go and internal/fecwire/header.go with this repo's patches."""
    for f in ("transfer.go", "rxbuf.go"):
        shutil.copy(REF / f, tmp_path / f)
        text = PATCHES[f + ".patch"].replace("go/fecquic/", "")
        r = subprocess.run(["patch", "-p1", "-s", "-d", str(tmp_path)], input=text, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    shutil.copy(REF_HDR, tmp_path / "header.go")
    r = subprocess.run(["patch", "-p1", "-s", "-d", str(tmp_path)], input=HDR_PATCH.replace("go/internal/fecwire/", ""),
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return {f: (tmp_path / f).read_text() for f in ("transfer.go", "rxbuf.go", "header.go")}


NEED_REF = pytest.mark.skipif(not REF.exists() or shutil.which("patch") is None, reason="reference tree or patch(1) absent")


@NEED_REF
def test_patches_apply_to_the_reference(tmp_path):
    src = _patched(tmp_path)
    # the sender's per-block fec.RaptorQEncodeBlock call is gone (rq_window.go makes it for the last block)
    assert "fec.RaptorQEncodeBlock" not in src["transfer.go"]
    # the receiver: the tracker in place of the decoder, ingest staging, the staging freed at the end
    rx = src["rxbuf.go"]
    assert "fec.NewRaptorQDecoder" not in rx and "fec.NewRaptorQTracker(s.DataSize, s.L)" in rx
    assert re.search(r"dec\s+\*fec\.RaptorQTracker", rx)
    assert "return m.stageIngest(blockID, esi, N, K, L, data, dataSize)" in rx
    assert "m.slabs.Get()" not in rx and "m.slabs.Put(" not in rx
    assert "m.stage = newStageTable()" in rx and "m.stage.close()" in rx
    assert rx.count("m.unstage(s)") == 3


@NEED_REF
def test_receiver_members_exist_in_the_reference(tmp_path):
    """Every rxManager / rxBlock / Symbol member the new files touch exists in the (patched) reference
    receiver; the only member the patch adds is the staging table."""
    ref = _patched(tmp_path)["rxbuf.go"]
    orig = (REF / "rxbuf.go").read_text()
    own = {"batchDecodeWorker", "decodeBatch", "decodeGroup", "stageIngest", "unstage", "stage"}
    for name in ("rq_batchdec.go", "rq_stage.go"):
        src = CODE[name]
        for member in set(re.findall(r"\bm\.(\w+)", src)) - own:
            assert re.search(r"^\s+%s\s" % member, orig, re.M), "rxManager has no %s" % member
    assert re.search(r"^\s+stage \*stageTable", ref, re.M) and not re.search(r"^\s+stage\s", orig, re.M)
    for field in set(re.findall(r"\bb\.(\w+)", CODE["rq_batchdec.go"])):
        assert re.search(r"^\s+(\w+, )*%s\b" % field, orig, re.M), "rxBlock has no %s" % field
    for field in set(re.findall(r"\bs\.(\w+)", CODE["rq_batchdec.go"])):
        assert field in ("b", "n"), field  # slab{b []byte; n int}
    # the Symbol literal of stageIngest names the reference's Symbol fields only
    lit = re.search(r"s := Symbol\{(.*?)\n\t\}", CODE["rq_stage.go"], re.S).group(1)
    sym = orig[orig.index("type Symbol struct {"):orig.index("}", orig.index("type Symbol struct {"))]
    for f in re.findall(r"^\t\t(\w+):", lit, re.M):
        assert re.search(r"\b%s\b" % f, sym), f


def test_receiver_stages_each_symbol_once():
    """rq_batchdec.go passes the staged rows to fec.DecodeBlocks as they lie (no slab -> staging copy);
    the only copy left in the decode path is the gather for a block with a hole among its repair rows."""
    bd = CODE["rq_batchdec.go"]
    assert "fec.HostAlloc" not in bd and "s.b[:s.n]" not in bd and "m.slabs" not in bd
    assert "sb.repair = bs.buf[kl*L : (kl+len(reps))*L]" in bd and "data: bs.buf[:kl*L]" in bd
    assert bd.count("copy(") == 1 and "if contiguous {" in bd
    st = CODE["rq_stage.go"]
    assert st.count("copy(") == 1  # ingest's one copy, into the staging row
    assert "groupKey{libraryK(b.dataSize, b.L), b.L}" in bd  # a DecodeBlocks call shares K and L


# ---- the version-2 symbol header
# golden headers (tests/golden/make_fec_header.py: struct-packed from the documented layouts, checked
# against the C++ marshal when written)
GOLDEN = json.loads((ROOT / "tests" / "golden" / "fec_header.json").read_text())


@pytest.fixture(scope="module")
def fq_lib(rq):  # rq: builds the package (libfecquic.so with it) on demand
    lib = ROOT / "rl-quic-raptor_amd" / "build" / "libfecquic.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(lib.parent.parent), "-j8"], check=True)
    L = ctypes.CDLL(str(lib))
    L.fq_header_marshal.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p]
    L.fq_header_marshal.restype = ctypes.c_uint32
    L.fq_header_unmarshal.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.fq_header_unmarshal.restype = ctypes.c_uint32
    return L


def _cpp_marshal(L, fields9):
    f = (ctypes.c_uint32 * 9)(*fields9)
    out = ctypes.create_string_buffer(24)
    n = L.fq_header_marshal(f, out)
    return out.raw[:n]


def _go_marshal(header_go, fields, version):
    """Interprets the patched header.go's MarshalBinary statements for one header version: every
    `b[i] = ...` and `binary.LittleEndian.PutUintNN(b[a:b], ...)` line of that branch, in order."""
    body = header_go[header_go.index("func (h *FECHeader) MarshalBinary"):header_go.index("func (h *FECHeader) UnmarshalBinary")]
    v2, v1 = body.split("\tb[0] = h.Version", 1)
    code = v2[v2.index("if h.Version == 2 {"):] if version == 2 else "b[0] = h.Version" + v1
    out = bytearray(24)
    consts = {"HeaderV2Len": 24}

    def val(expr):
        expr = expr.strip()
        m = re.fullmatch(r"(?:uint\d+\()?h\.(\w+)\)?", expr)
        if m:
            return fields[m.group(1)]
        if expr in consts:
            return consts[expr]
        return int(expr, 0)

    n = 0
    for line in code.splitlines():
        line = line.strip()
        m = re.fullmatch(r"b\[(\d+)\] = (.+)", line)
        if m:
            out[int(m.group(1))] = val(m.group(2)) & 0xFF
            n = max(n, int(m.group(1)) + 1)
            continue
        m = re.fullmatch(r"binary\.LittleEndian\.PutUint(16|32)\(b\[(\d+):(\d+)\], (.+)\)", line)
        if m:
            w, a, b = int(m.group(1)) // 8, int(m.group(2)), int(m.group(3))
            assert b - a == w, line
            out[a:b] = (val(m.group(4)) & ((1 << (8 * w)) - 1)).to_bytes(w, "little")
            n = max(n, b)
    return bytes(out[:n])


@NEED_REF
def test_header_v2_go_matches_cpp_golden(tmp_path, fq_lib):
    """The Go header (patched header.go) and the C++ harness (fq_wire.hpp) write the same bytes for the
    golden headers of tests/golden/fec_header.json, in both versions; version 1 is the reference's
    16-byte layout (header.go:29-43)."""
    hdr = _patched(tmp_path)["header.go"]
    # field widths of the Go struct: the ones fq_wire.hpp uses
    for f, t in (("BlockID", "uint32"), ("N", "uint32"), ("K", "uint32"), ("SymID", "uint32"), ("Flags", "uint16"),
                 ("PayloadLen", "uint32"), ("SeedOrIdx", "uint32"), ("Version", "uint8"), ("Scheme", "uint8")):
        assert re.search(r"^\s+%s\s+%s\b" % (f, t), hdr, re.M), f
    assert re.search(r"const HeaderLen = 1 \+ 1 \+ 2 \+ 1 \+ 1 \+ 1 \+ 1 \+ 4 \+ 4", hdr)
    assert "const HeaderV2Len = 24" in hdr
    for g in GOLDEN:
        fields = g["fields"]
        want = bytes.fromhex(g["bytes"])
        assert _go_marshal(hdr, fields, g["version"]) == want, g
        order = ("Version", "Scheme", "Flags", "BlockID", "N", "K", "SymID", "PayloadLen", "SeedOrIdx")
        assert _cpp_marshal(fq_lib, [g["version"]] + [fields[k] for k in order[1:]]) == want, g
        # and the C++ side reads it back (the Go UnmarshalBinary offsets are checked below)
        f = (ctypes.c_uint32 * 9)()
        assert fq_lib.fq_header_unmarshal(want, len(want), f) == len(want)
        assert list(f)[:8] == [fields[k] for k in order[:8]], g
    # UnmarshalBinary reads each field at the offset MarshalBinary wrote it (both versions)
    un = hdr[hdr.index("func (h *FECHeader) UnmarshalBinary"):]
    mar = hdr[hdr.index("func (h *FECHeader) MarshalBinary"):hdr.index("func (h *FECHeader) UnmarshalBinary")]
    puts = re.findall(r"PutUint(16|32)\(b\[(\d+):(\d+)\], (?:uint\d+\()?h\.(\w+)", mar)
    assert len(puts) == 9, puts  # v2: six, v1: three
    for w, a, b, f in puts:
        assert re.search(r"h\.%s = (?:uint\d+\()?binary\.LittleEndian\.Uint%s\(b\[%s:%s\]\)" % (f, w, a, b), un), (f, a, b)


@NEED_REF
def test_sender_emits_v2_for_large_blocks(tmp_path):
    """The patched sender builds every header wide and marks it version 2 whenever FitsV1 fails (K >= 256:
    the K=512/1024/2048 configs), sizing the datagram by h.Len(); both receive loops take either version."""
    src = _patched(tmp_path)
    hdr, tx = src["header.go"], src["transfer.go"]
    fits = re.search(r"func \(h \*FECHeader\) FitsV1\(\) bool \{\s*return (.+?)\n", hdr).group(1)
    for k, want in ((255, True), (256, False), (1024, False)):
        h = {"BlockID": 3, "N": min(k + 76, 255) if k < 256 else k + 76, "K": k, "SymID": 7, "Flags": 0}
        expr = re.sub(r"h\.(\w+)", lambda m: str(h[m.group(1)]), fits).replace("&&", "and")
        assert eval(expr) == want, (k, expr)
    assert re.search(r"if !h\.FitsV1\(\) \{\s*h\.Version = 2", tx)
    assert "hl := h.Len()" in tx and "copy(b[:hl], h.MarshalBinary(nil))" in tx
    assert "data := b[fh.Len() : fh.Len()+int(fh.PayloadLen)]" in tx
    assert "io.ReadFull(us, hdrb[fecwire.HeaderLen:fecwire.HeaderV2Len])" in tx
    assert tx.count("rxm.ingest(uint16(fh.BlockID)") == 2
    # no fixed-size header slicing is left on either side
    assert "data := b[fecwire.HeaderLen" not in tx and "fecwire.HeaderLen+len(p.Data)" not in tx
