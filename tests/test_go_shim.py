"""The committed cgo shim (go/fec/raptorq_rqhip.go, the drop-in for go/fec/raptorq_wrap.go:13-124) against
the C-ABI it binds (include/rqhip.h).  No Go toolchain exists here or on the GPU box, so the shim cannot be
compiled; this test keeps it from drifting: every C.rq_* function it calls is declared in the header with
the same number of parameters, every C.rq_* type and struct field it names exists, the exported Go API has
the reference's signatures, and the wrapper errors are the reference's strings."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
GO = (ROOT / "go" / "fec" / "raptorq_rqhip.go").read_text()
HDR = (ROOT / "include" / "rqhip.h").read_text()


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def _split_args(s):
    """Top-level comma split of an argument list."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def header_functions():
    """name -> parameter count of every prototype in rqhip.h."""
    src = _strip_c_comments(HDR)
    funcs = {}
    for m in re.finditer(r"\b(rq_\w+)\s*\(([^;{]*?)\)\s*;", src):
        params = m.group(2).strip()
        funcs[m.group(1)] = 0 if params in ("", "void") else len(_split_args(params))
    return funcs


def header_structs():
    """typedef'd struct name -> field names."""
    src = _strip_c_comments(HDR)
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(rq_\w+)\s*;", src, flags=re.S):
        fields = set()
        for decl in m.group(1).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            # "uint32_t T, K, n_blocks" or "const uint32_t* esi"
            head, _, rest = decl.partition(",")
            names = [re.findall(r"(\w+)\s*$", head)[0]] + [re.findall(r"(\w+)\s*$", r)[0] for r in rest.split(",") if r.strip()]
            fields.update(names)
        structs[m.group(2)] = fields
    for m in re.finditer(r"typedef\s+struct\s+(rq_\w+)\s+(rq_\w+)\s*;", src):
        structs.setdefault(m.group(2), set())
    return structs


def go_calls():
    """(name, argument count) of every C.rq_* call in the shim."""
    calls = []
    for m in re.finditer(r"\bC\.(rq_\w+)\(", GO):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(GO[i], 0)
            i += 1
        args = GO[m.end():i - 1]
        calls.append((m.group(1), len(_split_args(args)) if args.strip() else 0))
    return calls


def test_every_call_matches_a_prototype():
    funcs = header_functions()
    calls = go_calls()
    assert len(calls) >= 17, calls
    for name, n in calls:
        assert name in funcs, "C.%s is not declared in include/rqhip.h" % name
        assert funcs[name] == n, "C.%s: %d arguments in the shim, %d in rqhip.h" % (name, n, funcs[name])
    # the per-object API of the reference boundary is bound in full
    used = {c for c, _ in calls}
    for need in ("rq_encoder_create", "rq_encoder_symbol", "rq_encoder_symbols", "rq_encoder_k", "rq_encoder_symbol_size",
                 "rq_encoder_free", "rq_decoder_create", "rq_decoder_add", "rq_decoder_decode", "rq_decoder_k",
                 "rq_decoder_free", "rq_last_error", "rq_strerror", "rq_encode_batch_host", "rq_decode_blocks_host"):
        assert need in used, need


def test_types_and_fields_exist():
    structs = header_structs()
    for t in set(re.findall(r"\bC\.(rq_\w+)\b(?!\()", GO)):
        assert t in structs, "C.%s is not a type of include/rqhip.h" % t
    # field names of the composite literals and member accesses on the C structs
    for m in re.finditer(r"C\.(rq_\w+)\{(.*?)\}", GO, flags=re.S):
        for f in re.findall(r"(\w+)\s*:", m.group(2)):
            assert f in structs[m.group(1)], "C.%s has no field %s" % (m.group(1), f)
    for f in re.findall(r"io\[b\]\.(\w+)", GO):
        assert f in structs["rq_block_io"], f


def test_reference_api_and_error_strings():
    sigs = [
        r"func NewRaptorQEncoder\(data \[\]byte, K, L int\) \(\*RaptorQEncoder, error\)",
        r"func \(e \*RaptorQEncoder\) GenSymbol\(id uint32\) \[\]byte",
        r"func \(e \*RaptorQEncoder\) BaseSymbolsNum\(\) uint32",
        r"func NewRaptorQDecoder\(dataSize int, L int\) \(\*RaptorQDecoder, error\)",
        r"func \(d \*RaptorQDecoder\) AddSymbol\(id uint32, data \[\]byte\) \(bool, error\)",
        r"func \(d \*RaptorQDecoder\) Decode\(\) \(bool, \[\]byte, error\)",
        r"func RaptorQEncodeBlock\(data \[\]byte, N, K, L int\) \(\[\]Packet, error\)",
        r"func RaptorQDecodeBytes\(recv \[\]Packet, N, K, L, dataSize int\) \(\[\]byte, bool\)",
        r"type RaptorQEncoder struct \{\s*K int\s*L int",
        r"type RaptorQDecoder struct \{\s*K\s+int\s*L\s+int",
    ]
    for s in sigs:
        assert re.search(s, GO), s
    for msg in ("bad K or L", "bad dataSize or L", "bad N/K/L"):
        assert 'errors.New("%s")' % msg in GO, msg
    assert GO.startswith("//") and "\npackage fec\n" in GO
    # library errors carry the library's text: rq_last_error, else rq_strerror of the code
    assert "C.rq_last_error()" in GO and "C.rq_strerror(code)" in GO


def test_header_error_strings_match_library(rq):
    """The messages the shim forwards (rq_strerror) are the reference library's (rqhip.h comments)."""
    lib = rq.lib()
    assert lib.rq_strerror(rq.RQ_ERR_SYMBOL_SIZE_ZERO) == b"symbol size cannot be zero"
    assert lib.rq_strerror(rq.RQ_ERR_K_TOO_BIG) == b"k is too big"
    assert lib.rq_strerror(rq.RQ_ERR_NOT_ENOUGH) == b"not enough symbols to decode"
