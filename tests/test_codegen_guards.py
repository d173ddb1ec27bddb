"""The round-4 code-generation guards fire (DESIGN.md sec. 2.5 "Round 4 guards").

* check_registers (rq_comgr.cpp) stands before every in-process assembly: a program whose text names an
  architectural VGPR at or above .amdhsa_accum_offset (an AGPR of the unified file, silently aliased) or
  an AGPR past the allocation is refused with the register named -- the bug class of the round-4 fault.
* the source buffer resource is bounded at ColKernArgs::src_bytes: the host emulator with that bound
  reads 0 beyond it, the engine's bound (row_end * T for one block) covers every row the program reads,
  and one dword less changes the result exactly as a zeroed last dword would.
CPU only (no compute calls on a GPU)."""
import re

import numpy as np
import pytest

import rqhip

K, T = 64, 48
ESIS = list(range(K, K + 16))


@pytest.fixture(scope="module")
def prog():
    return rqhip.colprog_asm(K, ESIS)


def _alloc(text):
    acc = int(re.search(r"\.amdhsa_accum_offset\s+(\d+)", text).group(1))
    total = int(re.search(r"\.amdhsa_next_free_vgpr\s+(\d+)", text).group(1))
    return acc, total


def _first_xor3(text):
    m = re.search(r"^(\s*v_bitop3_b32 )v(\d+)(, .*)$", text, re.M)
    assert m, "program has an XOR3"
    return m


def test_generated_program_passes(prog):
    assert rqhip.assemble(prog) > 0


def test_vgpr_at_accum_offset_refused(prog):
    acc, _ = _alloc(prog)
    m = _first_xor3(prog)
    bad = prog[:m.start()] + f"{m.group(1)}v{acc}{m.group(3)}" + prog[m.end():]
    with pytest.raises(rqhip.RaptorQError, match=rf"register v{acc} beyond the allocation \({acc}\)"):
        rqhip.assemble(bad)
    # one below is the last architectural VGPR: accepted
    ok = prog[:m.start()] + f"{m.group(1)}v{acc - 1}{m.group(3)}" + prog[m.end():]
    assert rqhip.assemble(ok) > 0


def test_agpr_past_allocation_refused(prog):
    acc, total = _alloc(prog)
    lim = total - acc
    m = re.search(r"^(\s*v_accvgpr_write_b32 )a(\d+)(, .*)$", prog, re.M)
    if m is None:  # a program this small may never park a value: add one AGPR write
        m = _first_xor3(prog)
        line = f"\tv_accvgpr_write_b32 a{lim}, v0\n"
        bad = prog[:m.start()] + line + prog[m.start():]
    else:
        bad = prog[:m.start()] + f"{m.group(1)}a{lim}{m.group(3)}" + prog[m.end():]
    with pytest.raises(rqhip.RaptorQError, match=rf"register a{lim} beyond the allocation \({lim}\)"):
        rqhip.assemble(bad)


def test_register_range_upper_end_checked(prog):
    acc, _ = _alloc(prog)
    m = _first_xor3(prog)
    bad = prog[:m.start()] + f"\tbuffer_load_dwordx4 v[{acc - 2}:{acc + 1}], v0, s[0:3], 0 offen\n" + prog[m.start():]
    with pytest.raises(rqhip.RaptorQError, match=rf"register v{acc + 1} beyond"):
        rqhip.assemble(bad)


def test_missing_directives_refused():
    with pytest.raises(rqhip.RaptorQError, match="no register allocation directives"):
        rqhip.assemble("\t.text\n\ts_endpgm\n")


def test_source_bound_reads_zero():
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, (K, T), dtype=np.uint8)
    full, row_end = rqhip.colprog_bound(K, T, ESIS, src, 1 << 62)
    ref = rqhip.colprog_eval(K, T, ESIS, src)
    assert np.array_equal(full, ref)
    assert 1 <= row_end <= K
    # the engine's bound for one block: every row the program reads lies inside it
    exact, _ = rqhip.colprog_bound(K, T, ESIS, src, row_end * T)
    assert np.array_equal(exact, full)
    # one dword less: the last row's last dword reads 0 -- the same bytes as a source with it zeroed
    short, _ = rqhip.colprog_bound(K, T, ESIS, src, row_end * T - 4)
    z = src.copy()
    z[row_end - 1, T - 4:] = 0
    zref, _ = rqhip.colprog_bound(K, T, ESIS, z, 1 << 62)
    assert np.array_equal(short, zref)
    assert not np.array_equal(short, full)
    # a bound past the source span (an offset beyond src_bytes) reads zeros: nothing at all
    none, _ = rqhip.colprog_bound(K, T, ESIS, src, 0)
    zero_src, _ = rqhip.colprog_bound(K, T, ESIS, np.zeros_like(src), 1 << 62)
    assert np.array_equal(none, zero_src)


@pytest.mark.parametrize("n_rows,n_dma4", [(1024, 0), (1024, 1040), (0, 0)])
def test_program_cache_entry_round_trip(tmp_path, n_rows, n_dma4):
    """The on-disk program cache keeps both row lists: cache_load reads the n_rows source-load rows and
    the n_dma4 four-row staging rows that cache_store writes, and its body hash covers both (ADVICE r4:
    the loader used to read n_rows only, so a staged entry never matched)."""
    p = str(tmp_path / "entry.co").encode()
    rqhip._check(rqhip.lib().rq_debug_cache_roundtrip(p, n_rows, n_dma4))
