"""The release library carries only what ships.

The decode solvers measured and not shipped (k_solve_fast / pm / reg / lean, the in-place k_solve_ip,
the pinfo-column PF variant, other wave counts), the unshipped k_apply shapes (wider lanes, other
slices), and the pair / four-row-staging column programs are built into build_exp/librqhip.so alone
(experiments-only translation units rq_kernels_exp.hip, rq_colasm_exp.cpp, rq_colprog_exp.cpp, and
RQHIP_EXPERIMENTS sections).  k_apply<4|8, 1, ...> ships: it is the decode's apply for a batch beyond
the register-table stream's bound (rq_engine.cpp gi_stream_fits, some block with e > 512).  This test reads the code objects embedded
in build/librqhip.so (the kernel descriptors' `.kd` symbols) and requires exactly the kernels the engine
dispatches; the generated column programs are assembled at run time and are not in the file.  CPU only."""
import re
import subprocess
from pathlib import Path

import pytest

import rqhip

ROOT = Path(__file__).resolve().parent.parent
SHIPPED = {
    "void rq::k_solve_pq<1, 4, false, false, true>(rq::SolveArgs)",
    "void rq::k_solve_pq<2, 4, false, false, true>(rq::SolveArgs)",
    "rq::k_solve(rq::SolveArgs)",
    "rq::k_pack_rows(rq::PackArgs)",
    "rq::k_gather(rq::DevParams, unsigned char const*, unsigned int, unsigned int const*, unsigned int, unsigned char*)",
    "void rq::k_xbits<8, 5, 2, 0>(rq::XbitsArgs)",
    "void rq::k_apply<4, 1, 2, 4, true>(rq::ApplyArgs, unsigned int, unsigned int, unsigned int)",
    "void rq::k_apply<8, 1, 2, 3, true>(rq::ApplyArgs, unsigned int, unsigned int, unsigned int)",
}


def kernels(path):
    b = Path(path).read_bytes()
    names = sorted(set(m.decode() for m in re.findall(rb"(_Z\w*?k_[a-z_]+\w*?)\.kd", b)))
    out = subprocess.run(["c++filt"] + names, capture_output=True, text=True, check=True).stdout.split("\n")
    return {n for n in out if n}


def test_release_library_has_only_shipped_kernels():
    rqhip.ensure_built()
    got = kernels(rqhip.LIB_PATH)
    assert got == SHIPPED, {"unexpected": sorted(got - SHIPPED), "missing": sorted(SHIPPED - got)}


def test_release_library_has_no_experiment_host_paths():
    """The pair / four-row-staging emitters are not linked into the release library: its debug entry
    points say so instead of compiling them."""
    L = rqhip.lib()
    with pytest.raises(rqhip.RaptorQError, match="experiments build only"):
        rqhip._check(L.rq_debug_pair_emulate(1024, 8, None, 0, None, None, None, None, None), L)
    with pytest.raises(rqhip.RaptorQError, match="experiments build only"):
        rqhip._check(L.rq_debug_dma4_emulate(1024, 16, None, 0, None, None, 8, 0, None, None), L)
    b = Path(rqhip.LIB_PATH).read_bytes()
    for sym in (b"compile_pair", b"emit_pair_asm", b"split_pair", b"compile_colprog_dma4"):
        assert sym not in b, sym


def test_experiments_library_keeps_the_variants():
    try:
        rqhip.exp_lib()
    except rqhip.RaptorQError as ex:
        pytest.skip(str(ex))
    got = kernels(rqhip.EXP_LIB_PATH)
    assert SHIPPED <= got
    for k in ("k_solve_fast", "k_solve_pm", "k_solve_reg", "k_solve_lean", "k_solve_pq<1, 4, true, false, true>", "k_solve_pq<1, 4, false, true, true>",
              "k_solve_pq<1, 4, false, false, false>", "k_solve_ip<4>",
              "k_apply<8, 5, 2, 3, true>"):
        assert any(k in n for n in got), k
