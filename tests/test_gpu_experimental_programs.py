"""The column-program variants the experiments library keeps behind knobs, on the GPU: the two-wave
(pair) program with dword loads, with four-row staging of its load wave, with HDPC rows moved to the
load wave, and the single-wave program with four-row staging (profiles/r04_pair).
They are not the shipped programs (measured slower at K=1024), but they must stay bit-exact: each runs
in its own process (the knobs are read once per process) through tools/colbench.py, which checks the
first and last block of a batch against the oracle, or through bench.py, which checks a whole
encode + decode step.  Skipped when the experiments library was not built (__graft_entry__.build()
builds it)."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
EXP = ROOT / "rl-quic-raptor_amd" / "build_exp" / "librqhip.so"

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not EXP.exists(), reason="experiments library not built (tools/build_experiments.sh)")]

VARIANTS = {
    "pair_dword": {"RQHIP_PAIR": "1", "RQHIP_PAIR_CFG": "6,16,192,0"},
    "pair_staged": {"RQHIP_PAIR": "1"},
    "pair_hdpc3": {"RQHIP_PAIR": "1", "RQHIP_PAIR_CFG": "6,16,192,32,1200,3"},
    "single_staged": {"RQHIP_PAIR": "0", "RQHIP_DMA4": "8"},
}


def _run(args, knobs, timeout=150, stderr=False):
    env = dict(os.environ, RQHIP_LIB=str(EXP), **knobs)
    r = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return (r.stdout, r.stderr) if stderr else r.stdout


@pytest.mark.parametrize("name", sorted(VARIANTS))
@pytest.mark.parametrize("K,N,B", [(1024, 1100, 24), (2048, 2260, 6)])
def test_variant_encode_matches_oracle(name, K, N, B):
    out = _run(["tools/colbench.py", str(K), "1200", str(N), str(B), "1"], VARIANTS[name])
    counts = [int(m) for m in re.findall(r"mismatching repairs: \[\] (\d+)", out)]
    assert counts == [0, 0], out


@pytest.mark.parametrize("name", ["pair_staged", "single_staged"])
def test_variant_encode_decode_step(name):
    """A full config-3 step (1 024 blocks) through bench.py on the experiments library: the decode's
    syndrome program is the same variant; bench.py asserts every recovered block bit-exact and the
    post-timing bytes + statuses."""
    out = _run(["tools/experiments/bench_exp.py", "--steps", "1", "--warmup", "0", "--cpu-sample", "0"], VARIANTS[name])
    assert '"decode_ok_fraction": 1.0' in out and '"post_timing_check": "bytes+statuses"' in out, out


def test_in_place_solve_agrees():
    """k_solve_ip (experiments library, rq_debug_solve_mode(1)) and the shipped k_solve_pq<1, 4> give the
    same statuses and bytes, with and without the first pass's row margin
    (tools/experiments/solve_ip_check.py)."""
    out = _run(["tools/experiments/solve_ip_check.py"], {})
    assert out.count("ok ") == 4, out


def test_descriptor_fetch_with_four_wave_workgroups():
    """the decode's descriptor fetch rides on the syndrome launch's spare workgroups in 4 KiB x W
    round trips; the release library runs W = 1, so the per-trip / chunk arithmetic at W = 4 is exercised
    here (RQHIP_WG=4): the launch must carry the fetch at W = 4 (its logged shape) and every block of a
    config-3 decode must come back bit-exact, sync and async (tools/experiments/fetch_wg_check.py)."""
    out, err = _run(["tools/experiments/fetch_wg_check.py"], {"RQHIP_WG": "4", "RQHIP_FETCH_LOG": "1"}, stderr=True)
    assert out.strip().endswith("ok"), out
    assert re.search(r"\[fetch\] carried=1 W=4 ", err), err[-2000:]


def test_precomputed_syndromes_agree():
    """The precomputed syndromes (experiments library, RQHIP_APPLY_SX=1: the first solver launch's extra
    workgroups XOR the received rows into the r0 rows, the apply loads one row per syndrome; measured not
    to pay) give the k_apply bytes on every case of tests/test_gpu_apply.py, and
    a pivot row past the first e + margin rows (XORed by general_block itself) decodes."""
    out = _run(["-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider", "tests/test_gpu_apply.py",
                "tests/test_gpu_decode_limits.py::test_first_solver_finishes_rank_deficient_rows_inline"],
               {"RQHIP_APPLY_SX": "1"})
    assert re.search(r"\b1[0-9] passed", out) and "failed" not in out, out
