"""Schedule compiler (rq_plan.cpp) vs the oracle, on the CPU.

The per-K' program the GPU replays is exported through the C-ABI (rq_plan_export) and
interpreted in numpy (tests/plan_replay.py, the same semantics as k_encode); the resulting
intermediate symbols must equal the oracle's dense-Gauss solution of the reference's
constraint system (RQ/solver.go:25-185) bit for bit.
"""
import numpy as np
import pytest

from tests.plan_replay import replay


@pytest.mark.parametrize("K,T", [(1, 8), (5, 1100), (10, 16), (26, 64), (64, 48), (101, 12), (256, 16), (1024, 8)])
def test_plan_replay_matches_oracle(rq, oracle, K, T):
    rng = np.random.default_rng(1000 + K)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    p = rq.params(len(data), T)
    plan = rq.plan_export(K)
    assert plan["Kp"] == p["Kp"] and plan["L"] == p["L"]
    src = np.zeros((p["Kp"], T), np.uint8)
    src.reshape(-1)[:len(data)] = data
    C = replay(plan, src, p["K"], p["H"])
    C_ref = oracle.encode_C(data, T)
    assert np.array_equal(C, C_ref)


def test_plan_replay_partial_block(rq, oracle):
    """Library K < wrapper K (short final block of raptorq_eval generations)."""
    T = 32
    data = np.random.default_rng(5).integers(0, 256, 123 * T - 17, dtype=np.uint8)
    p = rq.params(len(data), T)
    assert p["K"] == 123
    plan = rq.plan_export(p["K"])
    src = np.zeros((p["Kp"], T), np.uint8)
    src.reshape(-1)[:len(data)] = data
    assert np.array_equal(replay(plan, src, p["K"], p["H"]), oracle.encode_C(data, T))


def test_plan_op_counts_vs_reference(rq):
    """the reference encode at K'=1032 performs 19 206 XOR + 2 625 mul-add
    symbol row-ops.  The default plan finishes pass B in place (C_k = y_k ^ W_k C_U, one
    dependency level instead of ~90), trading XOR reads for depth: it must stay within 2x the
    reference's row-ops and use fewer GF(256) mul-adds."""
    s = rq.plan_stats(1024)
    assert s["n_src_xor"] + s["n_src_mul"] < 2 * (19206 + 2625)
    assert s["n_src_mul"] < 2625
    assert s["n_levels"] <= 110
    assert s["u"] >= 50  # at least the P=50 permanently inactive columns


@pytest.mark.parametrize("K", [64, 256, 1024, 2048])
def test_plan_fits_lds(rq, K):
    s = rq.plan_stats(K)
    assert s["n_slots"] * 4 * 8 <= 160 * 1024  # at least an 8-dword strip fits the LDS


@pytest.mark.parametrize("K,T,sd", [(5, 16, 4), (64, 8, 2), (256, 8, 30), (1024, 4, 30), (64, 8, 13)])
def test_wave_streams_match_oracle(rq, oracle, K, T, sd):
    """The per-wave instruction streams k_encode executes (paired statements, paged segments,
    split Horner pieces) reproduce the oracle's intermediate symbols."""
    from tests.plan_replay import replay_waves
    rng = np.random.default_rng(77 + K)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    p = rq.params(len(data), T)
    plan = rq.plan_export(K)
    wave = rq.wave_export(K, sd)
    assert wave["words"].size % 64 == 0
    src = np.zeros((p["Kp"], T), np.uint8)
    src.reshape(-1)[:len(data)] = data
    assert np.array_equal(replay_waves(wave, plan, src, p["K"], p["H"]), oracle.encode_C(data, T))
