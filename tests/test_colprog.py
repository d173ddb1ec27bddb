"""The column program (the encode hot path's code generator) checked on the CPU, stage by stage:

* its IR (rq_colprog.cpp) evaluated on the host equals the oracle's repair / source symbols and
  intermediate symbols (C is the unique solution, so any elimination order
  must reproduce the reference bytes);
* the register-allocated machine program (rq_colasm.cpp: VGPR/AGPR/scratch tiers, prefetched
  loads, exact vmcnt waits) emulated on the host gives the same bytes, with every wait and
  scratch ordering checked by the emulator;
* the generated gfx950 assembly assembles in process (amd_comgr).

The GPU runs exactly this machine program (tests/test_gpu_parity.py)."""
import ctypes
import re

import numpy as np
import pytest

CASES = [(64, 48, 16), (5, 20, 6), (1, 8, 4), (26, 8, 40), (257, 16, 20), (1000, 12, 10), (1024, 16, 76),
         (2048, 8, 30)]


def _esis(K, nrep):
    # repairs, first/last source rows, one far repair ESI
    return list(range(K, K + nrep)) + [0, K - 1, K + 5000]


@pytest.mark.parametrize("K,T,nrep", CASES)
def test_ir_matches_oracle(rq, oracle, K, T, nrep):
    rng = np.random.default_rng(K * 3 + T)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = _esis(K, nrep)
    out = rq.colprog_eval(K, T, esis, data)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), (K, e)


@pytest.mark.parametrize("K,T,nrep", CASES)
def test_machine_program_matches_oracle(rq, oracle, K, T, nrep):
    rng = np.random.default_rng(K * 5 + T)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = _esis(K, nrep)
    out, st = rq.colprog_emulate(K, T, esis, data)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), (K, e)
    assert st["sync_reloads"] <= st["spill_loads"]


# opts = {n_vgpr, n_agpr, la_load, la_reload, max_vmem, n_lds + 1}
@pytest.mark.parametrize("opts", [[64, 32, 40, 20, 8, 1], [32, 4, 400, 400, 60, 1], [200, 8, 16, 8, 4, 1],
                                  [32, 4, 400, 400, 60, 9], [24, 1, 40, 20, 8, 17], [16, 2, 100, 50, 12, 3]])
def test_machine_program_under_register_pressure(rq, oracle, opts):
    """Tight register files, short/long look-aheads, a small vmcnt budget and a small LDS tier force
    every spill / reload / wait path of the allocator (global scratch, LDS slots, lgkmcnt); the bytes
    must not change."""
    K, T = 257, 12
    rng = np.random.default_rng(sum(opts))
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = list(range(K, K + 12)) + [3]
    out, st = rq.colprog_emulate(K, T, esis, data, opts)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), e
    assert st["spill_stores"] > 0
    if opts[5] > 1:
        assert 0 < st["lds_slots"] <= opts[5] - 1 and st["lds_loads"] > 0


@pytest.mark.parametrize("opts", [[123, 128, 0, 0, 0, 81], [246, 1, 0, 0, 0, 81], [79, 84, 0, 0, 0, 54]])
def test_two_and_three_wave_budgets(rq, oracle, opts):
    """Register budgets of 256 / 168 per lane (2 / 3 waves per SIMD) at K=1024: emulated bytes equal the
    oracle's and the program assembles."""
    K, T = 1024, 8
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = list(range(K, K + 20))
    out, st = rq.colprog_emulate(K, T, esis, data, opts)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), e


@pytest.mark.parametrize("K,T", [(64, 48), (1024, 8)])
def test_intermediate_symbols_mode(rq, oracle, K, T):
    """Per-object encoder program: outputs are C[0..L-1] (RQ/encoder.go:15-33, Encoder.relaxed)."""
    import ctypes
    rng = np.random.default_rng(K)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    p = rq.params(K * T, T)
    out = np.zeros((p["L"], T), np.uint8)
    st = np.zeros(12, np.uint32)
    rc = rq.lib().rq_debug_colprog_eval(K, T, None, 0, data.ctypes.data, out.ctypes.data,
                                        st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    assert rc == 0
    assert np.array_equal(out, oracle.encode_C(data, T))


SCALAR_ALLOWED = {"s_add_u32", "s_addc_u32", "s_and_b32", "s_and_b64", "s_endpgm", "s_load_dwordx8",
                  "s_lshl_b32", "s_lshr_b32", "s_mov_b32", "s_mul_hi_u32", "s_mul_i32", "s_nop",
                  "s_waitcnt", "s_cmp_ge_u32", "s_cbranch_scc1", "s_mov_b64", "s_cmp_lt_u32",
                  "s_cselect_b32", "s_load_dwordx2", "s_load_dwordx4", "s_load_dwordx16",
                  "s_getpc_b64", "s_sub_u32", "s_subb_u32", "s_setpc_b64",
                  "s_min_u32", "s_cbranch_execz", "s_branch",  # (the decode's descriptor-fetch loop)
                  "s_cbranch_scc0"}  # (cross-item prefetch: past the wave's last item)


def test_program_size_and_assembly(rq):
    st = rq.colprog_stats(1024, list(range(1024, 1100)))
    # every XOR / xtime of the schedule is one VALU op of the machine program
    assert st["valu"] > 5000 and st["src_loads"] == 1024 and st["out_stores"] == 76
    asm = rq.colprog_asm(64, list(range(64, 80)))
    assert ".amdhsa_kernel rq_colprog" in asm and "v_bitop3_b32" in asm
    # scalar instructions are limited to kernarg loads, address arithmetic and waits: every
    # memory write of the program goes through vector (buffer/global) stores
    scalar_ops = set(re.findall(r"^\s*(s_[a-z0-9_]+)", asm, re.M))
    assert scalar_ops <= SCALAR_ALLOWED, scalar_ops - SCALAR_ALLOWED
    assert rq.colprog_assemble(64, list(range(64, 80))) > 1000
    # a full-size program (>128 KiB of code: the loop back-edge must not be a 16-bit branch)
    assert rq.colprog_assemble(1024, list(range(1024, 1100))) > 131072


# cross-item prefetch (AllocOpts::cip): opts[6] = head rows + 1, opts[7] = rows per batch, opts[8] = IR nodes
# between batches
@pytest.mark.parametrize("K,T,nrep,cip,batch,gap", [(1024, 16, 76, 64, 8, 24), (1024, 8, 76, 96, 16, 8),
                                                    (64, 48, 16, 24, 4, 2), (5, 20, 6, 8, 1, 1), (1, 8, 4, 4, 8, 24),
                                                    (257, 16, 20, 48, 8, 64), (2048, 8, 30, 40, 8, 24)])
def test_cross_item_prefetch_matches_oracle(rq, oracle, K, T, nrep, cip, batch, gap):
    """The next item's first source rows are loaded during the item's load-free tail (MI_PFX) into the
    registers its first loads use (MI_HEAD).  The emulator runs the item twice, the second time as the
    wave's next item: each head register must hold its row from the prefetch, nothing may write a
    handed-over register in between, and the vmcnt waits must hold with the previous item's prefetch and
    stores still counted.  Both runs give the reference bytes."""
    rng = np.random.default_rng(K + cip)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = _esis(K, nrep)
    out, st = rq.colprog_emulate(K, T, esis, data, [0] * 6 + [cip + 1, batch, gap])
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), (K, e)


@pytest.mark.parametrize("opts", [[64, 32, 40, 20, 8, 1, 17, 4, 8], [32, 4, 400, 400, 60, 9, 9, 8, 24],
                                  [24, 1, 40, 20, 8, 17, 7, 2, 1], [200, 8, 16, 8, 4, 1, 49, 16, 4]])
def test_cross_item_prefetch_under_register_pressure(rq, oracle, opts):
    """Head registers vacated under pressure (values moved to AGPRs or out to LDS / scratch) and a small
    vmcnt budget (a batch waits for room first)."""
    K, T = 257, 12
    rng = np.random.default_rng(sum(opts))
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = list(range(K, K + 12)) + [3]
    out, st = rq.colprog_emulate(K, T, esis, data, opts)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), e


def test_cross_item_prefetch_random_shapes(rq, oracle):
    """Seeded random (K, outputs, register budget, prefetch rows / batch / gap) combinations through the
    two-item emulation: any head-register hand-over, vacate or vmcnt slip shows up as an emulator error
    or wrong bytes."""
    rng = np.random.default_rng(2026)
    for it in range(40):
        K = int(rng.integers(2, 300 if it % 4 else 1100))
        T = 4 * int(rng.integers(1, 5))
        nrep = int(rng.integers(1, 24))
        esis = sorted(set(int(x) for x in rng.integers(K, K + 3 * nrep + 2, nrep))) + [int(rng.integers(0, K))]
        nv = int(rng.choice([250, 120, 48, 24]))
        na = int(rng.choice([256, 64, 8, 1]))
        opts = [nv, na, int(rng.choice([0, 40, 320])), 0, int(rng.choice([0, 12, 56])), int(rng.choice([0, 9, 157])),
                int(rng.integers(2, 80)), int(rng.integers(1, 17)), int(rng.integers(1, 64))]
        data = rng.integers(0, 256, K * T, dtype=np.uint8)
        out, st = rq.colprog_emulate(K, T, esis, data, opts)
        enc = oracle.OracleEncoder(data.tobytes(), T)
        for i, e in enumerate(esis):
            assert np.array_equal(out[i], enc.gen_symbol(e)), (K, T, esis, opts, e)


def test_cross_item_prefetch_assembly(rq):
    """The prologue loads the wave's first item's head rows and the tail the next item's, into the top
    VGPRs, with V_LDS2 as the offset register and the item's lane mask in s[54:55].  Past the wave's last
    item the tail's loads re-read the current item's rows instead of being skipped: the allocator's vmcnt
    waits after them count them (a skipped batch left those waits short: a GPU race in round 6, two wrong
    rows of 552 on a one-item launch).  The program assembles."""
    K, esis = 1024, list(range(1024, 1100))
    asm = rq.colprog_asm(K, esis, [0] * 6 + [33, 8, 24])
    assert asm.count(".Lcipe0:") == 1 and asm.count("s_cbranch_scc0 .Lcip") == 1
    assert asm.count("s_cbranch_scc1 .Lcipn1") == 1 and asm.count("s_mov_b64 exec, s[54:55]") == 1 + 4
    pro, body = asm.split(".Lloop:", 1)
    head = "buffer_load_dword v249, v255, s[24:27], s42 offen"  # the first head row (V_LDS2 = v255)
    assert pro.count(head) == 1 and body.count(head) == 1 and body.count(", v255, s[24:27]") == 32
    assert body.count("s_mov_b64 exec, s[22:23]") >= 4
    assert ".error" not in asm
    scalar_ops = set(re.findall(r"^\s*(s_[a-z0-9_]+)", asm, re.M))
    assert scalar_ops <= SCALAR_ALLOWED, scalar_ops - SCALAR_ALLOWED
    size = ctypes.c_size_t(0)
    rq._check(rq.lib().rq_debug_assemble(asm.encode(), len(asm), ctypes.byref(size)))
    assert size.value > 131072


SCHED_RS, SCHED_4R = 1 << 16, 1 << 17  # rq_colprog.hpp


@pytest.mark.parametrize("passes", [0, 1, 2, 3, 5, SCHED_RS | 96, SCHED_RS | 400, SCHED_4R, SCHED_4R | 64, SCHED_4R | 2])
@pytest.mark.parametrize("K,T,nrep", [(64, 16, 16), (1024, 8, 76), (2048, 4, 30)])
def test_every_ir_schedule_matches_oracle(rq, oracle, K, T, nrep, passes):
    """Each IR schedule the engine may choose (one demand-driven scan, peeling-order production
    with P Horner passes or replacement-selection Horner runs, or no scan with bh accumulated bit
    by bit (SCHED_4R), rq_colprog.cpp build()) gives the reference bytes, as IR and as the
    allocated, emulated machine program."""
    rng = np.random.default_rng(K + 11 * passes)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    esis = _esis(K, nrep)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    old = rq.lib().rq_debug_colprog_passes(passes)
    try:
        ir_out = rq.colprog_eval(K, T, esis, data)
        mp_out, st = rq.colprog_emulate(K, T, esis, data)
    finally:
        rq.lib().rq_debug_colprog_passes(old)
    for i, e in enumerate(esis):
        ref = enc.gen_symbol(e)
        assert np.array_equal(ir_out[i], ref), (K, passes, e)
        assert np.array_equal(mp_out[i], ref), (K, passes, e)


# ---- two-wave (pair) programs: rq_colprog_exp.cpp split_pair + rq_colasm_exp.cpp compile_pair / emulate_pair ----
@pytest.fixture(scope="module")
def exp_rq(rq):
    """The pair and four-row-staging programs are compiled into the experiments library only (VERDICT r4
    item 4): these host tests load it beside the release library (built on first use)."""
    try:
        rq.exp_lib()
    except rq.RaptorQError as ex:
        pytest.skip(str(ex))
    return rq


@pytest.mark.parametrize("K,T,esis", [
    (1024, 16, list(range(1024, 1100))),                                  # config 3's encode program
    (1024, 8, [1024 + i for i in range(0, 160, 2)] + [0, 1023, 7000]),   # a sparse decode union + sources
    (2048, 8, list(range(2048, 2260))),                                   # config 5's K=2048 shape
    (1500, 12, list(range(1500, 1658))),
])
def test_pair_program_matches_oracle(exp_rq, oracle, K, T, esis):
    """Wave A (loads, forward pass, pushes) and wave B (HDPC bit accumulation, dense part, outputs) run on
    the host over two consecutive items, every ring read checked against the barrier intervals; the
    outputs equal the oracle's symbols, and the kernel assembles."""
    rng = np.random.default_rng(K + T)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    out, st = exp_rq.pair_emulate(K, T, esis, data.tobytes(), assemble=(K == 1024 and T == 16))
    assert st["sched_4r"] == 1
    assert st["a_barriers"] == st["transfers"] and st["a_ring_stores"] == st["b_ring_loads"] == st["handed"]
    assert st["b_stores"] <= len(esis) and st["a_loads"] >= K
    assert st["lds_bytes"] <= 80 * 1024
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), (K, e)
    if K == 1024 and T == 16:
        assert st["code_bytes"] > 0


@pytest.mark.parametrize("cfg", [(1, 8, 0), (2, 4, 0), (10, 16, 320), (3, 32, 0), (6, 16, 192, 32, 3), (2, 16, 0, 0xFFFFFFFF, 5)])
def test_pair_lag_and_transfer_sizes(exp_rq, oracle, cfg):
    """Other lags / transfer sizes / rings / staging / HDPC rows accumulated on wave A: the same bytes (the
    ring window check and the barrier intervals hold for each)."""
    K, T = 1024, 8
    esis = list(range(K, K + 76))
    rng = np.random.default_rng(sum(cfg))
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    out, st = exp_rq.pair_emulate(K, T, esis, data.tobytes(), cfg=cfg)
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e))
    assert st["ring"] >= min(cfg[1], 16)


@pytest.mark.parametrize("K,quads", [(1024, 4), (1024, 8), (2048, 8)])
def test_single_wave_four_row_staging_matches_oracle(exp_rq, oracle, K, quads):
    """The single-wave program re-allocated with four-row staging (1 KiB LDS-DMA per four source rows,
    rows then read from LDS): run on the host with the DMA / table-read ordering checked, the outputs
    equal the oracle's symbols, and the kernel assembles within its register and LDS budget."""
    T = 16
    esis = list(range(K, K + K // 10 + 8)) if K == 1024 else [0, 5, K - 1] + list(range(K, K + 40))
    rng = np.random.default_rng(K + quads)
    data = rng.integers(0, 256, K * T, dtype=np.uint8)
    out, st = exp_rq.dma4_emulate(K, T, esis, data.tobytes(), quads=quads, assemble=(K == 1024))
    assert st["sched_4r"] == 1 and st["dma4"] > 0
    assert st["tbl_slots"] + st["lds_slots"] <= 160
    enc = oracle.OracleEncoder(data.tobytes(), T)
    for i, e in enumerate(esis):
        assert np.array_equal(out[i], enc.gen_symbol(e)), (K, e)
    if K == 1024:
        assert st["code_bytes"] > 0


def test_pair_ring_too_small_is_refused(exp_rq):
    """A ring that cannot hold lag + 2 transfers is refused at compile time (never a runtime race)."""
    with pytest.raises(exp_rq.RaptorQError):
        exp_rq.pair_emulate(1024, 8, list(range(1024, 1100)), cfg=(8, 16, 40))
