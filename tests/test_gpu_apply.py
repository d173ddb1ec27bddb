"""GPU: the decode's alternative kernels give the same bytes (apply and first solve).

The register-table apply (k_xbits + the generated rq_apply_gi kernel, rq_applygi.cpp; the default) and
k_apply's v_perm byte tables (rq_debug_apply_mode(0)) compute x_E = g_E ^ X s from the same X.  Each case
decodes one batch with both and compares every block's bytes and status; solved blocks must equal their
source, unsolved ones keep their bytes.  Cases cover e from 1 to past 128 in one batch (a slice of 16
outputs partly used, a last group of 1..5 syndromes), T not a multiple of 256 (a strip with lanes off)
and T = 8 (two dwords), and a block left unsolved beside solved ones."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(rq, gpu, K, T, R, erase_counts, seed):
    g = torch.Generator().manual_seed(seed)
    n_blocks = len(erase_counts)
    src = torch.randint(0, 256, (n_blocks, K * T), dtype=torch.uint8, generator=g).to(gpu)
    esis = list(range(K, K + R))
    out = torch.empty((n_blocks, R * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    erased, reps, rows = [], [], []
    for b, ne in enumerate(erase_counts):
        er = sorted(rng.choice(K, ne, replace=False).tolist()) if ne else []
        rl = list(range(K, K + R))
        erased.append(er)
        reps.append(rl)
        rows.extend((b, r - K) for r in rl)
    rep = out.view(n_blocks, R, T)[torch.tensor([b for b, _ in rows], device=gpu),
                                   torch.tensor([r for _, r in rows], device=gpu)].contiguous()
    data = src.clone()
    for b, er in enumerate(erased):
        for i in er:
            data[b, i * T:(i + 1) * T] = (b * 31 + i) & 0xFF  # garbage g_E in the erased rows
    return src, data, erased, reps, rep


def _decode_both(rq, K, T, data, erased, reps, rep):
    res = []
    for mode in (0, 1):
        d = data.clone()
        old = rq.apply_mode(mode)
        try:
            st = rq.DecodeBatch(K, T, erased, reps).run(d, rep)
            torch.cuda.synchronize()
        finally:
            rq.apply_mode(old)
        res.append((d, np.array(st)))
    return res


@pytest.mark.parametrize("K,T,R,erase_counts", [
    (1024, 1200, 76, [55, 1, 16, 17, 33, 48, 49, 64, 70, 6, 7, 12, 13, 0, 2, 3]),
    (256, 1200, 140, [130, 129, 96, 5, 1]),
    (512, 68, 60, [40, 1, 17, 60]),
    (64, 8, 20, [20, 19, 1, 6]),
    (128, 256, 40, [40, 16, 15, 8]),
    (2048, 1200, 213, [200, 113, 6]),
])
def test_apply_kernels_agree(gpu, rq, K, T, R, erase_counts):
    src, data, erased, reps, rep = _case(rq, gpu, K, T, R, erase_counts, K + T)
    (d0, st0), (d1, st1) = _decode_both(rq, K, T, data, erased, reps, rep)
    assert np.array_equal(st0, st1)
    bad = [(b, ne, bool(torch.equal(d0[b], src[b])), bool(torch.equal(d1[b], src[b])))
           for b, ne in enumerate(erase_counts) if st1[b] == 1 and not (torch.equal(d0[b], src[b]) and torch.equal(d1[b], src[b]))]
    assert not bad, ("(block, e, k_apply == source, register-table == source)", bad)
    for b, ne in enumerate(erase_counts):
        assert torch.equal(d0[b], d1[b]), (b, ne)


def test_apply_unsolved_block_keeps_bytes(gpu, rq):
    # block 1 holds fewer repairs than erasures (not enough symbols, decided on the host): it keeps its
    # bytes while its neighbours in the batch are recovered, under either apply
    K, T, R = 256, 1200, 30
    src, data, erased, reps, _ = _case(rq, gpu, K, T, R, [20, 25, 10], 7)
    reps[1] = reps[1][:20]
    out = torch.empty((3, R * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, list(range(K, K + R)), out)
    rows = [(b, r - K) for b in range(3) for r in reps[b]]
    rep = out.view(3, R, T)[torch.tensor([b for b, _ in rows], device=gpu),
                            torch.tensor([r for _, r in rows], device=gpu)].contiguous()
    (d0, st0), (d1, st1) = _decode_both(rq, K, T, data, erased, reps, rep)
    assert np.array_equal(st0, st1)
    assert st1[0] == 1 and st1[2] == 1 and st1[1] == rq.RQ_ERR_NOT_ENOUGH
    assert torch.equal(d1[1], data[1])
    assert torch.equal(d0, d1)
    assert torch.equal(d1[0], src[0]) and torch.equal(d1[2], src[2])


def _decode_solve_modes(rq, K, T, data, erased, reps, rep):
    res = []
    for mode in (0, 1):
        d = data.clone()
        old = rq.solve_mode(mode)
        try:
            st = rq.DecodeBatch(K, T, erased, reps).run(d, rep)
            torch.cuda.synchronize()
        finally:
            rq.solve_mode(old)
        res.append((d, np.array(st)))
    return res


@pytest.mark.parametrize("K,T,R,erase_counts", [
    (1024, 1200, 76, [55, 1, 16, 17, 33, 48, 49, 64, 2, 3, 0, 63]),
    (256, 256, 80, [64, 70, 5, 1, 32]),
    (64, 8, 20, [20, 19, 1, 6]),
])
def test_in_place_solve_agrees(gpu, rq, K, T, R, erase_counts):
    """k_solve_ip (rows of e bytes, in-place Gauss-Jordan) and k_solve_pq<1, 4> give the same statuses
    and bytes; e > 64 takes the wide / general solvers either way."""
    src, data, erased, reps, rep = _case(rq, gpu, K, T, R, erase_counts, 3 * K + T)
    (d0, st0), (d1, st1) = _decode_solve_modes(rq, K, T, data, erased, reps, rep)
    assert np.array_equal(st0, st1)
    for b, ne in enumerate(erase_counts):
        assert torch.equal(d0[b], d1[b]), (b, ne)
        if st1[b] == 1:
            assert torch.equal(d1[b], src[b]), (b, ne)


def test_in_place_solve_margin_fallback(gpu, rq):
    """With no row margin the first pass sees exactly e rows: blocks rank-deficient on them go to the
    general solver under either first solver, with the same results."""
    K, T, R = 128, 256, 40
    src, data, erased, reps, rep = _case(rq, gpu, K, T, R, [40, 30, 20, 39, 8, 16], 11)
    old = rq.lib().rq_debug_decode_margin(0)
    try:
        (d0, st0), (d1, st1) = _decode_solve_modes(rq, K, T, data, erased, reps, rep)
    finally:
        rq.lib().rq_debug_decode_margin(old)
    assert np.array_equal(st0, st1)
    assert torch.equal(d0, d1)
    for b in range(len(st1)):
        if st1[b] == 1:
            assert torch.equal(d1[b], src[b]), b
