"""GPU: the decode's two apply kernels give the same bytes.

The register-table apply (k_xbits + the generated rq_apply_gi kernel, rq_applygi.cpp; the default) and
k_apply's v_perm byte tables (rq_debug_apply_mode(0)) compute x_E = g_E ^ X s from the same X.  Each case
decodes one batch with both and compares every block's bytes and status; solved blocks must equal their
source, unsolved ones keep their bytes.  The register-table apply runs twice, with rq_debug_apply_sx 1 and
0: in the experiments library (tests/test_gpu_experimental_programs.py runs this file against it) the first
reads syndromes that the first solver launch's extra workgroups precomputed into the r0 rows (when
T % 16 == 0 and the repair buffer is 16-byte aligned), the second XORs the received and r0 rows itself;
the two must give the same bytes.  (The release library has only the second.)  Cases cover e from 1 to past 128 in one batch (a slice of 16
outputs partly used, a last group of 1..5 syndromes), T not a multiple of 256 (a strip with lanes off)
and T = 8 (two dwords), and a block left unsolved beside solved ones.  (The in-place first solver lives in
the experiments library: tests/test_gpu_experimental_programs.py.)"""
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
    """[(bytes, statuses) under k_apply, under the register-table apply]; the register-table apply without
    the precomputed syndromes is checked against it here."""
    res = []
    for mode, sx in ((0, 1), (1, 1), (1, 0)):
        d = data.clone()
        old, old_sx = rq.apply_mode(mode), rq.apply_sx(sx)
        try:
            st = rq.DecodeBatch(K, T, erased, reps).run(d, rep)
            torch.cuda.synchronize()
        finally:
            rq.apply_mode(old)
            rq.apply_sx(old_sx)
        res.append((d, np.array(st)))
    (d1, st1), (d2, st2) = res[1], res[2]
    assert np.array_equal(st1, st2)
    bad = [b for b in range(d1.shape[0]) if not torch.equal(d1[b], d2[b])]
    assert not bad, ("blocks whose bytes differ with and without precomputed syndromes", bad)
    return res[:2]


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


def test_apply_stream_bound_falls_back(gpu, rq):
    """the register-table stream is laid out for the batch's largest e (~1.6 e^2 dwords per
    block).  A batch holding one block with e = 560 beside low-e blocks is past the bound and takes
    k_apply (every block recovered, the same bytes as rq_debug_apply_mode(0)); a single block at the
    bound (e = 512) takes the register-table apply with its largest stream, bit-identical to k_apply."""
    K, T = 1024, 64
    assert rq.lib().rq_debug_gi_fits(560, 5) == 0 and rq.lib().rq_debug_gi_fits(512, 1) == 1
    for ec, R in (([560, 3, 1, 7, 12], 600), ([512], 552)):
        src, data, erased, reps, rep = _case(rq, gpu, K, T, R, ec, 5 + ec[0])
        (d0, st0), (d1, st1) = _decode_both(rq, K, T, data, erased, reps, rep)
        assert list(st1) == [1] * len(ec) and list(st0) == list(st1), (ec, st0, st1)
        assert torch.equal(d0, d1), ec
        assert torch.equal(d1, src), ec


def test_apply_unaligned_repairs_skip_precomputed_syndromes(gpu, rq):
    """The precomputed syndromes take 16-byte row pieces: a repair buffer at a 4-byte offset (and T = 1 204,
    not a multiple of 16) decodes through the apply's own XOR, with the same bytes."""
    for T, off in ((1200, 4), (1204, 0)):
        K, R = 256, 40
        src, data, erased, reps, rep = _case(rq, gpu, K, T, R, [30, 7, 1, 22], 11 + off + T)
        buf = torch.empty(rep.numel() + 16, dtype=torch.uint8, device=gpu)
        base = (16 - buf.data_ptr() % 16) % 16 + off
        rep2 = buf[base:base + rep.numel()].view(rep.shape)
        rep2.copy_(rep)
        assert rep2.data_ptr() % 16 == off
        (d0, st0), (d1, st1) = _decode_both(rq, K, T, data, erased, reps, rep2)
        assert list(st1) == [1] * 4 and list(st0) == list(st1)
        assert torch.equal(d1, src) and torch.equal(d0, d1)
