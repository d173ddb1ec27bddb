"""GPU: a seeded sweep over source-block sizes, each against the oracle.

Every K' is its own generated column program (a different elimination, IR, schedule and register
allocation: P = 0 single scans for small K, the bit-accumulation program for large K, two or four waves
per SIMD where it fits), so a handful of BASELINE.json shapes leaves most programs untried on the
hardware.  For each K of the sweep (every K' of the RFC 6330 table up to K = 2 048, edges with padding rows,
both sides of the schedule switches, and seeded random sizes): a 3-block batch at T = 16 is encoded on the GPU with eight consecutive repair
ESIs and one far ESI, and blocks 0 and 2 are compared with the oracle byte for byte; then every block is
decoded with a few source rows erased and all nine repairs received (a union that is not a dense
range), and each block's status must equal the oracle decoder's decision on the same symbols
(recovered bytes equal to the source when it decodes; above K = 600 a block that decodes to its source is
taken as the oracle's decision without running its dense solve).  A second sweep runs the same checks over
symbol sizes from 8 to 4 096 bytes at K = 300."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

_RNG = np.random.default_rng(20261018)
KS = sorted({1, 2, 3, 4, 9, 10, 11, 17, 55, 101, 255, 256, 257, 333, 512, 513, 777, 1000, 1024, 1031, 1333, 1500,
             1800, 2000, 2048} | set(int(k) for k in _RNG.integers(5, 2049, 8)))
# every K' of RFC 6330's systematic-index table up to K = 2 048 (each a distinct elimination and program;
# K = K' has no padding rows)
KPRIME = (
    10, 12, 18, 20, 26, 30, 32, 36, 42, 46, 48, 49, 55, 60, 62, 69, 75, 84, 88, 91, 95, 97, 101, 114, 119,
    125, 127, 138, 140, 149, 153, 160, 166, 168, 179, 181, 185, 187, 200, 213, 217, 225, 236, 242, 248, 257,
    263, 269, 280, 295, 301, 305, 324, 337, 341, 347, 355, 362, 368, 372, 380, 385, 393, 405, 418, 428, 434,
    447, 453, 466, 478, 486, 491, 497, 511, 526, 532, 542, 549, 557, 563, 573, 580, 588, 594, 600, 606, 619,
    633, 640, 648, 666, 675, 685, 693, 703, 718, 728, 736, 747, 759, 778, 792, 802, 811, 821, 835, 845, 860,
    870, 891, 903, 913, 926, 938, 950, 963, 977, 989, 1002, 1020, 1032, 1050, 1074, 1085, 1099, 1111, 1136,
    1152, 1169, 1183, 1205, 1220, 1236, 1255, 1269, 1285, 1306, 1347, 1361, 1389, 1404, 1420, 1436, 1461,
    1477, 1502, 1522, 1539, 1561, 1579, 1600, 1616, 1649, 1673, 1698, 1716, 1734, 1759, 1777, 1800, 1824,
    1844, 1863, 1887, 1906, 1926, 1954, 1979, 2005, 2040, 2070
)
T = 16
FAR = 997  # a far repair ESI (K + FAR): its LT tuple reaches columns no near ESI touches


@pytest.mark.parametrize("K", sorted(set(KS) | set(KPRIME)))
def test_k_sweep_matches_oracle(gpu, rq, oracle, K):
    rng = np.random.default_rng(K)
    nb = 3
    esis = list(range(K, K + 8)) + [K + FAR]
    R = len(esis)
    src_h = rng.integers(0, 256, (nb, K * T), dtype=np.uint8)
    src = torch.from_numpy(src_h).to(gpu)
    out = torch.empty((nb, R * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, out)
    torch.cuda.synchronize()
    rep_h = out.view(nb, R, T).cpu().numpy()
    encs = {}
    for b in (0, nb - 1):
        encs[b] = oracle.OracleEncoder(src_h[b].tobytes(), T)
        ref = np.stack([encs[b].gen_symbol(e) for e in esis])
        assert np.array_equal(rep_h[b], ref), ("block", b, "repairs differ from the oracle")

    # decode: e source rows erased per block, every repair received
    erased = [sorted(rng.choice(K, min(K, e), replace=False).tolist()) for e in (8, 1, 5)]
    reps = [list(esis) for _ in range(nb)]
    data = src.clone()
    for b, er in enumerate(erased):
        for i in er:
            data[b, i * T:(i + 1) * T] = 0xA5
    rep = out.view(nb * R, T).contiguous()
    st = np.array(rq.DecodeBatch(K, T, erased, reps).run(data, rep))
    torch.cuda.synchronize()
    for b, er in enumerate(erased):
        if st[b] == 1 and K > 600:
            # a recovered block equal to its source was solvable on the symbols given (any e independent
            # received rows determine the erased ones), so the oracle would decode it too; its dense solve
            # of the whole system costs seconds at these sizes
            assert torch.equal(data[b], src[b]), ("block", b, "recovered bytes differ from the source")
            continue
        dec = oracle.OracleDecoder(K * T, T)
        for i in range(K):
            if i not in er:
                dec.add_symbol(i, src_h[b, i * T:(i + 1) * T].tobytes())
        for j, e in enumerate(esis):
            dec.add_symbol(e, rep_h[b, j].tobytes())
        ok = dec.decode()[0]
        assert st[b] == (1 if ok else 0), ("block", b, "status", st[b], "oracle decodes", ok)
        if ok:
            assert torch.equal(data[b], src[b]), ("block", b, "recovered bytes differ from the source")


# symbol sizes: one dword, lanes partly off in the last 64-column strip, exact strips, 16-byte multiples and not
TS = (8, 12, 20, 100, 252, 256, 260, 516, 1020, 1024, 1028, 1200, 1204, 2044, 4096)


@pytest.mark.parametrize("T_", TS)
def test_t_sweep_matches_oracle(gpu, rq, oracle, T_):
    """The same checks over symbol sizes at K = 300: every strip and lane-mask shape of the column program
    and the apply, 16-byte row multiples and not."""
    K, nb = 300, 3
    rng = np.random.default_rng(T_)
    esis = list(range(K, K + 8)) + [K + FAR]
    R = len(esis)
    src_h = rng.integers(0, 256, (nb, K * T_), dtype=np.uint8)
    src = torch.from_numpy(src_h).to(gpu)
    out = torch.empty((nb, R * T_), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T_, esis, out)
    torch.cuda.synchronize()
    rep_h = out.view(nb, R, T_).cpu().numpy()
    for b in (0, nb - 1):
        enc = oracle.OracleEncoder(src_h[b].tobytes(), T_)
        assert np.array_equal(rep_h[b], np.stack([enc.gen_symbol(e) for e in esis])), ("block", b)
    erased = [sorted(rng.choice(K, e, replace=False).tolist()) for e in (8, 1, 5)]
    data = src.clone()
    for b, er in enumerate(erased):
        for i in er:
            data[b, i * T_:(i + 1) * T_] = 0x5A
    st = np.array(rq.DecodeBatch(K, T_, erased, [list(esis)] * nb).run(data, out.view(nb * R, T_).contiguous()))
    torch.cuda.synchronize()
    for b, er in enumerate(erased):
        dec = oracle.OracleDecoder(K * T_, T_)
        for i in range(K):
            if i not in er:
                dec.add_symbol(i, src_h[b, i * T_:(i + 1) * T_].tobytes())
        for j, e in enumerate(esis):
            dec.add_symbol(e, rep_h[b, j].tobytes())
        ok = dec.decode()[0]
        assert st[b] == (1 if ok else 0), ("block", b, "status", st[b], "oracle decodes", ok)
        if ok:
            assert torch.equal(data[b], src[b]), ("block", b)
