"""CPU: the register-table apply kernel's generator (rq_applygi.cpp) -- every shape the experiments sweep
uses assembles in process, the shipped shape fits four waves per SIMD, the VGPR index mode can only reach
the table (the highest indexed register stays inside the allocation), and its scalar instructions are
loads, arithmetic, waits and the index mode only.  Its bytes are held to k_apply's on the GPU (tests/test_gpu_apply.py)."""
import re

import numpy as np
import pytest

import rqhip

SHAPES = [(8, 5, 2, 1), (8, 5, 1, 1), (8, 4, 1, 1), (8, 6, 2, 1), (12, 5, 2, 1), (16, 6, 2, 1), (4, 4, 1, 2),
          (8, 5, 1, 2), (8, 5, 2, 1, 1), (16, 5, 2, 1, 1), (8, 5, 1, 2, 1)]


def _vgprs(text):
    return int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", text).group(1))


@pytest.mark.parametrize("shape", SHAPES)
def test_shapes_assemble(shape):
    text, code = rqhip.apply_gi_asm(*shape)
    assert code > 0
    g = shape[1]
    nv = _vgprs(text)
    # the index mode reads v[table + idx] with idx < 2^G: every table register is allocated
    tables = [int(m) for m in re.findall(r"v_xor_b32_e32 v\d+, v(\d+), v\d+\n\ts_set_gpr_idx", text)]
    on = re.findall(r"s_set_gpr_idx_on s\d+, gpr_idx\(SRC0\)\n\tv_xor_b32_e32 v(\d+), v(\d+), v(\d+)", text)
    assert on, "no indexed lookup"
    for _, src, _ in on:
        assert int(src) + (1 << g) - 1 < nv
    assert all(t + (1 << g) - 1 < nv for t in tables)
    # scalar instructions: loads, address / loop arithmetic, waits and the index mode only (memory is
    # written by vector stores); every s_set_gpr_idx_on is turned off again
    scalar = {m for m in re.findall(r"^\t(s_[a-z0-9_]+)", text, re.M)}
    allowed = ("s_load_dword", "s_waitcnt", "s_lshl_b32", "s_lshr_b32", "s_add_u32", "s_addc_u32", "s_sub_u32",
               "s_mul_i32", "s_mul_hi_u32", "s_cmp_", "s_cbranch_", "s_branch", "s_min_u32", "s_mov_b32",
               "s_mov_b64", "s_and_b32", "s_and_b64", "s_nop", "s_set_gpr_idx_", "s_endpgm")
    assert all(m.startswith(allowed) for m in scalar), sorted(m for m in scalar if not m.startswith(allowed))
    assert text.count("s_set_gpr_idx_on") == text.count("s_set_gpr_idx_off")


def test_shipped_shape_occupancy():
    text, _ = rqhip.apply_gi_asm()  # the library's default shape
    nv = _vgprs(text)
    assert nv <= 128, nv  # four waves per SIMD (512 VGPRs)
    assert "rq_apply_gi_k8_g5_p2_c1" in text


@pytest.mark.parametrize("shape", [(8, 5, 2, 1), (8, 4, 1, 1), (8, 5, 1, 2), (16, 6, 2, 1)])
def test_precomputed_syndrome_shapes(shape):
    """GiShape::SX (syndromes precomputed into the r0 rows beside the first solver): one load per
    syndrome, from the r0 rows' buffer resource s[52:55] only (never the received rows' s[48:51]), a ring of
    G values per slot (fewer VGPRs than the two-row shape), the same index-mode guard."""
    kc, g, pdg, cpl = shape
    text, code = rqhip.apply_gi_asm(kc, g, pdg, cpl, sx=1)
    text2, _ = rqhip.apply_gi_asm(kc, g, pdg, cpl)
    assert code > 0 and f".globl rq_apply_gi_k{kc}_g{g}_p{pdg}_c{cpl}_s\n" in text
    assert "s[48:51]" not in "\n".join(l for l in text.splitlines() if "buffer_load" in l)
    loads = lambda t: sum(1 for l in t.splitlines() if "buffer_load_dword" in l and "s[52:55]" in l)
    assert loads(text) == loads(text2)  # the r0-row loads stay, the received-row ones go
    assert sum(1 for l in text2.splitlines() if "s[48:51]" in l and "buffer_load" in l) == loads(text2)
    assert _vgprs(text) == _vgprs(text2) - ((g * pdg * cpl) // 4) * 4 or _vgprs(text) < _vgprs(text2)
    assert rqhip.lib().rq_debug_apply_gi_check(kc, g, pdg, cpl | 512, text.encode()) == 0


def test_bad_shapes_refused():
    for shape in ((6, 5, 2, 1), (8, 7, 2, 1), (8, 5, 3, 1), (8, 5, 2, 3), (16, 6, 2, 2), (4, 4, 1, 1, 1), (12, 5, 2, 1, 1)):
        with pytest.raises(rqhip.RaptorQError):
            rqhip.apply_gi_asm(*shape)


def _gf_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ 0x11D) & 0xFF if a & 0x80 else a << 1
        b >>= 1
    return r


def test_bit_plane_identity():
    """The algebra the kernel relies on, on random bytes: sum_m X[k][m] s_m (GF(256)) equals Horner over
    the eight planes sum_g Tab_g[idx_{k,b,g}] with idx the G-bit subset of bit b of group g's coefficients
    and Tab_g[S] the XOR of the subset S of group g's syndromes."""
    rng = np.random.default_rng(4)
    e, G, n = 23, 5, 64
    X = rng.integers(0, 256, (e, e))
    s = rng.integers(0, 256, (e, n))
    for k in range(e):
        want = np.zeros(n, np.int64)
        for m in range(e):
            want ^= np.array([_gf_mul(int(X[k][m]), int(v)) for v in s[m]])
        planes = np.zeros((8, n), np.int64)
        for g0 in range(0, e, G):
            grp = list(range(g0, min(e, g0 + G)))
            tab = np.zeros((1 << G, n), np.int64)
            for S in range(1, 1 << G):
                for t, m in enumerate(grp):
                    if S >> t & 1:
                        tab[S] ^= s[m]
            for b in range(8):
                idx = sum(((int(X[k][m]) >> b) & 1) << t for t, m in enumerate(grp))
                planes[b] ^= tab[idx]
        x = planes[7].copy()
        for b in range(6, -1, -1):
            x = np.array([_gf_mul(int(v), 2) for v in x]) ^ planes[b]
        assert np.array_equal(x, want), k


def test_stream_bound():
    """The register-table apply runs only while its index stream stays bounded: e <= 512 and at
    most 512 MiB for the solve list; beyond it the decode takes k_apply (rq_engine.cpp gi_stream_fits)."""
    fits = rqhip.lib().rq_debug_gi_fits
    assert fits(60, 1024) == 1          # config 3: ~27 MB
    assert fits(200, 1024) == 1
    assert fits(512, 1) == 1 and fits(512, 300) == 1
    assert fits(512, 1024) == 0         # 1.7 MB per block
    assert fits(513, 1) == 0 and fits(56403, 1) == 0


# ---- the index stream the solvers write, emulated on the host, and the index-mode guard
KC, G, PDG = 8, 5, 2   # the shipped shape (rq_device.hpp GiShape)


def _stream(e, max_e, solved, X=None, piv=None, erased=None, ru=None, nr=None, n_union=76, T=1200, bi=1):
    """Runs rq_debug_gi_stream for block bi of a 3-block stream poisoned with 0xDEADBEEF; returns (words of
    the whole buffer, layout dict)."""
    import ctypes
    lay = np.zeros(7, np.uint32)
    L = rqhip.lib()
    P = lambda a: a.ctypes.data if a is not None else None
    # size first (the layout depends on max_e only): a buffer too small is refused before any write
    probe = np.zeros(1, np.uint32)
    rc = L.rq_debug_gi_stream(e, max_e, 0, None, None, None, None, 0, n_union, T, 0, probe.ctypes.data, 0,
                              lay.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    assert rc != 0 and probe[0] == 0
    block = int(lay[6])
    out = np.full(3 * block, 0xDEADBEEF, np.uint32)
    rqhip._check(L.rq_debug_gi_stream(e, max_e, 1 if solved else 0, P(X), P(piv), P(erased), P(ru), nr or 0, n_union,
                                      T, bi, out.ctypes.data, out.size,
                                      lay.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    names = ("nslm", "ngrm", "er", "of", "ix", "ix_slice", "block")
    return out, dict(zip(names, (int(x) for x in lay)))


def _random_block(rng, e, nr, K=1024, n_union=76):
    X = rng.integers(0, 256, (e, e), dtype=np.uint8)
    X[rng.random((e, e)) < 0.1] = 0                    # zeros and all-zero groups occur in real X
    piv = rng.permutation(nr)[:e].astype(np.uint16)
    erased = np.sort(rng.choice(K, e, replace=False)).astype(np.uint32)
    ru = np.sort(rng.choice(n_union, nr, replace=False)).astype(np.uint32)
    return np.ascontiguousarray(X), piv, erased, ru


@pytest.mark.parametrize("e,max_e", [(1, 1), (4, 9), (5, 5), (6, 64), (8, 8), (9, 70), (63, 64), (64, 128),
                                     (65, 65), (127, 300), (128, 128), (129, 512), (307, 307), (512, 512)])
def test_stream_indices_stay_in_the_table(e, max_e):
    """Every subset number the stream holds is < 2^G (the apply indexes a 2^G-entry VGPR table with it), every
    row offset points at a received row / an r0 row / an erased row of the block, and nothing is written
    outside the block's own part of the stream."""
    rng = np.random.default_rng(e * 1000 + max_e)
    n_union = max(76, e + 8)
    nr = min(n_union, e + 8)
    T = 1200
    X, piv, erased, ru = _random_block(rng, e, nr, n_union=n_union)
    out, L = _stream(e, max_e, True, X, piv, erased, ru, nr, n_union, T)
    blk = L["block"]
    assert (out[:blk] == 0xDEADBEEF).all() and (out[2 * blk:] == 0xDEADBEEF).all()
    b = out[blk:2 * blk]
    ngr, nsl = -(-e // G), -(-e // KC)
    assert list(b[:3]) == [1, e, ngr]
    # slices' output rows: E[k] * T, 0 past e
    er = b[L["er"]:L["er"] + 16 * nsl].reshape(nsl, 16)
    for sl in range(nsl):
        for k in range(16):
            ko = sl * KC + k
            assert er[sl, k] == (int(erased[ko]) * T if k < KC and ko < e else 0)
    # groups' (received row, r0 row) offsets, PDG + 1 records past the last group for the look-ahead
    of = b[L["of"]:L["of"] + 16 * (ngr + PDG + 1)].reshape(ngr + PDG + 1, 16)
    for q in range(ngr + PDG + 1):
        for t in range(8):
            m = G * q + t
            want = (int(piv[m]) * T, int(ru[piv[m]]) * T) if t < G and m < e else (0, 0)
            assert (of[q, 2 * t], of[q, 2 * t + 1]) == want
    assert (of[:, 2 * G:] == 0).all()
    # the index records: per slice, group, output, bit: the G-bit subset of the group's coefficients
    ix = b[L["ix"]:].reshape(L["nslm"], L["ix_slice"])
    for sl in range(nsl):
        rec = ix[sl, :ngr * 8 * KC].reshape(ngr, KC, 8)
        assert int(rec.max(initial=0)) < (1 << G)
        for g in range(ngr):
            for k in range(KC):
                ko = sl * KC + k
                for bit in range(8):
                    want = 0
                    for t in range(G):
                        m = G * g + t
                        if ko < e and m < e and (int(X[ko, m]) >> bit) & 1:
                            want |= 1 << t
                    assert rec[g, k, bit] == want, (sl, g, k, bit)


@pytest.mark.parametrize("e,max_e", [(1, 60), (60, 60), (200, 512)])
def test_stream_unsolved_block_header_only(e, max_e):
    """A block that ends rank-deficient (k_solve_pq when its rows are final, or k_solve) gets status 0 and
    nothing else: the apply kernel reads the header, sees 0 and exits before any index is used."""
    out, L = _stream(e, max_e, False)
    blk = L["block"]
    b = out[blk:2 * blk]
    assert list(b[:3]) == [0, e, -(-e // G)]
    assert (b[16:] == 0xDEADBEEF).all() and (out[:blk] == 0xDEADBEEF).all() and (out[2 * blk:] == 0xDEADBEEF).all()


def _check_text(text, shape=(8, 5, 2, 1)):
    return rqhip.lib().rq_debug_apply_gi_check(*shape, text.encode())


@pytest.mark.parametrize("shape", [(8, 5, 2, 1), (16, 6, 2, 1), (8, 5, 2, 2), (8, 5, 2, 1 | 256), (4, 4, 1, 2),
                                   (12, 5, 1, 1), (8, 4, 1, 1)])
def test_index_mode_guard_passes_generated_kernels(shape):
    text, _ = rqhip.apply_gi_asm(*shape[:3], cpl=shape[3] & 255, pack=shape[3] >> 8, assemble=False)
    assert _check_text(text, shape) == 0, rqhip.lib().rq_last_error()


def test_index_mode_guard_catches_violations():
    """The guard refuses what the round-5 fault (M0 written by SALU moves) and its relatives would do: an M0
    write, an indexed read that is not a table base, another VALU or a memory instruction inside a region,
    a DST-indexed mode, an unclosed region."""
    text, _ = rqhip.apply_gi_asm(8, 5, 2, cpl=1, assemble=False)
    lines = text.split("\n")
    first_on = next(i for i, l in enumerate(lines) if "s_set_gpr_idx_on" in l)
    first_xor = next(i for i in range(first_on, len(lines)) if "v_xor_b32_e32" in lines[i])
    m = re.match(r"\s*v_xor_b32_e32 v(\d+), v(\d+), v(\d+)", lines[first_xor])
    d, tb = int(m.group(1)), int(m.group(2))
    bad = {
        "m0 write": lines[:first_on + 1] + ["\ts_mov_b32 m0, s5"] + lines[first_on + 1:],
        "m0 write outside": lines[:3] + ["\ts_mov_b32 m0, 0"] + lines[3:],
        "not a table base": lines[:first_xor] + ["\tv_xor_b32_e32 v%d, v%d, v%d" % (d, tb + 1, d)] + lines[first_xor + 1:],
        "other VALU": lines[:first_xor] + ["\tv_perm_b32 v%d, v%d, v%d, s36" % (d, tb, d)] + lines[first_xor:],
        "memory": lines[:first_xor] + ["\tbuffer_load_dword v2, v1, s[48:51], s0 offen"] + lines[first_xor:],
        "dst mode": [l.replace("gpr_idx(SRC0)", "gpr_idx(SRC0,DST)") for l in lines],
        "unclosed": [l for l in lines if "s_set_gpr_idx_off" not in l],
        "into the table": lines[:first_xor] + ["\tv_xor_b32_e32 v%d, v%d, v%d" % (tb + 3, tb, tb + 3)] + lines[first_xor + 1:],
    }
    for name, ls in bad.items():
        assert _check_text("\n".join(ls)) != 0, name
