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
