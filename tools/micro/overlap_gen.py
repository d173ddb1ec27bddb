"""Memory/VALU overlap micro-benchmark generator (gfx950).  The column program's shape: each wave reads a
256-B piece of each of 1024 source rows (1200-B rows, scrambled order, a block's 5 waves on one XCD) and
runs ~20 VALU per row; memory alone takes ~0.23 ms and VALU alone ~0.24, but together ~0.33
(profiles/r05e).  Variants probe what recovers the overlap:
  k_d{D}_v20       D loads in flight
  k_2w_d16_v20     two waves per SIMD (256 registers each)
  k_vop2_d16       the same XOR work as 40 v_xor_b32_e32 (4-byte encodings) per row
  k_batch4_d16     loads issued four at a time (4 loads, then 4 x 20 VALU)
  k_nt_d16 / k_sc1_d16 / ...   load cache policies (and combinations with batching and D)
  k_wg4_d16        workgroups of 4 waves (a CU's 4 SIMDs take 4 adjacent pieces of the same rows)
Usage: python overlap_gen.py OUTDIR; GRID=... clockrun OUTDIR/overlap.hsaco NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK  # noqa: E402

V = 20


def kernel(name, D=16, nvgpr=512, op="bitop3", batch=1, pol="", wg=1, persist=0):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)"]
    if persist:
        # persistent: grid 1024 x 64 (one wave per SIMD), wave g runs items g, g + 1024, ... (5 rounds); the
        # item's XCD-aware block / piece from its index q as below (q = t * 1024 + g keeps g % 8)
        s += ["\ts_mov_b32 s15, 0", "\ts_mov_b32 s16, s2", "\ts_getpc_b64 s[28:29]", "\ts_mov_b32 s2, s16"]
    if wg == 1:
        # workgroup g on XCD g % 8, index g / 8 there -> block-local b = idx / 5, w = idx % 5, block 8b + g % 8
        s += ["\ts_lshr_b32 s13, s2, 3", "\ts_and_b32 s14, s2, 7",
              "\ts_mul_hi_u32 s8, s13, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s13, s9",
              "\ts_lshl_b32 s8, s8, 3", "\ts_add_u32 s8, s8, s14", "\ts_lshl_b32 s12, s9, 8",
              "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s12, v1"]
    else:
        # 4-wave workgroups of 256 columns (1 KiB of the row): 1280 workgroups, block = g % 1024 (the last
        # 256 workgroups re-read bytes 176.. of blocks 0..255: the same 1.26 GB in total)
        s += ["\ts_and_b32 s8, s2, 1023", "\ts_cmp_lt_u32 s2, 1024", "\ts_cselect_b32 s12, 0, 176",
              "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s12, v1"]
    s += ["\ts_mul_i32 s10, s8, %d" % BLK,
          "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000"]
    if not persist:
        s += ["\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", "\tv_mov_b32_e32 v4, 0", "\tv_mov_b32_e32 v5, 0"]
    ops = []

    def work(i):
        r = 10 + (i % D)
        out = []
        for k in range(V if op == "bitop3" else 2 * V):
            a = 2 + (k % 4)
            if op == "bitop3":
                out.append(f"\tv_bitop3_b32 v{a}, v{a}, v{r}, v{10 + (i + k) % D} bitop3:0x96")
            else:
                out.append(f"\tv_xor_b32_e32 v{a}, v{r if k % 2 == 0 else 10 + (i + k) % D}, v{a}")
        return out

    def load(i):
        ops.append(i)
        return [f"\ts_mov_b32 s24, {((i * 389) % ROWS) * T}",
                f"\tbuffer_load_dword v{10 + (i % D)}, v1, s[20:23], s24 offen{pol}"]

    i = 0
    while i < ROWS:
        grp = list(range(i, min(i + batch, ROWS)))
        for j in grp:
            if j >= D:
                after = len(ops) - 1 - ops.index(j - D)
                s.append(f"\ts_waitcnt vmcnt({min(after, 63)})")
                s += work(j - D)
        for j in grp:
            s += load(j)
        i += batch
    for j in range(ROWS - D, ROWS):
        after = len(ops) - 1 - ops.index(j)
        s.append(f"\ts_waitcnt vmcnt({after})")
        s += work(j)
    if persist:
        s += ["\ts_add_u32 s16, s16, 1024", "\ts_add_u32 s15, s15, 1", f"\ts_cmp_lt_u32 s15, {persist}",
              f"\ts_cbranch_scc0 .Ldone_{name}", "\ts_setpc_b64 s[28:29]", f".Ldone_{name}:", "\ts_and_b32 s2, s16, 1023"]
    s += ["\tv_xor_b32_e32 v2, v2, v3", "\tv_xor_b32_e32 v4, v4, v5",
          "\tv_xor_b32_e32 v2, v2, v4", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 10",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    kd = f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size 0
\t\t.amdhsa_private_segment_fixed_size 0
\t\t.amdhsa_kernarg_size 16
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr {nvgpr}
\t\t.amdhsa_next_free_sgpr 32
\t\t.amdhsa_accum_offset {min(nvgpr, 256)}
\t\t.amdhsa_reserve_vcc 0
\t\t.amdhsa_ieee_mode 0
\t\t.amdhsa_dx10_clamp 0
\t.end_amdhsa_kernel
\t.text
"""
    return "\n".join(s) + "\n" + kd, nvgpr, 64 * wg


def meta(ks):
    out = []
    for n, nv, wgs in ks:
        out.append(f"""  - .agpr_count: {nv - 256 if nv > 256 else 0}
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: {wgs}
    .name: {n}
    .private_segment_fixed_size: 0
    .sgpr_count: 32
    .symbol: {n}.kd
    .vgpr_count: {nv}
    .wavefront_size: 64""")
    return "\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "\n".join(out) + \
        "\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n"


PERSIST = {  # grid 1024
    "k_p_d16": dict(persist=5), "k_p_nt_d16": dict(persist=5, pol=" nt"), "k_p_ntsc1_d16": dict(persist=5, pol=" nt sc1"),
    "k_p_batch4_d16": dict(persist=5, batch=4), "k_p_d32": dict(persist=5, D=32), "k_p_nt_d32": dict(persist=5, D=32, pol=" nt"),
}
VARIANTS = {
    "k_d8_v20": dict(D=8), "k_d12_v20": dict(D=12), "k_d16_v20": dict(D=16), "k_d24_v20": dict(D=24),
    "k_d32_v20": dict(D=32), "k_2w_d16_v20": dict(D=16, nvgpr=256), "k_vop2_d16": dict(op="vop2"),
    "k_batch4_d16": dict(batch=4), "k_nt_d16": dict(pol=" nt"), "k_sc1_d16": dict(pol=" sc1"),
    "k_nt_batch4_d16": dict(pol=" nt", batch=4), "k_nt_d24": dict(D=24, pol=" nt"), "k_nt_d32": dict(D=32, pol=" nt"),
    "k_nt_d12": dict(D=12, pol=" nt"), "k_sc0_d16": dict(pol=" sc0"), "k_sc0sc1_d16": dict(pol=" sc0 sc1"),
    "k_ntsc1_d16": dict(pol=" nt sc1"), "k_ntsc0_d16": dict(pol=" nt sc0"), "k_nt_batch8_d16": dict(pol=" nt", batch=8),
    "k_batch8_d16": dict(batch=8), "k_nt_2w_d16": dict(pol=" nt", nvgpr=256),
}
WG4 = {"k_wg4_d16": dict(wg=4)}


def build(out, variants, tag):
    src, ks = HDR, []
    for n, kw in variants.items():
        text, nv, wgs = kernel(n, **kw)
        src += text
        ks.append((n, nv, wgs))
    src += meta(ks)
    with open(os.path.join(out, f"{tag}.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, f"{tag}.s"), "-o", os.path.join(out, f"{tag}.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, f"{tag}.o"), "-o",
                    os.path.join(out, f"{tag}.hsaco")], check=True)


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    build(out, VARIANTS, "overlap")
    build(out, WG4, "overlap_wg4")
    build(out, PERSIST, "overlap_p")
    print(" ".join(VARIANTS))


if __name__ == "__main__":
    main()
