"""VGPR-index-mode micro-benchmark generator (gfx950): can a wave-uniform table lookup in registers
(`s_set_gpr_idx_idx` + a VOP2 XOR whose src0 is indexed) replace the three `v_perm` of a GF(256)
mul-add in k_apply?  gfx950 has no v_movrels; the VGPR index mode of s_set_gpr_idx_on is there.
Every kernel runs NP instruction groups per wave on registers only (one store at the end), 128 VGPRs,
so up to four waves per SIMD: launch GRID = 1024 * W one-wave workgroups for W waves per SIMD.
  k_gi     index mode on; NP x (s_set_gpr_idx_idx s_k; v_xor_b32 acc, v[64 + idx], acc)
  k_gi2    the same with two lookups per index change (two tables 32 registers apart)
  k_x2     NP x v_xor_b32_e32 (VOP2 reference)
  k_sidx   index mode on; NP x s_set_gpr_idx_idx (SALU only)
  k_salu   NP x s_add_u32 (SALU reference)
  k_perm   NP x v_perm_b32 (the current apply's lookup)
  k_mul45  NP/4.5 x (3 v_perm + 1.5 v_bitop3): the current apply's mul-add mix, NP instructions
Usage: python gidx_gen.py OUTDIR; GRID=... WGS=64 clockrun OUTDIR/gidx.hsaco NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, meta  # noqa: E402

NP = int(os.environ.get("GI_NP", "16000"))
BODY = 200


def body(kind):
    out = []
    x = 7
    for i in range(BODY):
        x = (x * 1103515245 + 12345) & 0x7FFFFFFF
        acc = 1 + i % 40
        s = 16 + i % 16
        if kind == "gi":
            out += [f"\ts_set_gpr_idx_idx s{s}", f"\tv_xor_b32_e32 v{acc}, v64, v{acc}"]
        elif kind == "gi2":
            if i % 2 == 0:
                out.append(f"\ts_set_gpr_idx_idx s{s}")
            out.append(f"\tv_xor_b32_e32 v{acc}, v{64 if i % 2 == 0 else 96}, v{acc}")
        elif kind == "x2":
            out.append(f"\tv_xor_b32_e32 v{acc}, v{64 + (x >> 8) % 60}, v{acc}")
        elif kind == "sidx":
            out.append(f"\ts_set_gpr_idx_idx s{s}")
        elif kind == "salu":
            out.append(f"\ts_add_u32 s{32 + i % 8}, s{32 + i % 8}, s{s}")
        elif kind == "perm":
            out.append(f"\tv_perm_b32 v{acc}, v{64 + (x >> 8) % 60}, v{65 + (x >> 16) % 60}, v{41 + i % 20}")
        elif kind == "mul45":  # per 9 instructions: 6 perms + 3 XOR3 (two mul-adds)
            j = i % 9
            if j < 6:
                out.append(f"\tv_perm_b32 v{41 + j}, v{64 + (x >> 8) % 60}, v{65 + (x >> 16) % 60}, v{50 + i % 10}")
            else:
                out.append(f"\tv_bitop3_b32 v{acc}, v{acc}, v{41 + 2 * (j - 6)}, v{42 + 2 * (j - 6)} bitop3:0x96")
    return out


def kernel(name, kind):
    idx = kind in ("gi", "gi2", "sidx")
    nv = 128
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)"]
    for r in range(1, nv):
        s.append(f"\tv_add_u32_e32 v{r}, {r * 0x9E37 & 0x7fff}, v0")
    for k in range(16):
        s.append(f"\ts_mov_b32 s{16 + k}, {(k * 37 + 11) % 30}")
    for k in range(8):
        s.append(f"\ts_mov_b32 s{32 + k}, {k}")
    s += [f"\ts_mov_b32 s12, {max(1, NP // BODY)}"]
    if idx:
        s.append("\ts_set_gpr_idx_on s16, gpr_idx(SRC0)")
    s.append(f".Lloop_{name}:")
    s += body(kind)
    s += ["\ts_sub_u32 s12, s12, 1", "\ts_cmp_lg_u32 s12, 0", f"\ts_cbranch_scc1 .Lloop_{name}"]
    if idx:
        s.append("\ts_set_gpr_idx_off")
    s += ["\tv_xor_b32_e32 v1, v1, v2", "\tv_xor_b32_e32 v1, v1, v3", "\tv_lshlrev_b32_e32 v0, 2, v0",
          "\ts_lshl_b32 s11, s2, 8", "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v1, s[6:7]",
          "\ts_endpgm", f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
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
\t\t.amdhsa_next_free_vgpr {nv}
\t\t.amdhsa_next_free_sgpr 48
\t\t.amdhsa_accum_offset {nv}
\t\t.amdhsa_reserve_vcc 0
\t\t.amdhsa_ieee_mode 0
\t\t.amdhsa_dx10_clamp 0
\t.end_amdhsa_kernel
\t.text
"""
    return "\n".join(s) + "\n" + kd


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    names, src = [], HDR
    for kind in ("gi", "gi2", "x2", "sidx", "salu", "perm", "mul45"):
        n = f"k_{kind}"
        src += kernel(n, kind)
        names.append(n)
    src += meta(names, 128)
    with open(os.path.join(out, "gidx.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "gidx.s"), "-o", os.path.join(out, "gidx.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "gidx.o"), "-o",
                    os.path.join(out, "gidx.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
