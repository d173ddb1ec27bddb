"""Row-order micro-benchmark generator (gfx950): is the column program's memory-only cap (0.268 ms =
4.7 TB/s for 1 024 blocks K=1024 T=1200) set by the scrambled order in which it reads a block's rows?
One wave per SIMD-slot streams its 256-B piece of every row of its block (5 waves per block, 16 loads in
flight, one VALU per load), rows in program-like scrambled order (i * 389 mod 1024) or ascending; waves
mapped to blocks XCD-aware (a block's five waves on one XCD, as the program) or round-robin.
Usage: python order_gen.py OUTDIR; loadrun OUTDIR/order.hsaco NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, meta, ROWS, T, BLK  # noqa: E402

NW = 5120  # loadrun's grid


def kernel(name, seq, xcd, D=16, persist=0):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)"]
    if persist:  # persist waves, each looping over items w, w + persist, ... < NW (the column program's grid)
        s += [f"\ts_cmp_ge_u32 s2, {persist}", f"\ts_cbranch_scc1 .Lend_{name}", "\ts_mov_b32 s30, s2",
              "\ts_mov_b32 s31, s2", f".Lit_{name}:", "\ts_mov_b32 s2, s31"]
    if xcd:  # logical item L = (w % 8) * (NW / 8) + w / 8
        s += ["\ts_and_b32 s12, s2, 7", f"\ts_mul_i32 s12, s12, {NW // 8}", "\ts_lshr_b32 s13, s2, 3",
              "\ts_add_u32 s2, s12, s13"]
    s += ["\ts_mul_hi_u32 s8, s2, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s2, s9",
          "\ts_lshl_b32 s9, s9, 8", f"\ts_mul_i32 s10, s8, {BLK}",
          "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
          "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s9, v1", "\tv_mov_b32_e32 v2, 0"]

    for i in range(ROWS):
        row = i if seq else (i * 389) % ROWS
        r = 10 + (i % D)
        if i >= D:
            s.append(f"\ts_waitcnt vmcnt({D - 1})")
            s.append(f"\tv_xor_b32_e32 v2, v2, v{r}")
        s.append(f"\ts_mov_b32 s24, {row * T}")
        s.append(f"\tbuffer_load_dword v{r}, v1, s[20:23], s24 offen")
    if persist:
        s += ["\ts_getpc_b64 s[34:35]", f".Lpc_{name}:", f"\ts_sub_u32 s34, s34, .Lpc_{name}-.Lit_{name}",
              "\ts_subb_u32 s35, s35, 0", f"\ts_add_u32 s31, s31, {persist}", f"\ts_cmp_lt_u32 s31, {NW}",
              f"\ts_cbranch_scc0 .Ldone_{name}", "\ts_setpc_b64 s[34:35]", f".Ldone_{name}:", "\ts_mov_b32 s2, s30"]
    s += ["\ts_waitcnt vmcnt(0)", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", f".Lend_{name}:", "\ts_endpgm",
          f".Lsz_{name}:", f"\t.size {name}, .Lsz_{name}-{name}"]
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
\t\t.amdhsa_next_free_vgpr 512
\t\t.amdhsa_next_free_sgpr 32
\t\t.amdhsa_accum_offset 256
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
    for seq in (0, 1):
        for xcd in (0, 1):
            for D in (16, 48):
                n = f"k_{'seq' if seq else 'scr'}_{'xcd' if xcd else 'rr'}_d{D}"
                src += kernel(n, seq, xcd, D)
                names.append(n)
    for D in (16, 48):
        n = f"k_scr_xcd_d{D}_p960"
        src += kernel(n, 0, 1, D, persist=960)
        names.append(n)
    src += meta(names)
    with open(os.path.join(out, "order.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "order.s"), "-o", os.path.join(out, "order.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "order.o"), "-o",
                    os.path.join(out, "order.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
