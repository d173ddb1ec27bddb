"""Clock / power micro-benchmark generator (gfx950): is the column program's lost memory/VALU overlap a
clock effect?  Kernels in the shape of load_gen.py (one wave per SIMD, the encode program's 256-B source
pattern, 5 waves per block, D loads in flight, V VALU per load) whose VALU work differs only in how many
bits it toggles:
  k_xor_d16_v{V}   v_bitop3 XOR3 chains over the loaded (random) data -- the program's kind of work
  k_and_d16_v{V}   the same instruction count as v_bitop3 AND with zero (result constant: little toggling)
  k_xor_nold_v{V}  XOR3 work with the loads replaced by v_mov (issue only, no memory)
  k_and_nold_v{V}  AND work, no memory
Run under rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT to read each kernel's effective shader clock.
Usage: python clock_gen.py OUTDIR; clockrun OUTDIR/clock.hsaco NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK, meta  # noqa: E402


def kernel(name, D, V, op, loads=True):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         "\ts_mul_hi_u32 s8, s2, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s2, s9",
         "\ts_lshl_b32 s9, s9, 8", "\ts_mul_i32 s10, s8, %d" % BLK,
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s9, v1",
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", "\tv_mov_b32_e32 v4, 0", "\tv_mov_b32_e32 v5, 0", "\tv_mov_b32_e32 v9, 0"]
    # four independent accumulators (v2..v5) so the data stream, not one chain, toggles
    for i in range(ROWS):
        row = (i * 389) % ROWS
        r = 10 + (i % D)
        if i >= D:
            if loads:
                s.append(f"\ts_waitcnt vmcnt({D - 1})")
            for k in range(V):
                a = 2 + (k % 4)
                if op == "xor":
                    s.append(f"\tv_bitop3_b32 v{a}, v{a}, v{r}, v{10 + (i + k) % D} bitop3:0x96")
                else:  # AND with v3-equivalent zero register v9: result stays 0
                    s.append(f"\tv_bitop3_b32 v{a}, v9, v{r}, v{10 + (i + k) % D} bitop3:0x80")
        if loads:
            s.append(f"\ts_mov_b32 s24, {row * T}")
            s.append(f"\tbuffer_load_dword v{r}, v1, s[20:23], s24 offen")
        else:
            s.append(f"\tv_xor_b32_e32 v{r}, v1, v{10 + (i + 1) % D}")
    s += ["\ts_waitcnt vmcnt(0)", "\tv_xor_b32_e32 v2, v2, v3", "\tv_xor_b32_e32 v4, v4, v5",
          "\tv_xor_b32_e32 v2, v2, v4", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
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
    for V in (1, 20):
        for op in ("xor", "and"):
            n = f"k_{op}_d16_v{V}"
            src += kernel(n, 16, V, op)
            names.append(n)
    for op in ("xor", "and"):
        n = f"k_{op}_nold_v20"
        src += kernel(n, 16, 20, op, loads=False)
        names.append(n)
    src += meta(names)
    with open(os.path.join(out, "clock.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "clock.s"), "-o", os.path.join(out, "clock.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "clock.o"), "-o",
                    os.path.join(out, "clock.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
