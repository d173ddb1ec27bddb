"""Four-rows-per-instruction source staging micro-benchmark (gfx950), against load_gen.py's one row
per buffer_load_dword: one buffer_load_dwordx4 ... lds fetches 1 KiB = four scattered 256-B row
segments (lane l: row group l/16, 16 B at (l%16)*16) into an LDS ring of D groups; each row then goes
to a register with ds_read_b32 (lane*4) and feeds V VALU.  Same rows, bytes and VALU per row as
load_gen.py's k_d*_v* kernels (1024 rows x 256 B per wave, 5 waves per block, one wave per SIMD).
Usage: python dma4_gen.py OUTDIR; loadrun OUTDIR/dma4.hsaco k_dma4_d4_v20 ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK, meta  # noqa: E402


def kernel(name, D, V):
    NG = ROWS // 4
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         "\ts_mul_hi_u32 s8, s2, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s2, s9",
         "\ts_lshl_b32 s9, s9, 8", "\ts_mul_i32 s10, s8, %d" % BLK,
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshlrev_b32_e32 v1, 2, v0",                                   # lane*4: LDS read address
         "\tv_and_b32_e32 v4, 15, v0", "\tv_lshlrev_b32_e32 v4, 4, v4", "\tv_add_u32_e32 v4, s9, v4",  # chunk base
         "\tv_lshrrev_b32_e32 v5, 4, v0",                                   # row group g
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", f"\ts_mov_b32 s12, {T}"]

    def dma(j):
        slot = j % D
        return [f"\tv_add_u32_e32 v6, {4 * j}, v5",                        # 4j + g
                "\tv_mul_u32_u24_e32 v6, 389, v6", "\tv_and_b32_e32 v6, 1023, v6",
                "\tv_mad_u32_u24 v6, v6, s12, v4",                               # row * T + chunk base
                f"\ts_mov_b32 m0, {slot * 1024}", "\ts_nop 0",
                "\tbuffer_load_dwordx4 v6, s[20:23], 0 offen lds"]

    for j in range(min(D, NG)):
        s += dma(j)
    for j in range(NG):
        # group j landed once at most D-1 younger DMAs are outstanding
        out = min(D - 1, NG - 1 - j)
        s.append(f"\ts_waitcnt vmcnt({out})")
        slot = j % D
        for g in range(4):
            r = 10 + g
            s.append(f"\tds_read_b32 v{r}, v1 offset:{slot * 1024 + g * 256}")
        for g in range(4):
            r = 10 + g
            s.append(f"\ts_waitcnt lgkmcnt({3 - g})")
            for _ in range(V):
                s.append(f"\tv_bitop3_b32 v2, v2, v{r}, v3 bitop3:0x96")
        if j + D < NG:
            s += dma(j + D)  # the ring slot of group j is free again (its rows are in registers)
    s += ["\ts_waitcnt vmcnt(0) lgkmcnt(0)", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    kd = f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size {D * 1024}
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
    for D in (4, 8, 16):
        for V in (1, 20):
            n = f"k_dma4_d{D}_v{V}"
            src += kernel(n, D, V)
            names.append(n)
    m = meta(names)
    src += m.replace(".group_segment_fixed_size: 0", ".group_segment_fixed_size: 16384")
    with open(os.path.join(out, "dma4.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "dma4.s"), "-o", os.path.join(out, "dma4.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "dma4.o"), "-o",
                    os.path.join(out, "dma4.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
