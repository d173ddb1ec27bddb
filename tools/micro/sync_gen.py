"""Barrier-aligned row loads (gfx950): a workgroup of 4 waves (one per SIMD) reads the column program's
source pattern for 4 adjacent 64-column items of one block -- wave w reads its 256 B of each row with
one buffer_load_dword, so together they read 1 KiB of the row -- with D loads in flight and V VALU per
load, as load_gen.py.  B > 0: an s_barrier every B loads keeps the four waves at the same row, so the
four 256-B pieces of a row reach the memory system together (DRAM row-buffer locality), with no LDS and
no data exchange.  Same bytes as coop_gen.py (1 228 workgroups x 1 MiB).
Usage: python sync_gen.py OUTDIR; loadrun_wg OUTDIR/sync.hsaco k_b0_d16_v20 ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK  # noqa: E402
from coop_gen import meta  # noqa: E402


def kernel(name, D, V, B):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         "\ts_cmp_lt_u32 s2, 1024", "\ts_cselect_b32 s12, 0, 176", "\ts_and_b32 s11, s2, 1023",
         "\ts_mul_i32 s10, s11, %d" % BLK, "\ts_add_u32 s10, s10, s12",
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshlrev_b32_e32 v1, 2, v0",                 # thread t of 256: byte 4t of the 1 KiB row chunk
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0"]
    for i in range(ROWS):
        row = (i * 389) % ROWS
        r = 10 + (i % D)
        if i >= D:
            s.append(f"\ts_waitcnt vmcnt({D - 1})")
            for _ in range(V):
                s.append(f"\tv_bitop3_b32 v2, v2, v{r}, v3 bitop3:0x96")
        if B and i % B == 0 and i:
            s.append("\ts_barrier")
        s.append(f"\ts_mov_b32 s24, {row * T}")
        s.append(f"\tbuffer_load_dword v{r}, v1, s[20:23], s24 offen")
    s += ["\ts_waitcnt vmcnt(0)", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 10",
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
    names, src, lds = [], HDR, {}
    for B in (0, 4, 16, 64):
        for V in (1, 24):
            n = f"k_b{B}_d16_v{V}"
            src += kernel(n, 16, V, B)
            names.append(n)
            lds[n] = 0
    src += meta(names, lds)
    with open(os.path.join(out, "sync.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "sync.s"), "-o", os.path.join(out, "sync.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "sync.o"), "-o",
                    os.path.join(out, "sync.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
