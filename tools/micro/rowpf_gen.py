"""Whole-row prefetch micro-benchmark generator (gfx950).  The column program's waves read 256-B pieces of
1200-B source rows (one item = 64 dword columns; the 5 items of a block run the same row order at about
the same time on one XCD), and that pattern saturates at ~4.8 TB/s where 1 KiB contiguous reads reach
6.5 (profiles/r02_micro).  Here each of a block's 5 waves also fetches every 5th upcoming row whole --
one buffer_load_dwordx4 ... lds (1 KiB) + one buffer_load_dword ... lds (256 B) into a dummy LDS area,
PF loads ahead -- so the row comes from HBM in one contiguous burst and the five 256-B loads hit L2.
Kernels (random source bytes, XOR3 work like clock_gen.py):
  k_base_v{V}      the plain pattern, D=16 loads in flight, V VALU per load
  k_pf{PF}_v{V}    the same plus the whole-row prefetch PF loads ahead
Usage: python rowpf_gen.py OUTDIR; clockrun OUTDIR/rowpf.hsaco (also k_base: XCD-aware) NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK  # noqa: E402


def kernel(name, D, V, PF):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         # XCD-aware: workgroup g runs on XCD g % 8; its index there g / 8 -> block-local b = idx / 5, w = idx % 5,
         # block = 8 b + g % 8, so a block's five waves share one XCD (and its L2), as in the column program
         "\ts_lshr_b32 s13, s2, 3", "\ts_and_b32 s14, s2, 7",
         "\ts_mul_hi_u32 s8, s13, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s13, s9",  # s9 = w
         "\ts_lshl_b32 s8, s8, 3", "\ts_add_u32 s8, s8, s14",
         "\ts_lshl_b32 s12, s9, 8", "\ts_mul_i32 s10, s8, %d" % BLK,
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s12, v1",
         "\tv_lshlrev_b32_e32 v6, 4, v0",                       # prefetch: lane * 16
         "\tv_lshlrev_b32_e32 v7, 2, v0", "\tv_add_u32_e32 v7, 0x400, v7",  # tail: 1024 + lane * 4
         "\ts_mov_b32 m0, 0",
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", "\tv_mov_b32_e32 v4, 0", "\tv_mov_b32_e32 v5, 0"]
    ops = []  # issued vector-memory operations: load index or -1 (prefetch)
    for i in range(ROWS):
        row = (i * 389) % ROWS
        r = 10 + (i % D)
        if i >= D:
            after = len(ops) - 1 - ops.index(i - D)  # operations issued after load i - D
            s.append(f"\ts_waitcnt vmcnt({min(after, 63)})")
            for k in range(V):
                a = 2 + (k % 4)
                s.append(f"\tv_bitop3_b32 v{a}, v{a}, v{r}, v{10 + (i + k) % D} bitop3:0x96")
        if PF and i % 5 == 0 and i + PF + 4 < ROWS:
            # wave w prefetches the row of load i + PF + w: ((i + PF + w) * 389 % 1024) * T
            s += [f"\ts_add_u32 s25, s9, {i + PF}", "\ts_mul_i32 s25, s25, 389", "\ts_and_b32 s25, s25, 1023",
                  f"\ts_mul_i32 s25, s25, {T}",
                  "\tbuffer_load_dwordx4 v6, s[20:23], s25 offen lds",
                  "\tbuffer_load_dword v7, s[20:23], s25 offen lds"]
            ops += [-1, -1]
        s.append(f"\ts_mov_b32 s24, {row * T}")
        s.append(f"\tbuffer_load_dword v{r}, v1, s[20:23], s24 offen")
        ops.append(i)
    s += ["\ts_waitcnt vmcnt(0)", "\tv_xor_b32_e32 v2, v2, v3", "\tv_xor_b32_e32 v4, v4, v5",
          "\tv_xor_b32_e32 v2, v2, v4", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    kd = f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size 2048
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


def meta(names):
    ks = []
    for n in names:
        ks.append(f"""  - .agpr_count: 256
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: 2048
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 64
    .name: {n}
    .private_segment_fixed_size: 0
    .sgpr_count: 32
    .symbol: {n}.kd
    .vgpr_count: 512
    .wavefront_size: 64""")
    return "\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "\n".join(ks) + \
        "\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n"


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    names, src = [], HDR
    for V in (1, 20):
        for PF in (0, 20, 40, 80):
            n = f"k_pf{PF}_v{V}" if PF else f"k_base_v{V}"
            src += kernel(n, 16, V, PF)
            names.append(n)
    src += meta(names)
    with open(os.path.join(out, "rowpf.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "rowpf.s"), "-o", os.path.join(out, "rowpf.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "rowpf.o"), "-o",
                    os.path.join(out, "rowpf.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
