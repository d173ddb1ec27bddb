"""Cooperative row staging micro-benchmark (gfx950): a workgroup of 4 waves (one per SIMD) works on 4
adjacent 64-column items (256 dword columns) of a block.  At each staging point every wave issues ONE
buffer_load_dwordx4 ... lds of 1 KiB -- its own row of the point's 4 rows, the WG's 256 columns of it,
contiguous -- into a shared LDS ring; an s_barrier after each wave's vmcnt wait publishes a point D
points later; every wave then reads its 256-B part of each row with ds_read_b32 and runs V VALU.
Same rows, bytes and VALU per row per wave as load_gen.py's k_d*_v* kernels.
Usage: python coop_gen.py OUTDIR; loadrun_wg OUTDIR/coop.hsaco k_coop_d4_v20 ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK  # noqa: E402


def kernel(name, D, V, G):
    """D: points in flight; G: ring groups (4 rows = 4 KiB each), G >= D + 1."""
    NP = ROWS // 4
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         # workgroup g < 1024: block g, row bytes [0, 1024); g >= 1024: block g - 1024, bytes [176, 1200)
         # (1 228 workgroups x 1 MiB ~ the 1.26 GB of load_gen's grid)
         "\ts_cmp_lt_u32 s2, 1024", "\ts_cselect_b32 s12, 0, 176", "\ts_and_b32 s11, s2, 1023",
         "\ts_mul_i32 s10, s11, %d" % BLK, "\ts_add_u32 s10, s10, s12",
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshrrev_b32_e32 v5, 6, v0",                 # wave id w
         "\tv_and_b32_e32 v9, 63, v0",                    # lane
         "\tv_lshlrev_b32_e32 v4, 4, v9",                 # DMA: lane*16 within the 1 KiB row chunk
         "\tv_lshlrev_b32_e32 v1, 2, v9",                 # read: lane*4 ...
         "\tv_lshlrev_b32_e32 v6, 8, v5", "\tv_add_u32_e32 v1, v1, v6",  # ... + w*256
         "\tv_readfirstlane_b32 s13, v5",                 # wave id in an SGPR
         "\ts_lshl_b32 s14, s13, 10",                     # M0 part: w*1024
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0"]

    def dma(p):
        q = p % G
        # wave w loads row (4p + w): soffset = row * T; rows spread like load_gen's order
        out = [f"\ts_lshl_b32 s15, s13, 0", f"\ts_add_u32 s15, s15, {4 * p}",
               "\ts_mul_i32 s15, s15, 389", "\ts_and_b32 s15, s15, 1023", f"\ts_mul_i32 s15, s15, {T}",
               f"\ts_add_u32 m0, s14, {q * 4096}", "\ts_nop 0",
               "\tbuffer_load_dwordx4 v4, s[20:23], s15 offen lds"]
        return out

    for p in range(min(D, NP)):
        s += dma(p)
    for p in range(NP):
        out = min(D - 1, NP - 1 - p)
        s.append(f"\ts_waitcnt vmcnt({out})")
        s.append("\ts_barrier")                          # point p visible to every wave
        q = p % G
        for j in range(4):
            s.append(f"\tds_read_b32 v{10 + j}, v1 offset:{(4 * q + j) * 1024}")
        for j in range(4):
            s.append(f"\ts_waitcnt lgkmcnt({3 - j})")
            for _ in range(V):
                s.append(f"\tv_bitop3_b32 v2, v2, v{10 + j}, v3 bitop3:0x96")
        if p + D < NP:
            # ring group (p + D) % G was last read at point p + D - G <= p - 1: every wave passed the
            # barrier of point p after reading it, so it is free
            s += dma(p + D)
    s += ["\ts_waitcnt vmcnt(0) lgkmcnt(0)", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 10",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    kd = f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size {G * 4096}
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


def meta(names, lds):
    ks = []
    for n in names:
        ks.append(f"""  - .agpr_count: 256
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: {lds[n]}
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 256
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
    names, src, lds = [], HDR, {}
    for D, G in ((4, 6), (8, 10)):
        for V in (1, 20):
            n = f"k_coop_d{D}_v{V}"
            src += kernel(n, D, V, G)
            names.append(n)
            lds[n] = G * 4096
    src += meta(names, lds)
    with open(os.path.join(out, "coop.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "coop.s"), "-o", os.path.join(out, "coop.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "coop.o"), "-o",
                    os.path.join(out, "coop.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
