"""Outstanding-load micro-benchmark generator (gfx950): one wave per SIMD (512 registers) streams the column
program's source-row pattern (64 lanes x 4 B of each of 1024 rows of a 1200-B-row block, rows in
a scrambled order, 5 waves per block) with D loads in flight (s_waitcnt vmcnt(D-1) before a
register is reused) and one VALU per load.  Measures achieved bandwidth vs D.
Usage: python load_gen.py OUTDIR; loadrun OUTDIR/load.hsaco k_d8 k_d16 ..."""
import os
import subprocess
import sys

HDR = '\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"\n\t.amdhsa_code_object_version 6\n\t.text\n'
ROWS, T, BLK = 1024, 1200, 1024 * 1200


def kernel(name, D, valu_per_load, nvgpr=512, width=1):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
         # wave w: block w / 5, column chunk (w % 5) * 256 (the last chunk of 1200 B is partial)
         "\ts_mul_hi_u32 s8, s2, 0x33333334", "\ts_mul_i32 s9, s8, 5", "\ts_sub_u32 s9, s2, s9",
         "\ts_lshl_b32 s9, s9, 8", "\ts_mul_i32 s10, s8, %d" % BLK,
         "\ts_add_u32 s20, s4, s10", "\ts_addc_u32 s21, s5, 0", "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         "\tv_lshlrev_b32_e32 v1, 2, v0", "\tv_add_u32_e32 v1, s9, v1", "\tv_mov_b32_e32 v2, 0"]
    nl = ROWS // width
    if width > 1:  # lane l reads 4*width bytes at 4*width*l: the same bytes per wave in fewer loads
        s.append(f"\tv_lshlrev_b32_e32 v1, {2 + (width.bit_length() - 1)}, v0")
        s.append("\tv_add_u32_e32 v1, s9, v1")
    for i in range(nl):
        row = (i * 389) % nl
        r = 10 + width * (i % D)
        if i >= D:
            s.append(f"\ts_waitcnt vmcnt({D - 1})")
            for _ in range(valu_per_load):
                s.append(f"\tv_bitop3_b32 v2, v2, v{r}, v3 bitop3:0x96")
        s.append(f"\ts_mov_b32 s24, {row * T * width}")
        op = {1: "buffer_load_dword", 2: "buffer_load_dwordx2", 4: "buffer_load_dwordx4"}[width]
        dst = f"v{r}" if width == 1 else f"v[{r}:{r + width - 1}]"
        s.append(f"\t{op} {dst}, v1, s[20:23], s24 offen")
    s += ["\ts_waitcnt vmcnt(0)", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
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
    return "\n".join(s) + "\n" + kd


def meta(names, nvgpr=512):
    ks = []
    for n in names:
        nv = 256 if n.endswith("_2w") else nvgpr
        ks.append(f"""  - .agpr_count: {nv - 256 if nv > 256 else 0}
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 64
    .name: {n}
    .private_segment_fixed_size: 0
    .sgpr_count: 32
    .symbol: {n}.kd
    .vgpr_count: {nv}
    .wavefront_size: 64""")
    return "\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "\n".join(ks) + \
        "\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n"


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    names, src = [], HDR
    for D in (8, 16, 24, 32, 48, 60):
        for v in (1, 20):
            n = f"k_d{D}_v{v}"
            src += kernel(n, D, v)
            names.append(n)
    for w, v in ((2, 40), (4, 80), (4, 1)):  # same bytes and VALU per byte, fewer (wider) loads
        n = f"k_x{w}_d16_v{v}"
        src += kernel(n, 16, v, width=w)
        names.append(n)
    src += kernel("k_d32_v20_2w", 32, 20, nvgpr=256)  # two waves per SIMD
    names.append("k_d32_v20_2w")
    src += meta(names)
    with open(os.path.join(out, "load.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "load.s"), "-o", os.path.join(out, "load.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "load.o"), "-o",
                    os.path.join(out, "load.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
