"""Instruction-fetch micro-benchmark generator (gfx950).

Emits straight-line kernels of N VALU instructions over v0..v(R-1) (the shape of a compiled
per-K' column program) and a looped kernel of the same dynamic instruction count, so the cost
of streaming a >64 KiB instruction footprint through the instruction cache can be measured
against an i-cache-resident loop.  Usage: python ifetch_gen.py OUTDIR
"""
import os
import random
import subprocess
import sys

HDR = """\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
\t.amdhsa_code_object_version 6
\t.text
"""


def kernel(name, body, nvgpr=512, accum=256):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:"]
    s += body
    s += ["\ts_endpgm", f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    kd = f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size 0
\t\t.amdhsa_private_segment_fixed_size 0
\t\t.amdhsa_kernarg_size 16
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_sgpr_workgroup_id_y 0
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr {nvgpr}
\t\t.amdhsa_next_free_sgpr 16
\t\t.amdhsa_accum_offset {accum}
\t\t.amdhsa_reserve_vcc 0
\t\t.amdhsa_ieee_mode 0
\t\t.amdhsa_dx10_clamp 0
\t.end_amdhsa_kernel
\t.text
"""
    return "\n".join(s) + "\n" + kd


def meta(names, nvgpr):
    ks = []
    for n in names:
        ks.append(f"""  - .agpr_count: 256
    .args:
      - .offset: 0
        .size: 8
        .value_kind: global_buffer
        .address_space: global
      - .offset: 8
        .size: 4
        .value_kind: by_value
    .group_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 64
    .name: {n}
    .private_segment_fixed_size: 0
    .sgpr_count: 16
    .symbol: {n}.kd
    .vgpr_count: {nvgpr}
    .wavefront_size: 64""")
    return "\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "\n".join(ks) + \
        "\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n"


def valu(rng, R):
    d, a, b, c = (rng.randrange(2, R) for _ in range(4))
    return f"\tv_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96"


def store(R):
    # out[wave*64 + lane] = v2 ^ ... (keeps the work live)
    return ["\ts_load_dwordx2 s[4:5], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)",
            "\tv_lshlrev_b32 v0, 2, v0", "\ts_lshl_b32 s6, s2, 8", "\tv_add_u32 v0, s6, v0",
            "\tv_xor_b32 v1, v2, v3", "\tglobal_store_dword v0, v1, s[4:5]"]


def init(R):
    return [f"\tv_mov_b32 v{r}, {r}" for r in range(1, R)]


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    rng = random.Random(1)
    R = 256
    N = 20000
    names = []
    src = HDR
    # straight-line N
    body = init(R) + [valu(rng, R) for _ in range(N)] + store(R)
    src += kernel("k_line", body); names.append("k_line")
    # loop: 64-instruction body x (N/64)
    body = init(R) + ["\ts_mov_b32 s8, %d" % (N // 64), ".Lloop:"] + [valu(rng, R) for _ in range(64)] + \
        ["\ts_sub_u32 s8, s8, 1", "\ts_cmp_lg_u32 s8, 0", "\ts_cbranch_scc1 .Lloop"] + store(R)
    src += kernel("k_loop", body); names.append("k_loop")
    # straight-line with 2-byte-cheaper VOP2 xors (4-byte encodings)
    body = init(R)
    for _ in range(N):
        d, a, b = (rng.randrange(2, R) for _ in range(3))
        body.append(f"\tv_xor_b32 v{d}, v{a}, v{b}")
    body += store(R)
    src += kernel("k_line4", body); names.append("k_line4")
    src += meta(names, 512)
    with open(os.path.join(out, "ifetch.s"), "w") as f:
        f.write(src)
    clang = "/opt/rocm/llvm/bin/clang"
    subprocess.run([clang, "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    os.path.join(out, "ifetch.s"), "-o", os.path.join(out, "ifetch.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "ifetch.o"), "-o",
                    os.path.join(out, "ifetch.hsaco")], check=True)
    print("ok", os.path.join(out, "ifetch.hsaco"))


if __name__ == "__main__":
    main()
