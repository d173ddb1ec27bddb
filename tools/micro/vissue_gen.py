"""VALU issue-rate micro-benchmark generator (gfx950): why does one wave per SIMD of the column program
take ~5.2 shader cycles per instruction (profiles/r05b) instead of 4?  Candidates: instruction fetch of a
~175 KB straight-line program, VGPR bank conflicts of three-operand v_bitop3, AGPR moves.  Every kernel
runs N VALU instructions per wave on registers only (no memory until the final store); grid 1024 = one
wave per SIMD.
  k_sl_spread   straight line, v_bitop3 XOR3, operands spread like the program (mixed banks)
  k_loop_spread the same 200-instruction body looped (code stays in the instruction cache)
  k_sl_bank4    straight line, dst and the three sources in four different banks (reg % 4)
  k_sl_bank1    straight line, the three sources in one bank
  k_loop_bank1  looped, three sources in one bank
  k_sl_vop2     straight line v_xor_b32_e32 (4-byte encoding)
  k_loop_vop2   looped v_xor_b32_e32
  k_sl_acc      straight line, one v_accvgpr_write + one v_accvgpr_read per two XOR3
  k_loop_acc    looped, the same mix
Usage: python vissue_gen.py OUTDIR; clockrun-style runner: vissuerun OUTDIR/vissue.hsaco NAMES..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, meta  # noqa: E402

N = int(os.environ.get("VI_N", "20000"))
BODY = 200


def body(kind, n, seed):
    out = []
    x = seed
    for i in range(n):
        x = (x * 1103515245 + 12345) & 0x7FFFFFFF
        a, b, c = 8 + (x >> 4) % 200, 8 + (x >> 12) % 200, 8 + (x >> 20) % 200
        d = 8 + (i * 7) % 200
        if kind == "spread":
            out.append(f"\tv_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96")
        elif kind == "bank4":  # d % 4 = 0, a % 4 = 1, b % 4 = 2, c % 4 = 3
            out.append(f"\tv_bitop3_b32 v{d - d % 4}, v{a - a % 4 + 1}, v{b - b % 4 + 2}, v{c - c % 4 + 3} bitop3:0x96")
        elif kind == "bank1":  # three sources in bank 1
            out.append(f"\tv_bitop3_b32 v{d - d % 4}, v{a - a % 4 + 1}, v{b - b % 4 + 1}, v{c - c % 4 + 1} bitop3:0x96")
        elif kind == "bop2":  # v_bitop3 with two distinct sources (c = b)
            out.append(f"\tv_bitop3_b32 v{d}, v{a}, v{b}, v{b} bitop3:0x96")
        elif kind == "e64":  # v_xor_b32 in the 8-byte VOP3 encoding
            out.append(f"\tv_xor_b32_e64 v{d}, v{a}, v{b}")
        elif kind == "vop2":
            out.append(f"\tv_xor_b32_e32 v{d}, v{a}, v{b}")
        elif kind == "acc":
            if i % 4 == 0:
                out.append(f"\tv_accvgpr_write_b32 a{(i >> 2) % 200}, v{a}")
            elif i % 4 == 1:
                out.append(f"\tv_accvgpr_read_b32 v{d}, a{(i * 5) % 200}")
            else:
                out.append(f"\tv_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96")
    return out


def kernel(name, kind, loop):
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)"]
    for r in range(8, 208):
        s.append(f"\tv_add_u32_e32 v{r}, {r * 0x9E37 & 0x7fff}, v0")
    if kind == "acc":
        for r in range(200):
            s.append(f"\tv_accvgpr_write_b32 a{r}, v{8 + r}")
    if loop:
        s += [f"\ts_mov_b32 s12, {N // BODY}", f".Lloop_{name}:"]
        s += body(kind, BODY, 7)
        s += ["\ts_sub_u32 s12, s12, 1", "\ts_cmp_lg_u32 s12, 0", f"\ts_cbranch_scc1 .Lloop_{name}"]
    else:
        s += body(kind, N, 7)
    s += ["\tv_xor_b32_e32 v1, v8, v9", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s11, s2, 8",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v1, s[6:7]", "\ts_endpgm",
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
    for kind, loop in (("spread", 0), ("spread", 1), ("bank4", 0), ("bank4", 1), ("bank1", 0), ("bank1", 1),
                       ("vop2", 0), ("vop2", 1), ("acc", 0), ("acc", 1),
                       ("bop2", 0), ("bop2", 1), ("e64", 0), ("e64", 1)):
        n = f"k_{'loop' if loop else 'sl'}_{kind}"
        src += kernel(n, kind, loop)
        names.append(n)
    src += meta(names)
    with open(os.path.join(out, "vissue.s"), "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", os.path.join(out, "vissue.s"), "-o", os.path.join(out, "vissue.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "vissue.o"), "-o",
                    os.path.join(out, "vissue.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
