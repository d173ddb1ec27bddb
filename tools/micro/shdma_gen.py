"""Row-shared LDS-DMA micro-benchmark generator (gfx950), round 6.  The question: can the column program's
memory side (the no-XOR build takes 0.264 ms against 0.241 for the no-load build, profiles/r05_micro/
cap_settled.txt: the memory side is the larger cap) run closer to the dwordx4 streaming rate if the four
waves of a CU (one per SIMD, four consecutive 64-column items of the same source rows) fetch each row
once, as ONE buffer_load_dwordx4 ... lds of 1 KiB (lane l: 16 B of item l / 16's 256-B piece), issued by
the four waves in turn, into an LDS ring; every wave then reads its 256-B piece by ds_read_b32.  No VGPR is
held while a row is in flight, so the prefetch can be deep.  Waves synchronise by s_barrier every G rows.
  k_base_d16 / k_base_d32   the program's pattern today: one dword load per row per wave, D in flight
  k_sh_p{P}_g{G}            row-shared DMA, P rows prefetched, barrier every G rows, ring P + G rows
  *_m                       memory side only (no XOR work)      *_v  VALU side only (no memory loads)
Each wave: 5 rounds x 1024 rows (scrambled order) x 20 XOR3 per row.  Grids: base 1024 one-wave
workgroups (WGS=64), shared 256 four-wave workgroups (WGS=256), both one wave per SIMD.
Usage: python shdma_gen.py OUTDIR; GRID=1024 WGS=64 clockrun OUTDIR/shdma_base.hsaco ...;
       GRID=256 WGS=256 clockrun OUTDIR/shdma_sh.hsaco ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from load_gen import HDR, ROWS, T, BLK  # noqa: E402

V = 20
ROUNDS = 5


def perm4(k):  # row order: rows 4 perm4(k) + w for the k-th DMA of wave w (a permutation of the 256 quads)
    return (k * 97) % (ROWS // 4)


def kd(name, nvgpr, lds, wgs):
    return f"""\t.section .rodata,"a",@progbits
\t.p2align 6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size {lds}
\t\t.amdhsa_private_segment_fixed_size 0
\t\t.amdhsa_kernarg_size 16
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr {nvgpr}
\t\t.amdhsa_next_free_sgpr 48
\t\t.amdhsa_accum_offset {min(nvgpr, 256)}
\t\t.amdhsa_reserve_vcc 0
\t\t.amdhsa_ieee_mode 0
\t\t.amdhsa_dx10_clamp 0
\t.end_amdhsa_kernel
\t.text
""", (name, nvgpr, lds, wgs)


def work(r, valu):
    return [f"\tv_bitop3_b32 v{2 + k % 4}, v{2 + k % 4}, v{r}, v{6 + k % 4} bitop3:0x96" for k in range(V)] if valu else []


def base(name, D, mem=True, valu=True):
    """One wave per SIMD, persistent over 5 rounds: wave g takes piece g + 1024 r (5 pieces per block, on one
    XCD: piece -> XCD-aware block / offset), one dword load per row, D in flight."""
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0", "\ts_waitcnt lgkmcnt(0)", "\ts_mov_b32 s15, 0",
         "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000", "\tv_lshlrev_b32_e32 v1, 2, v0",
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", "\tv_mov_b32_e32 v4, 0", "\tv_mov_b32_e32 v5, 0",
         f".Lround_{name}:",
         # piece p = (g % 8) * 640 + (g / 8) + 128 r  (XCD x = g % 8 takes pieces [640 x, 640 x + 640))
         "\ts_and_b32 s8, s2, 7", "\ts_mul_i32 s8, s8, 640", "\ts_lshr_b32 s9, s2, 3", "\ts_add_u32 s8, s8, s9",
         "\ts_mul_i32 s9, s15, 128", "\ts_add_u32 s8, s8, s9",
         "\ts_mul_hi_u32 s9, s8, 0x33333334", "\ts_mul_i32 s10, s9, 5", "\ts_sub_u32 s10, s8, s10",  # block, piece % 5
         "\ts_lshl_b32 s10, s10, 8", f"\ts_mul_i32 s11, s9, {BLK}", "\ts_add_u32 s20, s4, s11", "\ts_addc_u32 s21, s5, 0",
         "\tv_add_u32_e32 v10, s10, v1"]
    if not mem:
        s.append("\tv_mov_b32_e32 v11, v10")
    issued = []
    for i in range(ROWS + D):
        if i >= D:
            j = i - D
            if mem:
                s.append(f"\ts_waitcnt vmcnt({min(len(issued) - 1 - issued.index(j), 63)})")
            s += work(12 + j % D if mem else 11, valu)
        if i < ROWS and mem:
            row = 4 * perm4(i // 4) + i % 4
            s += [f"\ts_mov_b32 s24, {row * T}", f"\tbuffer_load_dword v{12 + i % D}, v10, s[20:23], s24 offen"]
            issued.append(i)
    s += ["\ts_waitcnt vmcnt(0)", "\ts_add_u32 s15, s15, 1", f"\ts_cmp_lt_u32 s15, {ROUNDS}",
          f"\ts_cbranch_scc0 .Ldone_{name}", f"\ts_getpc_b64 s[28:29]", f".Lpc_{name}:",
          f"\ts_sub_u32 s28, s28, .Lpc_{name}-.Lround_{name}", "\ts_subb_u32 s29, s29, 0", "\ts_setpc_b64 s[28:29]",
          f".Ldone_{name}:", "\tv_xor_b32_e32 v2, v2, v3", "\tv_xor_b32_e32 v4, v4, v5", "\tv_xor_b32_e32 v2, v2, v4",
          "\ts_lshl_b32 s11, s2, 8", "\tv_add_u32_e32 v0, s11, v1", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    k, meta = kd(name, 512, 0, 64)
    return "\n".join(s) + "\n" + k, meta


def shared(name, P, G, mem=True, valu=True, AH=4):
    """Four-wave workgroups (one wave per SIMD of a CU), persistent over 5 rounds; per round the workgroup
    takes 4 consecutive pieces; row j is fetched by wave j % 4 as one dwordx4 LDS-DMA (1 KiB) into ring slot
    j % R; every wave reads its 256-B piece of each row by ds_read_b32, AH rows ahead."""
    R = P + G
    assert P % G == 0 and G % 4 == 0 and P // 4 <= 63 and R * 1024 <= 65536
    s = [f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:",
         "\ts_load_dwordx4 s[4:7], s[0:1], 0x0",
         "\tv_lshrrev_b32_e32 v1, 6, v0", "\ts_nop 4", "\tv_readfirstlane_b32 s12, v1",   # s12 = wave w
         "\tv_and_b32_e32 v0, 63, v0", "\ts_waitcnt lgkmcnt(0)", "\ts_mov_b32 s15, 0",
         "\ts_mov_b32 s22, -1", "\ts_mov_b32 s23, 0x20000",
         f"\ts_mul_i32 s13, s12, {T}",                                      # w T (the wave's row within each quad)
         # reader: lane's dword of its wave's 256-B piece in a 1-KiB ring slot; v9 = the same + 64 KiB
         "\tv_lshlrev_b32_e32 v8, 2, v0", "\ts_lshl_b32 s14, s12, 8", "\tv_add_u32_e32 v8, s14, v8",
         "\tv_add_u32_e32 v9, 0x10000, v8",
         "\tv_mov_b32_e32 v2, 0", "\tv_mov_b32_e32 v3, 0", "\tv_mov_b32_e32 v4, 0", "\tv_mov_b32_e32 v5, 0",
         f".Lround_{name}:",
         # workgroup g on XCD g % 8: quad of pieces q = (g % 8) * 160 + g / 8 + 32 r; lane l: piece 4q + l / 16
         "\ts_and_b32 s8, s2, 7", "\ts_mul_i32 s8, s8, 160", "\ts_lshr_b32 s9, s2, 3", "\ts_add_u32 s8, s8, s9",
         "\ts_mul_i32 s9, s15, 32", "\ts_add_u32 s8, s8, s9", "\ts_lshl_b32 s8, s8, 2",
         "\tv_lshrrev_b32_e32 v1, 4, v0", "\tv_add_u32_e32 v1, s8, v1",                       # piece
         "\ts_mov_b32 s26, 0x33333334", f"\ts_mov_b32 s27, {BLK}",
         "\tv_mul_hi_u32 v6, v1, s26", "\tv_mul_lo_u32 v7, v6, 5", "\tv_sub_u32_e32 v7, v1, v7",  # block, piece % 5
         "\tv_lshlrev_b32_e32 v7, 8, v7", "\tv_mul_lo_u32 v6, v6, s27", "\tv_add_u32_e32 v7, v6, v7",
         "\tv_and_b32_e32 v6, 15, v0", "\tv_lshlrev_b32_e32 v6, 4, v6", "\tv_add_u32_e32 v10, v7, v6",  # DMA address
         "\ts_mov_b32 s20, s4", "\ts_and_b32 s21, s5, 0xffff"]
    if not valu:
        pass
    n_dma_own = ROWS // 4
    issued = [0]  # DMAs this wave has issued

    def dma(j):  # the k-th DMA of every wave: rows 4 perm4(k) + w, slot = (4 k + w) % R; uniform code
        k = j // 4
        slot = (4 * k) % R  # + w: per-wave, folded into M0 by s12 * 1024
        if not mem:
            return []
        issued[0] += 1
        return [f"\ts_add_u32 s24, s13, {4 * perm4(k) * T}",
                f"\ts_lshl_b32 s25, s12, 10", f"\ts_add_u32 m0, s25, {slot * 1024}", "\ts_nop 0",
                "\tbuffer_load_dwordx4 v10, s[20:23], s24 offen lds"]

    def read(j):  # ds_read of row j's slot, this wave's piece
        slot = j % R
        base = "v8" if slot < 64 else "v9"
        return [f"\tds_read_b32 v{12 + j % 8}, {base} offset:{(slot % 64) * 1024}"]

    # every wave issues the DMA of rows 4k + w for k over quads; quad k covers rows [4k, 4k + 4)
    for k in range(P // 4):
        s += dma(4 * k)
    for m in range(ROWS // G):
        lo, hi = m * G, m * G + G
        need = min(hi, ROWS) // 4
        if mem:
            s.append(f"\ts_waitcnt vmcnt({issued[0] - need})")
        s += ["\ts_waitcnt lgkmcnt(0)", "\ts_barrier"]
        for j in range(P + lo, min(P + hi, ROWS), 4):
            s += dma(j)
        # consume rows lo..hi-1: reads AH ahead within the group
        for j in range(lo, min(lo + AH, hi)):
            s += read(j)
        for j in range(lo, hi):
            if j + AH < hi:
                s += read(j + AH)
            s.append(f"\ts_waitcnt lgkmcnt({min(AH, hi - 1 - j)})")
            s += work(12 + j % 8, valu)
    s += ["\ts_waitcnt vmcnt(0) lgkmcnt(0)", "\ts_barrier", "\ts_add_u32 s15, s15, 1", f"\ts_cmp_lt_u32 s15, {ROUNDS}",
          f"\ts_cbranch_scc0 .Ldone_{name}", f"\ts_getpc_b64 s[28:29]", f".Lpc_{name}:",
          f"\ts_sub_u32 s28, s28, .Lpc_{name}-.Lround_{name}", "\ts_subb_u32 s29, s29, 0", "\ts_setpc_b64 s[28:29]",
          f".Ldone_{name}:", "\tv_xor_b32_e32 v2, v2, v3", "\tv_xor_b32_e32 v4, v4, v5", "\tv_xor_b32_e32 v2, v2, v4",
          "\ts_lshl_b32 s11, s2, 10", "\tv_lshlrev_b32_e32 v0, 2, v0", "\ts_lshl_b32 s14, s12, 8", "\tv_add_u32_e32 v0, s14, v0",
          "\tv_add_u32_e32 v0, s11, v0", "\tglobal_store_dword v0, v2, s[6:7]", "\ts_endpgm",
          f".Lend_{name}:", f"\t.size {name}, .Lend_{name}-{name}"]
    k, meta = kd(name, 512, R * 1024, 256)
    return "\n".join(s) + "\n" + k, meta


def metadata(ms):
    out = []
    for n, nv, lds, wgs in ms:
        out.append(f"""  - .agpr_count: {nv - 256 if nv > 256 else 0}
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: {lds}
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: {wgs}
    .name: {n}
    .private_segment_fixed_size: 0
    .sgpr_count: 48
    .symbol: {n}.kd
    .vgpr_count: {nv}
    .wavefront_size: 64""")
    return "\t.amdgpu_metadata\n---\namdhsa.kernels:\n" + "\n".join(out) + \
        "\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata\n"


def build(out, tag, kernels):
    src, ms = HDR, []
    for text, meta in kernels:
        src += text
        ms.append(meta)
    src += metadata(ms)
    p = os.path.join(out, tag)
    with open(p + ".s", "w") as f:
        f.write(src)
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", p + ".s", "-o", p + ".o"], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", p + ".o", "-o", p + ".hsaco"], check=True)
    return [m[0] for m in ms]


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    b = build(out, "shdma_base", [base("k_base_d16", 16), base("k_base_d32", 32), base("k_base_d16_m", 16, valu=False),
                                  base("k_base_d16_v", 16, mem=False)])
    sh = []
    for P, G in ((24, 8), (32, 16), (48, 16), (32, 32)):  # rings of 32..64 rows (64 KiB: M0-safe)
        sh.append(shared(f"k_sh_p{P}_g{G}", P, G))
        sh.append(shared(f"k_sh_p{P}_g{G}_m", P, G, valu=False))
    sh.append(shared("k_sh_p48_g16_v", 48, 16, mem=False))
    s = build(out, "shdma_sh", sh)
    print("BASE", " ".join(b))
    print("SH", " ".join(s))


if __name__ == "__main__":
    main()
