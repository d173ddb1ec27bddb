"""VALU dependency micro-benchmark generator (gfx950): what one wave per SIMD sustains on
independent XORs, on one dependent chain, and on the column program's xtime sequence as one chain
(the Horner scan) or several interleaved chains.  Usage: python dep_gen.py OUTDIR, then
modrun OUTDIR/dep.hsaco GRID k_indep k_chain ...  (N instructions per kernel: time/N = cycles per
instruction at the measured clock)."""
import os
import random
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ifetch_gen import HDR, kernel, meta, init, store  # noqa: E402

N = 20000


def xtime(d, a, b=None, t1=250, t2=251):
    # the emitter's 5-VALU alpha*a (^ b): s36 = 0x090b080a, s37 = 0xfefefefe, s38 = 0x1d1d1d1d
    out = [f"\tv_lshlrev_b32_e32 v{t1}, 8, v{a}", f"\tv_perm_b32 v{t1}, v{t1}, v{a}, s12"]
    out.append(f"\tv_and_b32_e32 v{t1}, s14, v{t1}" if b is None else f"\tv_bitop3_b32 v{t1}, v{t1}, v{b}, s14 bitop3:0x6c")
    out += [f"\tv_lshlrev_b32_e32 v{t2}, 1, v{a}", f"\tv_bitop3_b32 v{d}, v{t2}, v{t1}, s13 bitop3:0x6c"]
    return out


def consts():
    return ["\ts_mov_b32 s12, 0x090b080a", "\ts_mov_b32 s13, 0xfefefefe", "\ts_mov_b32 s14, 0x1d1d1d1d"]


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    rng = random.Random(1)
    R = 240
    names, src = [], HDR
    pre = init(R) + consts()

    def add(name, body):
        nonlocal src
        src += kernel(name, pre + body + store(R))
        names.append(name)

    add("k_indep", [f"\tv_bitop3_b32 v{rng.randrange(2, R)}, v{rng.randrange(2, R)}, v{rng.randrange(2, R)}, "
                    f"v{rng.randrange(2, R)} bitop3:0x96" for _ in range(N)])
    add("k_chain", [f"\tv_bitop3_b32 v2, v2, v{rng.randrange(3, R)}, v{rng.randrange(3, R)} bitop3:0x96"
                    for _ in range(N)])
    body = []
    for _ in range(N // 5):
        body += xtime(2, 2, rng.randrange(3, R))
    add("k_xt_chain", body)
    for nc in (2, 4):
        body = []
        for _ in range(N // (5 * nc)):
            seqs = [xtime(2 + c, 2 + c, rng.randrange(10, R), t1=240 + 2 * c, t2=241 + 2 * c) for c in range(nc)]
            for i in range(5):
                for c in range(nc):
                    body.append(seqs[c][i])
        add("k_xt_%dchains" % nc, body)
    # one chain + independent pushes (the Horner column: xtime then two accumulator XORs)
    body = []
    for _ in range(N // 6):
        body += xtime(2, 2, rng.randrange(10, R))
        body.append(f"\tv_bitop3_b32 v{rng.randrange(10, R)}, v{rng.randrange(10, R)}, v2, v{rng.randrange(10, R)} bitop3:0x96")
    add("k_horner", body)
    body = []
    for _ in range(N // 2):
        a, r = rng.randrange(0, 200), rng.randrange(10, R)
        body += [f"\tv_accvgpr_write_b32 a{a}, v{r}", f"\tv_accvgpr_read_b32 v{rng.randrange(10, R)}, a{(a + 37) % 200}"]
    add("k_acc", body)
    # instruction kinds at one vs two waves per SIMD (the _2w kernels use 256 registers)
    kinds = {
        "bitop3": lambda: f"\tv_bitop3_b32 v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, "
                          f"v{rng.randrange(2, 120)} bitop3:0x96",
        "perm": lambda: f"\tv_perm_b32 v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, "
                        f"v{rng.randrange(2, 120)}",
        "xor": lambda: f"\tv_xor_b32_e32 v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}",
        "fma": lambda: f"\tv_fma_f32 v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, v{rng.randrange(2, 120)}, "
                       f"v{rng.randrange(2, 120)}",
        "lshl": lambda: f"\tv_lshlrev_b32_e32 v{rng.randrange(2, 120)}, 3, v{rng.randrange(2, 120)}",
    }
    two = []
    for kname, gen in kinds.items():
        body = [gen() for _ in range(N)]
        add("k_%s_1w" % kname, body)
        src += kernel("k_%s_2w" % kname, init(120) + consts() + body + store(120), nvgpr=256, accum=256)
        two.append("k_%s_2w" % kname)
    m1 = meta(names, 512)
    m2 = meta(two, 256).replace(".agpr_count: 256", ".agpr_count: 0")
    body2 = m2.split("amdhsa.kernels:\n", 1)[1].split("\namdhsa.target", 1)[0]
    src += m1.replace("\namdhsa.target", "\n" + body2 + "\namdhsa.target", 1)
    names += two
    with open(os.path.join(out, "dep.s"), "w") as f:
        f.write(src)
    clang = "/opt/rocm/llvm/bin/clang"
    subprocess.run([clang, "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                    os.path.join(out, "dep.s"), "-o", os.path.join(out, "dep.o")], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", os.path.join(out, "dep.o"), "-o",
                    os.path.join(out, "dep.hsaco")], check=True)
    print(" ".join(names))


if __name__ == "__main__":
    main()
