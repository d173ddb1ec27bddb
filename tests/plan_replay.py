"""Host-side (numpy) interpreter of an exported rqhip encode plan -- test infrastructure.

Executes the straight-line statement program exactly as k_encode does (rq_kernels.hip), one
uint32 column vector per slot, so the CPU suite can check the schedule compiler against the
oracle without a GPU.
"""
import numpy as np

ST_XOR, ST_MUL, ST_SCALE, ST_HORNER = 0, 1, 3, 4
ALPHA_POW = [1, 2, 4, 8, 16, 32, 64, 128, 29, 58, 116, 232, 205, 135, 19, 38]


def xtime4(x):
    hi = (x >> 7) & np.uint32(0x01010101)
    return ((x & np.uint32(0x7F7F7F7F)) << np.uint32(1)) ^ (hi * np.uint32(0x1D))


def gfmul4(x, c):
    r = np.zeros_like(x)
    for b in range(8):
        if (c >> b) & 1:
            r ^= x
        x = xtime4(x)
    return r


def replay(plan, src_rows, K, H, erased=()):
    """src_rows: (K', T) uint8 (rows >= K ignored).  Returns C as (L, T) uint8."""
    Kp, L = plan["Kp"], plan["L"]
    T = src_rows.shape[1]
    Td = T // 4
    words, so, lv = plan["words"], plan["stmt_off"], plan["level_start"]
    n_slots = int(max(int(plan["col_slot"].max()), int(plan["load_slot"].max()))) + 1
    n_slots = max(n_slots, L + 16 * H + 128)
    src32 = np.ascontiguousarray(src_rows).view(np.uint32).reshape(Kp, Td).copy()
    er = set(int(e) for e in erased)
    for i in range(Kp):
        if i >= K or i in er:
            src32[i] = 0
    slots = np.zeros((n_slots, Td), np.uint32)
    for i in range(K):
        if i not in er:
            slots[plan["load_slot"][i]] = src32[i]

    def fetch(sw):
        if sw >> 31:
            return src32[sw & 0xFFFFFF]
        return slots[sw & 0xFFFF]

    for s in range(len(so) - 1):
        o = int(so[s])
        w0 = int(words[o])
        dst, ns, ty, acc = w0 & 0xFFFF, (w0 >> 16) & 0xFFF, (w0 >> 28) & 7, w0 >> 31
        if ty == ST_XOR:
            v = slots[dst].copy() if acc else np.zeros(Td, np.uint32)
            for k in range(ns):
                v ^= fetch(int(words[o + 1 + k]))
            slots[dst] = v
        elif ty == ST_MUL:
            v = slots[dst].copy() if acc else np.zeros(Td, np.uint32)
            for k in range(ns):
                sw = int(words[o + 1 + k])
                v ^= gfmul4(fetch(sw), (sw >> 16) & 0xFF)
            slots[dst] = v
        elif ty == ST_SCALE:
            slots[dst] = gfmul4(slots[dst], int(words[o + 1]))
        elif ty == ST_HORNER:
            P = np.zeros((H, Td), np.uint32)
            t = np.zeros(Td, np.uint32)
            for j in range(ns):
                e = int(words[o + 1 + j])
                sl = e & 0xFFFF
                t = xtime4(t) ^ (slots[sl] if sl != 0xFFFF else 0)
                if (e >> 26) & 1:
                    for h in range(H):
                        P[h] ^= gfmul4(t, ALPHA_POW[h])
                else:
                    P[(e >> 16) & 31] ^= t
                    P[(e >> 21) & 31] ^= t
            for h in range(H):
                tau = (int(words[o + 1 + ns + h // 4]) >> (8 * (h & 3))) & 0xFF
                P[h] ^= gfmul4(t, tau)
            slots[dst:dst + H] = P
        else:
            raise ValueError("bad statement type %d" % ty)
    C32 = slots[plan["col_slot"].astype(np.int64)]
    return C32.view(np.uint8).reshape(L, T)


OP_XOR, OP_MUL, OP_HORNER, OP_END = 0, 1, 4, 7
FLAG_G, FLAG_HSTART, FLAG_HFINISH, FLAG_BARRIER, FLAG_ADVANCE = 1 << 5, 1 << 6, 1 << 7, 1 << 8, 1 << 9


def gfmul4_tab(x, t):
    """v_perm table multiply (rq_kernels.hip gfmul4_tab) on uint32 arrays."""
    def perm(hi, lo, sel):
        tab = np.array([(lo >> (8 * i)) & 0xFF for i in range(4)] + [(hi >> (8 * i)) & 0xFF for i in range(4)], np.uint32)
        out = np.zeros_like(sel)
        for b in range(4):
            out |= tab[(sel >> (8 * b)) & 0xFF] << (8 * b)
        return out
    s0, s1, s2 = x & 0x07070707, (x >> 3) & 0x07070707, (x >> 6) & 0x03030303
    return perm(t[1], t[0], s0) ^ perm(t[3], t[2], s1) ^ perm(t[4], t[4], s2)


def replay_waves(wave, plan, src_rows, K, H):
    """Emulate k_encode's wave streams (rq_wave_format.hpp): pages of 8-word groups, half A/B
    words, byte-offset slot fields, END barriers; waves run level by level."""
    Kp, L = plan["Kp"], plan["L"]
    T = src_rows.shape[1]
    Td = T // 4
    words = wave["words"]
    sd = int(wave["sd"])
    row_bytes = sd * 4

    def S(off):
        assert off % row_bytes == 0, "slot offset not a multiple of the strip row"
        return off // row_bytes

    src32 = np.ascontiguousarray(src_rows).view(np.uint32).reshape(Kp, Td).copy()
    src32[K:] = 0
    slots = np.zeros((wave["n_slots"], Td), np.uint32)
    for i in range(K):
        slots[plan["load_slot"][i]] = src32[i]
    nw = wave["n_waves"]
    gpos = [int(o) for o in wave["wave_off"]]  # word index of the next group
    hstate = [None] * nw
    for _lv in range(wave["n_levels"]):
        for w in range(nw):
            def G():
                g = [int(x) for x in words[gpos[w]:gpos[w] + 8]]
                gpos[w] += 8
                return g
            while True:
                h = G()
                hdr = h[0]
                assert h[4] == hdr
                ty, n = hdr & 7, hdr >> 16
                if ty == OP_END:
                    if hdr & FLAG_ADVANCE:
                        gpos[w] = (gpos[w] + 63) // 64 * 64
                    if hdr & FLAG_BARRIER:
                        break
                    continue
                start = gpos[w] - 8
                span = 8 * (n + 1 + (1 if ty == OP_HORNER and hdr & FLAG_HFINISH else 0))
                assert start // 64 == (start + span + 8 - 1) // 64, "op (and a closing END) cross a page"
                body = [G() for _ in range(n)]
                if ty == OP_HORNER:
                    tau = G()[:4] if hdr & FLAG_HFINISH else None
                    dst = S(h[1])
                    if hdr & FLAG_HSTART:
                        hstate[w] = [np.zeros(Td, np.uint32), np.zeros((16, Td), np.uint32)]
                    t, hp = hstate[w]
                    for g in body:
                        for e in g:
                            t = xtime4(t) ^ slots[S(e & 0x3FFFF)]
                            hp[(e >> 18) & 15] ^= t
                            hp[(e >> 22) & 15] ^= t
                    hstate[w] = [t, hp]
                    if tau is not None:
                        for hh in range(H):
                            slots[dst + hh] = hp[hh] ^ gfmul4(t, (tau[hh // 4] >> (8 * (hh & 3))) & 0xFF)
                    continue
                res = []
                for half in (0, 1):
                    o = 4 * half
                    v = np.zeros(Td, np.uint32)
                    gi = h[o + 2]
                    if hdr & FLAG_G and gi != 0xFFFFFFFF and gi < K:
                        v ^= src32[gi]
                    if ty == OP_XOR:
                        for g in body:
                            for e in g[o:o + 4]:
                                v ^= slots[S(e)]
                    else:
                        for k in range(0, n, 2):
                            g1, g2 = body[k], body[k + 1]
                            v ^= gfmul4_tab(slots[S(g1[o])], (g1[o + 1], g1[o + 2], g1[o + 3], g2[o], g2[o + 1]))
                    res.append((S(h[o + 1]), v))
                for d, v in res:
                    slots[d] = v
    return slots[plan["col_slot"].astype(np.int64)].view(np.uint8).reshape(L, T)
