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


def replay_waves(wave, plan, src_rows, K, H):
    """Emulate k_encode's wave streams (paged segments, paired statements A|B, Horner pieces)."""
    Kp, L = plan["Kp"], plan["L"]
    T = src_rows.shape[1]
    Td = T // 4
    words = wave["words"]
    sd = int(wave.get("sd", 0))  # sd > 0: slot fields are LDS dword offsets (slot * sd)

    def S(f):
        if not sd:
            return f
        assert f % sd == 0, "slot offset not a multiple of the strip width"
        return f // sd

    src32 = np.ascontiguousarray(src_rows).view(np.uint32).reshape(Kp, Td).copy()
    src32[K:] = 0
    slots = np.zeros((wave["n_slots"], Td), np.uint32)
    for i in range(K):
        slots[plan["load_slot"][i]] = src32[i]
    nw = wave["n_waves"]
    page = [int(o) for o in wave["wave_off"]]
    pos = [0] * nw
    ht = [[np.zeros(Td, np.uint32), np.zeros(Td, np.uint32)] for _ in range(nw)]
    for _lv in range(wave["n_levels"]):
        for w in range(nw):
            def F():
                assert pos[w] < 64, "segment crosses a page"
                v = int(words[page[w] + pos[w]])
                pos[w] += 1
                return v
            while True:
                nops = F()
                for _ in range(nops):
                    hdr = F()
                    ty, n = hdr & 7, hdr >> 16
                    dd = F()
                    g = (F(), F()) if hdr & 32 else (0xFFFFFFFF, 0xFFFFFFFF)
                    if ty == ST_XOR:
                        body = [F() for _ in range(n)]
                    elif ty == ST_MUL:
                        body = [(F(), F()) for _ in range(n)]
                    elif ty == ST_SCALE:
                        body = F()
                    else:
                        body = [(F(), F()) for _ in range(n)]
                        nt = (H + 3) // 4
                        taus = ([F() for _ in range(nt)], [F() for _ in range(nt)]) if hdr & 128 else None
                    for half in (0, 1):
                        dst = S((dd >> 16) if half else (dd & 0xFFFF))
                        acc = (hdr >> (4 if half else 3)) & 1
                        pk = (lambda x: S(x >> 16)) if half else (lambda x: S(x & 0xFFFF))
                        if ty == ST_XOR:
                            v = slots[dst].copy() if acc else np.zeros(Td, np.uint32)
                            gi = g[half]
                            if gi != 0xFFFFFFFF and gi < K:
                                v ^= src32[gi]
                            for x in body:
                                v ^= slots[pk(x)]
                            slots[dst] = v
                        elif ty == ST_MUL:
                            v = slots[dst].copy() if acc else np.zeros(Td, np.uint32)
                            for x, c in body:
                                v ^= gfmul4(slots[pk(x)], (c >> 8) & 0xFF if half else c & 0xFF)
                            slots[dst] = v
                        elif ty == ST_SCALE:
                            slots[dst] = gfmul4(slots[dst], (body >> 8) & 0xFF if half else body & 0xFF)
                        else:
                            if hdr & 64:
                                ht[w][half] = np.zeros(Td, np.uint32)
                                slots[dst:dst + H] = 0
                            t = ht[w][half]
                            for ea, eb in body:
                                e = eb if half else ea
                                sl = e & 0xFFFF
                                t = xtime4(t) ^ (slots[S(sl)] if sl != 0xFFFF else 0)
                                if (e >> 26) & 1:
                                    for h in range(H):
                                        slots[dst + h] ^= gfmul4(t, ALPHA_POW[h])
                                else:
                                    slots[dst + ((e >> 16) & 31)] ^= t
                                    slots[dst + ((e >> 21) & 31)] ^= t
                            ht[w][half] = t
                            if taus is not None:
                                tw = taus[half]
                                for h in range(H):
                                    slots[dst + h] ^= gfmul4(t, (tw[h // 4] >> (8 * (h & 3))) & 0xFF)
                nx = F()
                if nx & 2:
                    page[w] += 64
                    pos[w] = 0
                if nx & 1:
                    break
    return slots[plan["col_slot"].astype(np.int64)].view(np.uint8).reshape(L, T)
