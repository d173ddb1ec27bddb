"""GPU probes used by the round-3 experiments (run.sh's `py` step): one file, one subcommand each.

  python tools/experiments/probes.py perobj          per-object round trips vs the oracle (K=5, L=1100)
  python tools/experiments/probes.py host_enqueue    cost of the bench's timing events and host enqueue
  python tools/experiments/probes.py encode_position encode launch by position in the step / buffer
  python tools/experiments/probes.py encode_position2 encode launch in three step shapes
  python tools/experiments/probes.py out_offset      encode launch by the output buffer's placement
  python tools/experiments/probes.py launch_order    column-program launch after an apply vs after itself

Set RQHIP_LIB to probe another library build."""
import os
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402

if os.environ.get("RQHIP_LIB"):
    rqhip.LIB_PATH = Path(os.environ["RQHIP_LIB"])

K3, T3, N3, B3 = 1024, 1200, 1100, 1024


def perobj():
    """Per-object round trips (K=5, L=1100, N=8, 10 % loss, 50 trials) through the Python mirror, and
    the encoder's repairs against the oracle: a regression probe for column-program launch changes."""
    from oracle import oracle as O
    rng = random.Random(1337)
    K, L, N = 5, 1100, 8
    bad_rep = bad_dec = ok = 0
    for t in range(50):
        data = bytes(rng.getrandbits(8) for _ in range(K * L - (t % 7) * 13))
        enc = rqhip.NewRaptorQEncoder(data, K, L)
        ref = O.OracleEncoder(data, L)
        for i in range(N):
            if bytes(enc.GenSymbol(i)) != bytes(ref.gen_symbol(i)):
                bad_rep += 1
        pk = rqhip.RaptorQEncodeBlock(data, N, K, L)
        recv = [p for p in pk if rng.random() >= 0.1]
        got, okf = rqhip.RaptorQDecodeBytes(recv, N, K, L, len(data))
        if okf:
            ok += 1
            bad_dec += bytes(got) != data
    print("trials 50 ok %d bad_repair_symbols %d bad_decodes %d" % (ok, bad_rep, bad_dec))


def _config3():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 256, (B3, K3 * T3), dtype=torch.uint8, device=dev)
    rep = torch.empty((B3, (N3 - K3) * T3), dtype=torch.uint8, device=dev)
    er, rl = bench.erasure_pattern(K3, N3, B3, 55, 7)
    rb = torch.tensor([b for b in range(B3) for _ in rl[b]], device=dev, dtype=torch.long)
    rr = torch.tensor([e - K3 for b in range(B3) for e in rl[b]], device=dev, dtype=torch.long)
    data = src.clone()
    db = rqhip.DecodeBatch(K3, T3, er, rl)
    esis = list(range(K3, N3))
    s = torch.cuda.current_stream(dev)
    rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
    recv = rep.view(B3, N3 - K3, T3)[rb, rr].contiguous()
    return torch, src, rep, data, db, esis, s, recv


def host_enqueue():
    """Wall ms per config-3 step with the bench's three timing events per step, one, and none; and the
    pure host time of one encode_batch / run_async call on an idle device."""
    torch, src, rep, data, db, esis, s, recv = _config3()
    S = 30

    def loop(n_ev):
        for _ in range(3):
            rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
            db.run_async(data, recv, stream=s)
        torch.cuda.synchronize()
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(S)]
        t0 = time.perf_counter()
        for i in range(S):
            if n_ev >= 1:
                ev[i][0].record(s)
            rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
            if n_ev >= 3:
                ev[i][1].record(s)
            db.run_async(data, recv, stream=s)
            if n_ev >= 3:
                ev[i][2].record(s)
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / S

    for n_ev in (3, 0, 1, 3, 0):
        print("events per step %d: %.4f ms per step" % (n_ev, loop(n_ev)), flush=True)
    he, hd = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        a = time.perf_counter()
        rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
        b = time.perf_counter()
        torch.cuda.synchronize()
        c = time.perf_counter()
        db.run_async(data, recv, stream=s)
        d = time.perf_counter()
        he.append(b - a)
        hd.append(d - c)
    print("host ms per call on an idle device: encode %.3f, decode %.3f (min %.3f)" %
          (1e3 * sum(he) / 10, 1e3 * sum(hd) / 10, 1e3 * min(hd)))


def encode_position():
    """Step = encode(src), encode(src), encode(data), decode, 12 times (run under a kernel trace)."""
    torch, src, rep, data, db, esis, s, recv = _config3()
    rep2 = torch.empty_like(rep)
    for _ in range(12):
        rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
        rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
        rqhip.encode_batch(data, K3, T3, esis, rep2, stream=s)
        db.run_async(data, recv, stream=s)
    torch.cuda.synchronize()
    print("done")


def encode_position2():
    """[encode, decode] x 12 with the bench's buffers, with alternating outputs, and with the encode
    reading the decode's data buffer (run under a kernel trace); PROBE_INTERLEAVE=1 rotates the three
    modes step by step instead."""
    torch, src, rep, data, db, esis, s, recv = _config3()
    rep2 = torch.empty_like(rep)
    interleave = os.environ.get("PROBE_INTERLEAVE") == "1"  # modes rotate per step (no clock drift)
    order = [i % 3 for i in range(36)] if interleave else [m for m in range(3) for _ in range(12)]
    idle = os.environ.get("PROBE_IDLE") == "1"  # mode 1 instead: the bench's buffers, 2 ms idle before the encode
    for i, mode in enumerate(order):
        if idle and mode == 1:
            torch.cuda.synchronize()
            time.sleep(0.002)
        a = data if mode == 2 else src
        o = (rep2 if i % 2 else rep) if mode == 1 and not idle else rep
        rqhip.encode_batch(a, K3, T3, esis, o, stream=s)
        db.run_async(data, recv, stream=s)
    torch.cuda.synchronize()
    print("done")


def out_offset():
    """[encode, decode] steps with the encode's output buffer placed at byte offsets 0 / 256 / 4 KiB /
    64 KiB / 1 MiB / 2 MiB + 4 KiB into one allocation, offsets rotating step by step (run under a
    kernel trace): does the output's placement relative to the source change the launch?"""
    torch, src, rep, data, db, esis, s, recv = _config3()
    offs = [0, 256, 4096, 65536, 1 << 20, (2 << 20) + 4096]
    n = rep.numel()
    big = torch.empty(n + max(offs), dtype=torch.uint8, device=src.device)
    print("src %#x data %#x rep %#x big %#x" % (src.data_ptr(), data.data_ptr(), rep.data_ptr(), big.data_ptr()))
    outs = [big[o:o + n].view(rep.shape) for o in offs]
    for i in range(6 * 8):
        rqhip.encode_batch(src, K3, T3, esis, outs[i % 6], stream=s)
        db.run_async(data, recv, stream=s)
    torch.cuda.synchronize()
    assert torch.equal(outs[(6 * 8 - 1) % 6], rep)  # the views overlap: only the last one written is whole
    print("done")


def launch_order():
    """Alternating steps A = [encode(src -> rep), decode, decode] and B = [encode(src -> rep),
    encode(src -> rep2), decode], 12 of each (run under a kernel trace): the column program's time
    after an apply against after another column-program launch, for both the encode and the syndrome."""
    torch, src, rep, data, db, esis, s, recv = _config3()
    rep2 = torch.empty_like(rep)
    if os.environ.get("PROBE_WARM") == "1":  # A becomes [256 MiB device copy, encode, decode, decode]
        wa = torch.empty(256 << 20, dtype=torch.uint8, device=src.device)
        wb = torch.empty_like(wa)
    for i in range(24):
        if os.environ.get("PROBE_WARM") == "1" and i % 2 == 0:
            with torch.cuda.stream(s):
                wb.copy_(wa)
        rqhip.encode_batch(src, K3, T3, esis, rep, stream=s)
        if i % 2:
            rqhip.encode_batch(src, K3, T3, esis, rep2, stream=s)
            db.run_async(data, recv, stream=s)
        else:
            db.run_async(data, recv, stream=s)
            db.run_async(data, recv, stream=s)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    cmds = {f.__name__: f for f in (perobj, host_enqueue, encode_position, encode_position2, out_offset, launch_order)}
    if len(sys.argv) != 2 or sys.argv[1] not in cmds:
        raise SystemExit("usage: probes.py {%s}" % "|".join(cmds))
    cmds[sys.argv[1]]()
