"""Decode on config 3 (1 024 blocks K=1024 T=1200, 55 of 1 100 symbols erased) under the experiments
library's solver knobs: statuses and bytes against the source with the erased rows poisoned, then
decode_ms of rq_decode_batch_async over reps x 5 calls.  Run once per knob setting (the knobs are read
once per process); the solver's kernel time comes from a kernel trace around this script."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "rl-quic-raptor_amd"))
import rqhip as rq  # noqa: E402

if os.environ.get("RQHIP_LIB"):
    from pathlib import Path
    rq.LIB_PATH = Path(os.environ["RQHIP_LIB"])


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K, T, N, B, ne = 1024, 1200, 1100, 1024, 55
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, generator=g).to(dev)
    esis = list(range(K, N))
    out = torch.empty((B, (N - K) * T), dtype=torch.uint8, device=dev)
    rq.encode_batch(src, K, T, esis, out)
    rng = np.random.default_rng(5)
    erased, rl, rows = [], [], []
    for b in range(B):
        lost = set(rng.choice(N, ne, replace=False).tolist())
        erased.append(sorted(i for i in lost if i < K))
        r = [e for e in esis if e not in lost]
        rl.append(r)
        rows.extend((b, e - K) for e in r)
    rep = out.view(B, N - K, T)[torch.tensor([b for b, _ in rows], device=dev),
                                torch.tensor([r for _, r in rows], device=dev)].contiguous()
    eb = torch.tensor([b for b in range(B) for _ in erased[b]], device=dev, dtype=torch.long)
    ei = torch.tensor([i for b in range(B) for i in erased[b]], device=dev, dtype=torch.long)
    if os.environ.get("RQ_SOLVE_IP"):  # rq_debug_solve_mode: 1 = the in-place first solver (experiments library)
        rq.solve_mode(int(os.environ["RQ_SOLVE_IP"]))
    if os.environ.get("RQ_SX"):  # rq_debug_apply_sx: syndromes precomputed beside the first solver or not
        rq.apply_sx(int(os.environ["RQ_SX"]))
    db = rq.DecodeBatch(K, T, erased, rl)
    d = src.clone()
    d.view(B, K, T)[eb, ei] = 0xA5
    st = np.array(db.run(d, rep))
    torch.cuda.synchronize()
    print("solved %d/%d, bytes equal source: %s" % ((st == 1).sum(), B, bool(torch.equal(d, src))), flush=True)
    if ((st != 1).any() or not torch.equal(d, src)) and not os.environ.get("RQHIP_SOLVE_DIAG"):
        sys.exit(1)  # (the timing-only diagnostic builds give wrong bytes on purpose)
    s = torch.cuda.current_stream()
    res = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            db.run_async(d, rep, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 5)
    a = np.array(res)
    print("decode_ms median %.4f min %.4f max %.4f" % (np.median(a), a.min(), a.max()), flush=True)


if __name__ == "__main__":
    main()
