#!/usr/bin/env python3
"""bench.py -- RaptorQ encode+decode throughput on MI355X (BASELINE.json metric).

Metric: "RaptorQ encode+decode GB/s device-resident, K=1024 T=1200B, 1/2/4/8 MI355X".
Workload (BASELINE.json configs[2]; per-GPU shard of configs[3]): one step = encode every block of
the batch (K=1024, T=1200, N=1100 -> 76 repair symbols per block), then decode every block after
erasing exactly 5% of its N symbols (55, a seeded uniform subset).
value = source bytes (n_blocks * K * T, all ranks) / (encode + decode wall time, max over ranks).
Inputs are resident in HBM when the timed region starts; the erasure pattern's descriptor arrays
are host arrays prepared once and uploaded by every decode call (part of the timed work).

roofline: the dominant kernel is the encode column program (rq_colprog_K1024_n76).  achieved =
algorithmic bytes per launch (K*T source bytes per block x blocks, SURVEY.md sec. 8d: the HBM-read
roofline) / its mean launch time, measured with HIP events recorded on the launch stream inside the
timed region; traffic = FETCH_SIZE + WRITE_SIZE of one launch from the committed rocprofv3 PMC
passes of this exact workload (profiles/rNN_traffic.json, tools/gpu_profile.sh), else null.

Multi-GPU: one process per GPU (torch.distributed); each rank owns `--blocks` independent blocks
(weak scaling, no data-path collective: blocks are independent).  The only
collectives are the timing barrier and the max-over-ranks reduction (rqshard.max_over_ranks).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402
import rqshard  # noqa: E402

METRIC = "RaptorQ encode+decode GB/s device-resident, K=1024 T=1200B, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1024, help="blocks per GPU")
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--T", type=int, default=1200)
    ap.add_argument("--N", type=int, default=1100)
    ap.add_argument("--erase", type=float, default=0.05)
    ap.add_argument("--cpu-sample", type=int, default=20, help="blocks in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--sync-decode", action="store_true", help="time rq_decode_batch (host sync per step) "
                    "instead of rq_decode_batch_async")
    ap.add_argument("--dist-backend", default="nccl", help="process-group backend for the timing collectives "
                    "(nccl = RCCL; gloo lets several ranks share one GPU for a functional rehearsal)")
    return ap.parse_args()


def erasure_pattern(K, N, n_blocks, n_erase, seed):
    rng = np.random.default_rng(seed)
    er, rep = [], []
    for _ in range(n_blocks):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rep.append([e for e in range(K, N) if e not in lost])
    return er, rep


def pmc_traffic(kernel, K, T, N, B):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this exact
    workload (profiles/rNN_traffic.json, written by tools/gpu_profile.sh); (None, None) if absent."""
    for path in sorted((ROOT / "profiles").glob("r*_traffic.json"), reverse=True):
        t = json.loads(path.read_text())
        if t.get("kernel") == kernel and t.get("workload") == {"K": K, "T": T, "N": N, "blocks": B}:
            return t["traffic_bytes"], path.name
    return None, None


def cpu_block(O, K, T, N, n_erase, seed):
    """One block of the workload through the oracle: (encode + repairs seconds, decode seconds)."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, K * T, dtype=np.uint8).tobytes()
    t0 = time.perf_counter()
    enc = O.OracleEncoder(data, T)
    syms = {i: enc.gen_symbol(i).tobytes() for i in range(K, N)}
    t_enc = time.perf_counter() - t0
    lost = set(rng.choice(N, n_erase, replace=False).tolist())
    dec = O.OracleDecoder(len(data), T)
    for i in range(N):
        if i not in lost:
            dec.add_symbol(i, data[i * T:(i + 1) * T] if i < K else syms[i])
    t0 = time.perf_counter()
    ok, out = dec.decode()
    t_dec = time.perf_counter() - t0
    assert ok and out == data
    return t_enc, t_dec


def cpu_baseline(K, T, N, n_erase, n_blocks):
    """Oracle (C restatement) on a bounded sample of the same workload: 1 thread (the reported value),
    then all host cores with one block per thread (SURVEY.md sec. 8d asks for both)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    t_enc = t_dec = 0.0
    for b in range(n_blocks):
        e, d = cpu_block(O, K, T, N, n_erase, 4242 + b)
        t_enc += e
        t_dec += d
    gbs = n_blocks * K * T / (t_enc + t_dec) / 1e9
    threads = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16 cores
    nb_all = 2 * threads
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:  # the oracle's C calls release the GIL
        list(ex.map(lambda b: cpu_block(O, K, T, N, n_erase, 9000 + b), range(nb_all)))
    t_all = time.perf_counter() - t0
    return {"value": round(gbs, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "%d blocks K=%d T=%d N=%d, %d of N erased; oracle/rq_oracle.c (dense-Gauss C restatement, "
                      "1 thread): encode+repairs %.2f s, decode %.2f s" % (n_blocks, K, T, N, n_erase, t_enc, t_dec),
            "all_cores": {"value": round(nb_all * K * T / t_all / 1e9, 6), "unit": "GB/s", "cores": threads,
                          "sample": "%d blocks, one per thread, %.2f s wall" % (nb_all, t_all)}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group(args.dist_backend)
        dist = tdist
    gpu = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    rqhip.lib().rq_set_device(gpu)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    K, T, N, B = args.K, args.T, args.N, args.blocks
    R = N - K
    n_erase = int(round(args.erase * N))
    esis = list(range(K, N))
    g = torch.Generator(device=dev).manual_seed(rqshard.block_seed(rank * B))
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev, generator=g)
    rep = torch.empty((B, R * T), dtype=torch.uint8, device=dev)
    er, rl = erasure_pattern(K, N, B, n_erase, 7 + rank)
    # received repair rows (decode input, gathered once) and the decoder's working copy of the data
    rb = torch.tensor([b for b in range(B) for _ in rl[b]], device=dev, dtype=torch.long)
    rr = torch.tensor([e - K for b in range(B) for e in rl[b]], device=dev, dtype=torch.long)
    data = src.clone()
    db = rqhip.DecodeBatch(K, T, er, rl)
    stream = torch.cuda.current_stream(dev)

    # correctness of one full step before timing: every block recovered bit-exactly
    rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
    recv = rep.view(B, R, T)[rb, rr].contiguous()
    eb = torch.tensor([b for b in range(B) for _ in er[b]], device=dev, dtype=torch.long)
    ei = torch.tensor([i for b in range(B) for i in er[b]], device=dev, dtype=torch.long)
    data.view(B, K, T)[eb, ei] = 0xA5  # garbage in the erased rows
    st = db.run(data, recv, stream=stream)
    torch.cuda.synchronize()
    ok_frac = float((st == 1).mean())
    if not args.no_verify:
        good = torch.tensor(st == 1, device=dev)
        assert torch.equal(data[good], src[good]), "decode mismatch"

    # timed path: rq_decode_batch_async (statuses land in pinned memory; no host sync per step)
    for _ in range(args.warmup):
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        (db.run if args.sync_decode else db.run_async)(data, recv, stream=stream)
    torch.cuda.synchronize()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        ev[s][1].record(stream)
        st_async = (db.run if args.sync_decode else db.run_async)(data, recv, stream=stream)
        ev[s][2].record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = rqshard.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    assert np.array_equal(st_async, st), "async decode statuses differ"
    enc_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1, _ in ev]))
    dec_ms = float(np.mean([e1.elapsed_time(e2) for _, e1, e2 in ev]))
    total_blocks = rqshard.sum_over_ranks(B, dist, coll_dev)
    value = total_blocks * K * T * args.steps / dt / 1e9
    if rank == 0:
        kname = "rq_colprog_K%d_n%d" % (K, R)
        achieved = B * K * T / (enc_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(kname, K, T, N, B)
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded torch.randint payload per rank, seeded exact-count 5% erasures)",
            "config": {"workload": "encode+decode K=%d T=%d N=%d, erase %d of %d symbols per block" % (K, T, N, n_erase, N),
                       "blocks_per_gpu": B, "bytes_per_gpu": B * K * T, "parallelism": "block-sharded x%d" % world,
                       "decode_ok_fraction": ok_frac, "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4)},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "algorithmic_bytes_per_launch": B * K * T,
                         "launch_ms": round(enc_ms, 4)},
        }
        if args.cpu_sample > 0 and world == 1:
            line["cpu_baseline"] = cpu_baseline(K, T, N, n_erase, args.cpu_sample)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
