#!/usr/bin/env python3
"""bench.py -- RaptorQ encode+decode throughput on MI355X (BASELINE.json metric).

Metric: "RaptorQ encode+decode GB/s device-resident, K=1024 T=1200B, 1/2/4/8 MI355X".
Workload (BASELINE.json configs[2]; per-GPU shard of configs[3]): one step = encode every block of
the batch (K=1024, T=1200, N=1100 -> 76 repair symbols per block), then decode every block after
erasing exactly 5% of its N symbols (55, a seeded uniform subset).
value = source bytes (n_blocks * K * T, all ranks) / (encode + decode wall time, max over ranks).
Inputs are resident in HBM when the timed region starts; the erasure pattern's descriptor arrays
are host arrays prepared once and uploaded by every decode call (part of the timed work).

roofline: the dominant kernel is the column program (rq_colprog_K1024_n76), launched twice per step:
the encode and the decode's syndrome pass, the same kernel over the same bytes.  achieved =
algorithmic bytes per launch (K*T source bytes per block x blocks, SURVEY.md sec. 8d: the HBM-read
roofline) / its mean launch time over both launches (as rocprofv3's per-kernel average), measured with
HIP events recorded by the launches' own dispatches on the launch stream inside the timed region; traffic = FETCH_SIZE + WRITE_SIZE of one launch from the committed rocprofv3 PMC
passes of this exact workload (profiles/rNN_traffic.json, tools/gpu_profile.sh), else null.

Multi-GPU: one process per GPU (torch.distributed); each rank owns `--blocks` independent blocks
(weak scaling, no data-path collective: blocks are independent).  The only
collectives are the timing barrier and the max-over-ranks reduction (rqshard.max_over_ranks).
"""
import argparse
import json
import re
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
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed steps for about this long before the warmup, so that the timed steps run at "
                         "the GPU's sustained clocks (profiles/r05_settle: a 20-step line right after start-up "
                         "measures the power management ramping up, 0.89-0.91 against 0.86 ms per step)")
    ap.add_argument("--blocks", type=int, default=1024, help="blocks per GPU")
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--T", type=int, default=1200)
    ap.add_argument("--N", type=int, default=1100)
    ap.add_argument("--erase", type=float, default=0.05)
    ap.add_argument("--cpu-sample", type=int, default=1024, help="blocks in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--sync-decode", action="store_true", help="time rq_decode_batch (host sync per step) "
                    "instead of rq_decode_batch_async")
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 5),
                    help="BASELINE.json config: 3 = encode+decode K=1024 (the metric, default); 2 = encode-only "
                         "1024 blocks K=256 T=1200 R=26; 5 = mixed K x T stream end to end through the host API")
    ap.add_argument("--dist-backend", default="nccl", help="process-group backend for the timing collectives "
                    "(nccl = RCCL; gloo lets several ranks share one GPU for a functional rehearsal)")
    ap.add_argument("--total-blocks", type=int, default=0,
                    help="config 3/4: shard this many blocks over the ranks (strong scaling, BASELINE config 4 = "
                         "8192); default 0 = --blocks per GPU (weak scaling)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the rank launch plan (ranks, devices, block shards) as JSON and exit; no GPU call")
    return ap.parse_args()


def rank_env(world, rank, port):
    """Environment of rank `rank` of a `world`-rank run on this node (what torch.distributed.run sets)."""
    env = dict(os.environ)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RQHIP_BENCH_SPAWNED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def launch_plan(args, world):
    """Per rank: its GPU (= local rank) and its block range (global block index of its first block, count)."""
    plan = []
    for r in range(world):
        if args.total_blocks:
            start, count = rqshard.shard(args.total_blocks, world, r)
        else:
            start, count = r * args.blocks, args.blocks
        plan.append({"rank": r, "device": r, "first_block": start, "blocks": count})
    return plan


def spawn_ranks(args):
    """`--gpus N` without a launcher: start N rank processes of this script (one per GPU, rank r on GPU r)
    before this process touches the GPU, and exit with the first non-zero rank status.  Rank 0 prints the
    JSON line.  (Under `torch.distributed.run` WORLD_SIZE is already set and no process is spawned.)
    The parent builds librqhip.so first if it is missing (rqhip.ensure_built: no GPU call), so the ranks
    never race one build or load a half-written library."""
    import socket
    import subprocess
    rqhip.ensure_built()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=rank_env(args.gpus, r, port))
             for r in range(args.gpus)]
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def erasure_pattern(K, N, n_blocks, n_erase, seed):
    rng = np.random.default_rng(seed)
    er, rep = [], []
    for _ in range(n_blocks):
        lost = set(rng.choice(N, n_erase, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rep.append([e for e in range(K, N) if e not in lost])
    return er, rep


def settle(step, ms):
    """Run `step` untimed for about `ms` of wall time before the warmup, so that the timed steps see the
    GPU's sustained clocks rather than its power management ramping up; returns the steps run."""
    import torch
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            step()
            n += 1
        torch.cuda.synchronize()
    return n


def sample_steps(steps):
    """The timed steps that carry timing events: every eighth from the second (at least two when there
    are two steps or more), so that most steps run without the events' markers (a sampled step and the
    one after it wait ~10 + ~5 us more between the decode's apply and the next encode, profiles/r05t)."""
    s = [i for i in range(steps) if i % 8 == 1]
    if len(s) < 2:
        s = [i for i in range(steps) if i % 2 == 1][:2]
    return s or [0]


def pmc_traffic(kernel, K, T, N, B):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this exact
    workload (profiles/rNN_traffic.json, written by tools/gpu_profile.sh); (None, None) if absent."""
    def tag_order(path):  # r02y < r02z < r02aa < r02af: round, then the length and letters of the tag
        m = re.match(r"r(\d+)([a-z]*)(_k\d+)?_traffic\.json$", path.name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    for path in sorted((ROOT / "profiles").glob("r*_traffic.json"), key=tag_order, reverse=True):
        t = json.loads(path.read_text())
        if t.get("kernel") == kernel and t.get("workload") == {"K": K, "T": T, "N": N, "blocks": B}:
            return t["traffic_bytes"], path.name
    return None, None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_run(K, T, N, n_erase, n_blocks, threads, seed):
    """One pass of the workload through librqcpu.so on the host: (encode s, decode s); every block is
    checked to decode back to its source."""
    import rqcpu
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (n_blocks, K * T), dtype=np.uint8)
    esis = list(range(K, N))
    er, rl = erasure_pattern(K, N, n_blocks, n_erase, seed + 1)
    rqcpu.encode(src[:1], K, T, esis)  # compile the programs outside the timed region, as on the GPU
    t0 = time.perf_counter()
    rep = rqcpu.encode(src, K, T, esis, threads)
    t_enc = time.perf_counter() - t0
    R = N - K
    rows = np.concatenate([rep[b].reshape(R, T)[[e - K for e in rl[b]]] for b in range(n_blocks)])
    data = src.copy()
    for b in range(n_blocks):
        for i in er[b]:
            data[b, i * T:(i + 1) * T] = 0xA5
    warm = data[:1].copy()
    rqcpu.decode(warm, K, T, er[:1], rl[:1], rows[:len(rl[0])])
    t0 = time.perf_counter()
    st = rqcpu.decode(data, K, T, er, rl, rows, threads)
    t_dec = time.perf_counter() - t0
    assert (st == 1).all() and np.array_equal(data, src), "CPU baseline decode mismatch"
    return t_enc, t_dec


def host_cores():
    """Threads the CPU baseline may use on this host, and where that number comes from: the smallest of
    the process's CPU affinity, its cgroup CPU quota and OMP_NUM_THREADS (the GPU box sets 16 for its
    share of a larger machine), at most 16."""
    lim = {"affinity": len(os.sched_getaffinity(0))}
    try:  # cgroup v2: "quota period" or "max period"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            lim["cgroup_quota"] = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        if os.environ.get("OMP_NUM_THREADS"):
            lim["OMP_NUM_THREADS"] = max(1, int(os.environ["OMP_NUM_THREADS"]))
    except ValueError:
        pass
    lim["cap"] = 16
    src = min(lim, key=lambda k: lim[k])
    return lim[src], "%s (%s)" % (src, ", ".join("%s %d" % kv for kv in lim.items()))


def cpu_baseline(K, T, N, n_erase, n_blocks):
    """CPU baseline on the box's host cores: librqcpu.so, the C++ port of this
    engine's algorithm (the same column program evaluated in 64-byte strips; syndrome decode with
    AVX2 split-nibble GF(256) mul-adds, the reference's asmSSSE3MulAdd technique), on a bounded
    sample of the same workload: all cores of the process's share (host_cores, one block per thread at
    a time) as the reported value, and 1 thread beside it; the oracle (the library's per-block algorithm
    restated in C, oracle/) on one block beside both, as the reference's own CPU path."""
    threads, cores_src = host_cores()
    te1, td1 = cpu_run(K, T, N, n_erase, max(8, n_blocks // 8), 1, 4242)
    nb1 = max(8, n_blocks // 8)
    teN, tdN = cpu_run(K, T, N, n_erase, n_blocks, threads, 9000)
    teO, tdO = oracle_run(K, T, N, n_erase, 4343)
    gb = lambda nb, t: round(nb * K * T / t / 1e9, 4)
    return {"value": gb(n_blocks, teN + tdN), "unit": "GB/s", "cores": threads, "cores_source": cores_src,
            "kind": "port",
            "sample": "%d blocks K=%d T=%d N=%d, %d of N erased, %d threads on '%s' (os.cpu_count %d): "
                      "librqcpu.so (C++ port of this engine's column-program encode + syndrome decode, bit-exact "
                      "to the oracle), encode %.3f s, decode %.3f s" % (n_blocks, K, T, N, n_erase, threads, cpu_model(),
                                                                       os.cpu_count() or 0, teN, tdN),
            "encode_gbs": gb(n_blocks, teN), "decode_gbs": gb(n_blocks, tdN),
            "one_thread": {"value": gb(nb1, te1 + td1), "cores": 1, "encode_gbs": gb(nb1, te1),
                           "decode_gbs": gb(nb1, td1), "sample": "%d blocks" % nb1},
            "oracle_one_thread": {"value": gb(1, teO + tdO), "cores": 1, "encode_gbs": gb(1, teO),
                                  "decode_gbs": gb(1, tdO),
                                  "sample": "1 block: oracle/rq_oracle.c, a naive dense GF(256) elimination of the "
                                            "full constraint system per block (oracle/rq_oracle.c:199; no inactivation): "
                                            "the parity checker, slower than the reference's own Solve"},
            # the reference Go path (xssnick Solve with inactivation) on one core, measured in the survey
            # container: the stated reference figure
            "reference_go_1core_gbs": 0.094}


def oracle_run(K, T, N, n_erase, seed):
    """One block through the oracle (the C restatement of the library's per-block algorithm, 1 thread):
    encode of the N - K repairs, then a decode with n_erase of the N symbols lost; seconds each."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, K * T, dtype=np.uint8)
    t0 = time.perf_counter()
    enc = O.OracleEncoder(src.tobytes(), T)
    rep = {e: enc.gen_symbol(e).tobytes() for e in range(K, N)}
    te = time.perf_counter() - t0
    lost = set(rng.choice(N, n_erase, replace=False).tolist())
    t0 = time.perf_counter()
    dec = O.OracleDecoder(K * T, T)
    for i in range(K):
        if i not in lost:
            dec.add_symbol(i, src[i * T:(i + 1) * T].tobytes())
    for e, row in rep.items():
        if e not in lost:
            dec.add_symbol(e, row)
    ok, payload = dec.decode()
    td = time.perf_counter() - t0
    assert ok and payload == src.tobytes(), "oracle baseline decode mismatch"
    return te, td


def cpu_baseline_encode(K, T, esis, n_blocks):
    """Config 2's CPU baseline: librqcpu.so encode (the same column program on host cores) of a sample of
    the same workload, 16 threads (the GPU box's CPU share) and 1 thread."""
    import rqcpu
    threads, cores_src = host_cores()
    rng = np.random.default_rng(4343)
    src = rng.integers(0, 256, (n_blocks, K * T), dtype=np.uint8)
    rqcpu.encode(src[:1], K, T, esis)  # program compile outside the timed region, as on the GPU
    t0 = time.perf_counter()
    rqcpu.encode(src, K, T, esis, threads)
    tN = time.perf_counter() - t0
    n1 = max(8, n_blocks // 8)
    t0 = time.perf_counter()
    rqcpu.encode(src[:n1], K, T, esis, 1)
    t1 = time.perf_counter() - t0
    gb = lambda nb, t: round(nb * K * T / t / 1e9, 4)
    return {"value": gb(n_blocks, tN), "unit": "GB/s", "cores": threads, "cores_source": cores_src, "kind": "port",
            "sample": "%d blocks K=%d T=%d, %d repairs, %d threads on '%s': librqcpu.so encode (the engine's column "
                      "program on host cores, bit-exact to the oracle), %.3f s" % (n_blocks, K, T, len(esis), threads,
                                                                                 cpu_model(), tN),
            "one_thread": {"value": gb(n1, t1), "cores": 1, "sample": "%d blocks" % n1}}


def cpu_baseline_mixed(shapes, frac_div):
    """Config 5's CPU baseline: librqcpu.so encode + decode of a sample of every shape of the stream (1 /
    frac_div of its blocks, at least 2), 16 threads; every decode checked against the source."""
    import rqcpu
    threads, cores_src = host_cores()
    t_all, nbytes = 0.0, 0
    for sh in shapes:
        K, T, B = sh["K"], sh["T"], max(2, sh["B"] // frac_div)
        src = sh["src"][:B].numpy()
        esis = sh["esis"]
        rqcpu.encode(src[:1], K, T, esis)
        er, rl = sh["er"][:B], sh["rl"][:B]
        t0 = time.perf_counter()
        rep = rqcpu.encode(src, K, T, esis, threads)
        R = len(esis)
        rows = np.concatenate([rep[b].reshape(R, T)[[e - K for e in rl[b]]] for b in range(B)])
        data = src.copy()
        for b in range(B):
            for i in er[b]:
                data[b, i * T:(i + 1) * T] = 0
        st = rqcpu.decode(data, K, T, er, rl, rows, threads)
        t_all += time.perf_counter() - t0
        ok = st == 1
        assert np.array_equal(data[ok], src[ok]), "CPU baseline decode mismatch"
        nbytes += B * K * T
    return {"value": round(nbytes / t_all / 1e9, 4), "unit": "GB/s", "cores": threads, "cores_source": cores_src,
            "kind": "port",
            "sample": "1/%d of every shape's blocks (>= 2), encode + decode from host memory, %d threads on '%s': "
                      "librqcpu.so (bit-exact to the oracle)" % (frac_div, threads, cpu_model())}


def pcie_copy_peak(dev, mib=256, reps=5):
    """Pinned host <-> device copy rates on this box (GB/s): the roofline of the host-memory paths."""
    n = mib << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        out[name] = n * reps / (a.elapsed_time(b) * 1e-3) / 1e9
    del h, d
    return out


_JSON_OUT = None  # the process's original stdout once the rank's fd 1 is redirected (dist_setup)


def emit(line):
    """The bench line: the ONE line rank 0 writes to the original stdout."""
    print(json.dumps(line), file=_JSON_OUT or sys.stdout, flush=True)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    # rank r pins GPU r (several gloo ranks may share one GPU in a rehearsal on a smaller box)
    gpu = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        # the communication libraries write to fd 1 (gloo's "connected to N peer ranks"): point fd 1 at
        # stderr for the rest of the rank's life and keep the original stdout for the bench line only
        global _JSON_OUT
        if _JSON_OUT is None:
            sys.stdout.flush()
            _JSON_OUT = os.fdopen(os.dup(1), "w")
            os.dup2(2, 1)
        import torch.distributed as tdist
        if args.dist_backend == "nccl":  # bind the RCCL communicator to this rank's GPU explicitly
            tdist.init_process_group(args.dist_backend, device_id=dev)
        else:
            tdist.init_process_group(args.dist_backend)
        dist = tdist
        print("bench.py: rank %d of %d on GPU %d (%s)" % (rank, world, gpu, args.dist_backend), file=sys.stderr,
              flush=True)
        # every rank owns a distinct GPU under RCCL (gloo may share one GPU in a rehearsal)
        owners = [None] * world
        tdist.all_gather_object(owners, (rank, gpu, torch.cuda.device_count()))
        if args.dist_backend == "nccl":
            gpus = [o[1] for o in owners]
            if len(set(gpus)) != world or any(o[2] < world for o in owners):
                raise SystemExit("bench.py: ranks do not own distinct GPUs: %s" % owners)
    rqhip.lib().rq_set_device(gpu)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    return world, rank, dist, dev, coll_dev


def run_config2(args):
    """BASELINE.json configs[1]: encode only, 1024 independent blocks of K=256, T=1200, 26 repairs each,
    device resident.  value = source GB/s (all ranks); the first 8 blocks are checked against the CPU
    port (librqcpu.so, itself pinned to the oracle by tests/test_cpu_baseline.py)."""
    world, rank, dist, dev, coll_dev = dist_setup(args)
    K, T, R, B = 256, 1200, 26, args.blocks
    esis = list(range(K, K + R))
    g = torch.Generator(device=dev).manual_seed(rqshard.block_seed(rank * B) + 2)
    src = torch.randint(0, 256, (B, K * T), dtype=torch.uint8, device=dev, generator=g)
    rep = torch.empty((B, R * T), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
    torch.cuda.synchronize()
    if not args.no_verify:
        import rqcpu
        ref = rqcpu.encode(src[:8].cpu().numpy(), K, T, esis)
        assert np.array_equal(rep[:8].cpu().numpy(), ref), "config 2 repairs differ from the CPU port"
    settle_steps = settle(lambda: rqhip.encode_batch(src, K, T, esis, rep, stream=stream), args.settle_ms)
    for _ in range(args.warmup):
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    sampled = sample_steps(args.steps)  # timing events on a sample (as config 3)
    ev = {s: tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for s in sampled}
    rqhip.launch_time(reset=True)
    t0 = time.perf_counter()
    for s in range(args.steps):
        samp = s in ev
        if samp:
            ev[s][0].record(stream)
            rqhip.launch_timing(True)
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        if samp:
            rqhip.launch_timing(False)
            ev[s][1].record(stream)
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = rqshard.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    rank_ms = [t / args.steps * 1e3 for t in rqshard.all_over_ranks(t_rank, dist, coll_dev)]
    if not args.no_verify:  # the timed launches' output, checked after the loop
        import rqcpu
        assert np.array_equal(rep[-8:].cpu().numpy(), rqcpu.encode(src[-8:].cpu().numpy(), K, T, esis)), \
            "config 2 repairs differ from the CPU port after the timed loop"
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b in ev.values()]))
    kern_ms, n_launch = rqhip.launch_time(reset=True)
    total = rqshard.sum_over_ranks(B, dist, coll_dev)
    if rank == 0:
        achieved = B * K * T / (kern_ms / len(ev) * 1e-3) / 1e9
        kname = "rq_colprog_K%d_n%d" % (K, R)
        traffic, traffic_src = pmc_traffic(kname, K, T, K + R, B)
        line = {
            "metric": "RaptorQ encode GB/s device-resident, 1024 blocks K=256 T=1200B R=26 (BASELINE config 2)",
            "value": round(total * K * T * args.steps / dt / 1e9, 3), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded torch.randint payload)",
            "config": {"workload": "encode-only K=%d T=%d, %d repairs per block" % (K, T, R), "blocks_per_gpu": B,
                       "verified_blocks_vs_cpu_port": 0 if args.no_verify else 16,
                       "rank_ms_per_step": {"min": round(min(rank_ms), 4), "max": round(max(rank_ms), 4)},
                       "settle": {"ms": args.settle_ms, "steps": settle_steps}},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes_per_launch": B * K * T,
                         "launch_ms": round(kern_ms / max(n_launch, 1), 4), "step_event_ms": round(enc_ms, 4),
                         "launch_timing": "HIP events recorded by the launches' own dispatches "
                                          "(hipExtModuleLaunchKernel, rq_launch_timing) on timed steps %s" % sorted(ev),
                         "achieved_read_write": round(B * (K + R) * T / (kern_ms / len(ev) * 1e-3) / 1e9, 2)}}
        if args.cpu_sample > 0 and world == 1:
            line["cpu_baseline"] = cpu_baseline_encode(K, T, esis, args.cpu_sample)
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


def run_config5(args):
    """BASELINE.json configs[4]: a round-robin stream of K in {128, 512, 2048} x T in {256, 1200}
    (N = K + K/10 + 8, 5 % of N erased: the fecquic loopback shape), end to end through the library's
    host-memory batch API (rq_encode_batch_host / rq_decode_batch_host) on pinned buffers: source
    H2D, encode, repairs D2H, then data + received repairs H2D, decode, recovered rows D2H.  value =
    source GB/s of encode + decode over the whole stream (all ranks: each rank runs its own stream on
    its GPU).  Every decoded payload is checked bit-exactly."""
    world, rank, dist, dev, coll_dev = dist_setup(args)
    rng = np.random.default_rng(5 + rank)
    mb = 128  # source MiB per shape per step
    shapes = []
    for K in (128, 512, 2048):
        for T in (256, 1200):
            N = K + K // 10 + 8
            R, n_erase = N - K, round(0.05 * N)
            B = max(8, int(mb * 2 ** 20 // (K * T)))
            esis = list(range(K, N))
            src = torch.from_numpy(rng.integers(0, 256, (B, K * T), dtype=np.uint8)).pin_memory()
            rep = torch.empty((B, R * T), dtype=torch.uint8).pin_memory()
            er, rl = erasure_pattern(K, N, B, n_erase, 11 + K + T + rank)
            rqhip.encode_batch_host(src, K, T, esis, rep)
            rv = rep.view(B, R, T)
            repair = torch.cat([rv[b, [e - K for e in rl[b]]] for b in range(B)]).pin_memory()
            data = src.clone().pin_memory()
            db = rqhip.DecodeBatch(K, T, er, rl)
            st = rqhip.decode_batch_host(db, data, repair)
            ok = torch.from_numpy(st == 1)
            assert torch.equal(data[ok], src[ok]), (K, T)
            shapes.append(dict(K=K, T=T, N=N, B=B, esis=esis, src=src, rep=rep, repair=repair, data=data, db=db, er=er, rl=rl,
                               ok=float(ok.float().mean()), t_enc=0.0, t_dec=0.0))

    def step():
        for sh in shapes:
            t0 = time.perf_counter()
            rqhip.encode_batch_host(sh["src"], sh["K"], sh["T"], sh["esis"], sh["rep"])
            t1 = time.perf_counter()
            rqhip.decode_batch_host(sh["db"], sh["data"], sh["repair"])
            t2 = time.perf_counter()
            sh["t_enc"] += t1 - t0
            sh["t_dec"] += t2 - t1
    settle_steps = settle(step, args.settle_ms)
    for _ in range(args.warmup):
        step()
    for sh in shapes:
        sh["t_enc"] = sh["t_dec"] = 0.0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = rqshard.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    for sh in shapes:  # the stream's last decode left every payload intact
        ok = torch.from_numpy(sh["db"].status == 1)
        assert torch.equal(sh["data"][ok], sh["src"][ok]), (sh["K"], sh["T"])
    src_bytes = sum(sh["B"] * sh["K"] * sh["T"] for sh in shapes)
    total = rqshard.sum_over_ranks(src_bytes, dist, coll_dev)
    # PCIe bytes of one step (host-memory batch API): encode H2D source, D2H repairs; decode H2D data
    # blocks + received repair rows, D2H the recovered rows of the blocks that decoded
    h2d = sum(sh["B"] * sh["K"] * sh["T"] * 2 + sh["repair"].numel() for sh in shapes)
    d2h = sum(sh["rep"].numel() + sum(len(x) for x in sh["er"]) * sh["T"] for sh in shapes)
    link = pcie_copy_peak(dev) if rank == 0 else None
    if rank == 0:
        per = [{"K": sh["K"], "T": sh["T"], "N": sh["N"], "blocks": sh["B"], "ok_fraction": sh["ok"],
                "encode_GBps": round(sh["B"] * sh["K"] * sh["T"] * args.steps / sh["t_enc"] / 1e9, 2),
                "decode_GBps": round(sh["B"] * sh["K"] * sh["T"] * args.steps / sh["t_dec"] / 1e9, 2)} for sh in shapes]
        line = {
            "metric": "RaptorQ encode+decode GB/s end to end incl. pinned H2D/D2H, mixed K{128,512,2048} x "
                      "T{256,1200} stream at 5% loss (BASELINE config 5)",
            "value": round(total * args.steps / dt / 1e9, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded numpy payload, seeded exact-count erasures), pinned host buffers",
            "config": {"workload": "mixed stream, %d MiB of source per shape per step, host-memory batch API" % mb,
                       "settle": {"ms": args.settle_ms, "steps": settle_steps},
                       "shapes": per},
            # the path is bound by the PCIe link (pinned copies measured on this box), not HBM: achieved =
            # H2D bytes per second of the whole stream (the busier direction) against the box's pinned
            # H2D copy rate; D2H beside it
            "roofline": {"bound": "pcie", "achieved": round(h2d * args.steps / dt / 1e9, 2),
                         "peak": round(link["h2d"], 2), "unit": "GB/s",
                         "frac": round(h2d * args.steps / dt / 1e9 / link["h2d"], 4), "traffic": h2d + d2h,
                         "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
                         "d2h_achieved": round(d2h * args.steps / dt / 1e9, 2), "d2h_peak": round(link["d2h"], 2),
                         "peak_source": "torch pinned copy_ of 256 MiB, 5 reps, this box"}}
        if args.cpu_sample > 0 and world == 1:
            line["cpu_baseline"] = cpu_baseline_mixed(shapes, max(1, args.cpu_sample // 128))
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.plan_only:
        # a rehearsal of the launch without any GPU call: the parent builds the library if it is missing,
        # then (no launcher) starts the N ranks, each of which only checks that the library is there
        if os.environ.get("RQHIP_BENCH_SPAWNED") == "1":
            built = rqhip.ensure_built()
            print("bench.py --plan-only: rank %s sees %s (built here: %s)" % (os.environ.get("RANK"), rqhip.LIB_PATH, built),
                  file=sys.stderr, flush=True)
            return 0
        world = args.gpus
        launcher = "spawn" if "WORLD_SIZE" not in os.environ else "external"
        built = rqhip.ensure_built()
        rc = spawn_ranks(args) if launcher == "spawn" and world > 1 else 0
        print(json.dumps({"world": world, "launcher": launcher, "scaling": "strong" if args.total_blocks else "weak",
                          "ranks": launch_plan(args, world), "library": str(rqhip.LIB_PATH), "built_by_parent": built,
                          "ranks_rc": rc}))
        return rc
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    if args.config == 2:
        return run_config2(args)
    if args.config == 5:
        return run_config5(args)
    world, rank, dist, dev, coll_dev = dist_setup(args)
    K, T, N = args.K, args.T, args.N
    first, B = launch_plan(args, world)[rank]["first_block"], launch_plan(args, world)[rank]["blocks"]
    R = N - K
    n_erase = int(round(args.erase * N))
    esis = list(range(K, N))
    g = torch.Generator(device=dev).manual_seed(rqshard.block_seed(first))
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
    def one_step():
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        (db.run if args.sync_decode else db.run_async)(data, recv, stream=stream)
    settle_steps = settle(one_step, args.settle_ms)
    for _ in range(args.warmup):
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        (db.run if args.sync_decode else db.run_async)(data, recv, stream=stream)
    torch.cuda.synchronize()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # Timing events on every eighth timed step (from the second): the stream markers and the
    # dispatch-recorded events of rq_launch_timing add ~1 % each to a step they bracket
    # (profiles/r03_dense/r03tb, r03f), so the other steps run as a caller would run them.
    sampled = sample_steps(args.steps)
    ev = {s: tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for s in sampled}
    rqhip.launch_time(reset=True)
    t0 = time.perf_counter()
    for s in range(args.steps):
        samp = s in ev
        if samp:
            ev[s][0].record(stream)
            # the column program's launches (the encode's and the decode's syndrome pass) record their
            # own kernel start / stop (rq_launch_timing)
            rqhip.launch_timing(True)
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        if samp:
            ev[s][1].record(stream)
        st_async = (db.run if args.sync_decode else db.run_async)(data, recv, stream=stream)
        if samp:
            rqhip.launch_timing(False)
            ev[s][2].record(stream)
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0  # this rank's own time, before the closing barrier
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = rqshard.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    rank_ms = [t / args.steps * 1e3 for t in rqshard.all_over_ranks(t_rank, dist, coll_dev)]
    if not args.no_verify:
        assert np.array_equal(st_async, st), "async decode statuses differ"
        # the timed decodes ran on rows already recovered (zero syndromes; the work is data-independent):
        # poison the erased rows again and decode once more, checking bytes as well as statuses
        rqhip.encode_batch(src, K, T, esis, rep, stream=stream)
        data.view(B, K, T)[eb, ei] = 0x5A
        st_post = db.run(data, recv, stream=stream)
        torch.cuda.synchronize()
        assert np.array_equal(st_post, st), "post-timing decode statuses differ"
        good = torch.tensor(st_post == 1, device=dev)
        assert torch.equal(data[good], src[good]), "post-timing decode bytes differ"
    enc_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1, _ in ev.values()]))
    dec_ms = float(np.mean([e1.elapsed_time(e2) for _, e1, e2 in ev.values()]))
    kern_ms, n_launch = rqhip.launch_time(reset=True)
    # the column program's time per pass over the B blocks, the mean of the sampled steps' encode and
    # syndrome passes (one launch each, unless a 4 GiB buffer span splits one)
    col_kernel_ms = kern_ms / (2 * len(ev))
    total_blocks = rqshard.sum_over_ranks(B, dist, coll_dev)
    value = total_blocks * K * T * args.steps / dt / 1e9
    if rank == 0:
        kname = "rq_colprog_K%d_n%d" % (K, R)
        achieved = B * K * T / (col_kernel_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(kname, K, T, N, B)
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong" if args.total_blocks else "weak", "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded torch.randint payload per rank, seeded exact-count 5% erasures)",
            "config": {"workload": "encode+decode K=%d T=%d N=%d, erase %d of %d symbols per block" % (K, T, N, n_erase, N),
                       "blocks_per_gpu": B, "total_blocks": total_blocks, "bytes_per_gpu": B * K * T,
                       "parallelism": "block-sharded x%d" % world,
                       "decode_ok_fraction": ok_frac, "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                       "rank_ms_per_step": {"min": round(min(rank_ms), 4), "max": round(max(rank_ms), 4),
                                            "per_rank": [round(x, 4) for x in rank_ms]},
                       "post_timing_check": "skipped" if args.no_verify else "bytes+statuses",
                       "settle": {"ms": args.settle_ms, "steps": settle_steps}},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "algorithmic_bytes_per_launch": B * K * T,
                         "launch_ms": round(kern_ms / max(n_launch, 1), 4), "launches_per_step": n_launch // len(ev),
                         "launch_timing": "HIP events recorded by the column program's own dispatches "
                                          "(hipExtModuleLaunchKernel, rq_launch_timing) on the bench stream: "
                                          "the encode and the decode's syndrome launch of timed steps %s" % sorted(ev),
                         # total read + write rate of the launch, (K + R) * T per block
                         "achieved_read_write": round(B * (K + R) * T / (col_kernel_ms * 1e-3) / 1e9, 2)},
        }
        if args.cpu_sample > 0 and world == 1:
            line["cpu_baseline"] = cpu_baseline(K, T, N, n_erase, args.cpu_sample)
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
