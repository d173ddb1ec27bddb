"""Per-stream device state of the batched device-resident calls: a caller that uses a fresh stream per
window (a fecquic-style pipeline; go/fecquic/rxbuf.go:336-377 runs repeated worker decodes) must not
grow device memory without bound (rq_engine.cpp DevCtx::MAX_WS = 8 caller-stream workspaces, LRU), the
results must not depend on the stream, rq_stream_release frees a stream's workspace, and rq_shutdown
releases everything and the next call starts afresh."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K, T, N, NB = 256, 1200, 282, 64


def _case(gpu, rq, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    src = torch.randint(0, 256, (NB, K * T), dtype=torch.uint8, device=gpu, generator=g)
    rng = np.random.default_rng(seed)
    er, rl = [], []
    for _ in range(NB):
        lost = set(rng.choice(N, 14, replace=False).tolist())
        er.append(sorted(i for i in lost if i < K))
        rl.append([e for e in range(K, N) if e not in lost])
    return src, er, rl


def _round(gpu, rq, src, er, rl, stream):
    esis = list(range(K, N))
    rep = torch.empty((NB, (N - K) * T), dtype=torch.uint8, device=gpu)
    with torch.cuda.stream(stream):
        rq.encode_batch(src, K, T, esis, rep, stream=stream)
        rv = rep.view(NB, N - K, T)
        recv = torch.cat([rv[b, [e - K for e in rl[b]]] for b in range(NB)])
        data = src.clone()
        for b in range(NB):
            for i in er[b]:
                data[b, i * T:(i + 1) * T] = 0x33
        st = rq.DecodeBatch(K, T, er, rl).run(data, recv, stream=stream)
    stream.synchronize()
    return rep.cpu(), data.cpu(), st


def _used():  # device memory in use, torch's per-stream allocator caches emptied first
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info()
    return total - free


def test_64_streams_bounded_and_identical(gpu, rq):
    src, er, rl = _case(gpu, rq, 17)
    ref_rep, ref_data, ref_st = _round(gpu, rq, src, er, rl, torch.cuda.Stream())
    assert (ref_st == 1).all() and torch.equal(ref_data, src.cpu())
    streams = [torch.cuda.Stream() for _ in range(64)]
    used = []
    for i, s in enumerate(streams):
        rep, data, st = _round(gpu, rq, src, er, rl, s)
        assert torch.equal(rep, ref_rep) and torch.equal(data, ref_data) and np.array_equal(st, ref_st), i
        used.append(_used())
    # one workspace here is ~10 MB (64 blocks K=256); at most 8 caller streams keep one, so from the 9th
    # stream on device memory stays flat: the stated bound is 64 MiB of growth over streams 16..64
    # (allocator noise), against ~55 x 10 MB = 550 MB without the bound
    grow = max(used[15:]) - used[15]
    assert grow < 64 << 20, (grow, used[::8])


def test_stream_release_and_shutdown(gpu, rq):
    src, er, rl = _case(gpu, rq, 23)
    s = torch.cuda.Stream()
    ref_rep, ref_data, _ = _round(gpu, rq, src, er, rl, s)
    before = _used()
    assert rq.lib().rq_stream_release(ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    assert _used() <= before
    assert rq.lib().rq_shutdown() == 0  # every device resource released ...
    rep, data, st = _round(gpu, rq, src, er, rl, torch.cuda.Stream())  # ... and re-created on demand
    assert torch.equal(rep, ref_rep) and torch.equal(data, ref_data) and (st == 1).all()


def test_device_resident_symbol_size_limit(gpu, rq):
    """Device-resident batches take T a multiple of 4 and at least 8 (documented in rqhip.h); T=4 is
    refused with RQ_ERR_BAD_ARG instead of failing inside the launch, and the host-memory batch (which
    pads rows) still encodes T=4 blocks."""
    Ks = 16
    src = torch.randint(0, 256, (2, Ks * 4), dtype=torch.uint8, device=gpu)
    out = torch.empty((2, 4 * 4), dtype=torch.uint8, device=gpu)
    with pytest.raises(rq.RaptorQError) as e:
        rq.encode_batch(src, Ks, 4, list(range(Ks, Ks + 4)), out)
    assert e.value.code == rq.RQ_ERR_BAD_ARG
    hsrc = src.cpu().pin_memory()
    hout = torch.empty((2, 16), dtype=torch.uint8).pin_memory()
    rq.encode_batch_host(hsrc, Ks, 4, list(range(Ks, Ks + 4)), hout)
    o8 = torch.empty((2, 4 * 8), dtype=torch.uint8, device=gpu)
    s8 = torch.zeros((2, Ks * 8), dtype=torch.uint8, device=gpu)
    s8.view(2, Ks, 8)[:, :, :4] = src.view(2, Ks, 4)
    rq.encode_batch(s8, Ks, 8, list(range(Ks, Ks + 4)), o8)  # the same bytes, padded to T=8 by hand
    assert torch.equal(hout, o8.view(2, 4, 8)[:, :, :4].reshape(2, 16).cpu())


def test_launch_timing(gpu, rq):
    """rq_launch_timing / rq_launch_time (bench.py's roofline): only launches issued while timing is on
    are counted, their dispatch-recorded kernel time fits inside the stream events around them, and the
    timed launches compute the same bytes as untimed ones."""
    src, _, _ = _case(gpu, rq, 29)
    esis = list(range(K, N))
    ref = torch.empty((NB, (N - K) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, ref)
    rep = torch.empty_like(ref)
    rq.launch_time(reset=True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    rq.launch_timing(True)
    for _ in range(3):
        rq.encode_batch(src, K, T, esis, rep)
    rq.launch_timing(False)
    b.record()
    rq.encode_batch(src, K, T, esis, rep)  # not timed
    torch.cuda.synchronize()
    ms, n = rq.launch_time(reset=True)
    assert n == 3 and 0 < ms <= a.elapsed_time(b) * 1.01, (ms, n, a.elapsed_time(b))
    assert torch.equal(rep, ref)
    assert rq.launch_time(reset=True) == (0.0, 0)


def test_shutdown_with_concurrent_caller(gpu, rq):
    """rq_shutdown while another thread is inside library calls: each call holds its context (a
    shared_ptr, rq_engine.cpp CtxRef), so the context is destroyed only when the last call using it
    returns, and calls after the shutdown build a fresh one.  Every encode still returns the reference
    bytes; nothing faults."""
    import threading
    src, _, _ = _case(gpu, rq, 31)
    esis = list(range(K, N))
    ref = torch.empty((NB, (N - K) * T), dtype=torch.uint8, device=gpu)
    rq.encode_batch(src, K, T, esis, ref)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    outs = [torch.empty_like(ref) for _ in range(24)]
    errors = []

    def worker():
        try:
            for o in outs:
                rq.encode_batch(src, K, T, esis, o, stream=s)
                s.synchronize()
        except Exception as ex:  # noqa: BLE001 -- reported by the main thread
            errors.append(repr(ex))

    th = threading.Thread(target=worker)
    th.start()
    import time
    for _ in range(3):
        time.sleep(0.05)
        assert rq.lib().rq_shutdown() == 0
    th.join(timeout=120)
    assert not th.is_alive() and not errors, errors
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert torch.equal(o, ref), i
