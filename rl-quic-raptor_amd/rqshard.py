"""Block sharding across ranks (one process per GPU) and the timing reduction of bench.py.

Source blocks are independent (go/fecquic/transfer.go:166-268 splits an object into
K*T blocks and encodes each on its own), so ranks partition the block index space with no data-path
collective.  The only collectives are the timing barrier and the max-over-ranks reduction.
"""


def shard(n_total, world, rank):
    """Contiguous block range [start, start+count) of `rank`; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def block_seed(global_block):
    """Payload seed of a block: splitmix-style 1337 + global index (BASELINE.md synthetic inputs)."""
    return 1337 + global_block


def max_over_ranks(x, dist=None, device=None):
    """Max of a float over all ranks (the bench's wall time); identity without a process group."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, dist=None, device=None):
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(x)
    import torch
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def all_over_ranks(x, dist=None, device=None):
    """Every rank's value of a float, in rank order (per-rank timings in the bench line)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [float(x)]
    import torch
    out = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(dist.get_world_size())]
    dist.all_gather(out, torch.tensor([float(x)], dtype=torch.float64, device=device))
    return [float(t.item()) for t in out]
