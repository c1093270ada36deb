"""Batch sharding across GPUs.

Trajectories are independent, so a batch of B trajectories is split into contiguous slices, one
per rank (one process per GPU, ``torch.distributed`` with RCCL). The solve itself needs no
communication; the only collective is the batch-statistics exchange used for batch-level stopping
and reporting: [n_active, Σ cost, max c_max] per shard, gathered in one call (≤ 24 B per rank) and
reduced locally (sum, sum, max). The same code runs on gloo for the CPU tests.
"""
from __future__ import annotations


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """(offset, count) of this rank's contiguous slice; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def reduce_stats(stats, gathered, dist, group=None):
    """All-gather the per-shard [n_active, Σ cost, max c_max] (a 3-element float64 tensor) into
    ``gathered`` (3*world) and return the batch-wide (n_active, Σ cost, max c_max) as a tensor,
    without a host synchronisation (stream-ordered on RCCL)."""
    dist.all_gather_into_tensor(gathered, stats, group=group)
    g = gathered.view(-1, 3)
    out = g.sum(dim=0)
    out[2] = g[:, 2].max()
    return out


def job_rate(steps_local: float, elapsed_local: float, dist, device=None):
    """Whole-job throughput for weak scaling: Σ trajectory-steps over ranks ÷ max wall time."""
    import torch

    t = torch.tensor([float(steps_local), float(elapsed_local)], dtype=torch.float64, device=device)
    s = t[0:1].clone()
    e = t[1:2].clone()
    dist.all_reduce(s)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(s.item()) / float(e.item()), float(s.item()), float(e.item())
