"""Multi-rank path on CPU: world_size 2 over gloo (127.0.0.1). Each rank takes its contiguous
shard of a config-3 batch, solves it (with the CPU oracle standing in for the per-GPU handle —
test infrastructure only), exchanges the batch statistics with the same collective bench.py uses,
and the reduced totals must equal a single-process solve of the whole batch."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_shard_partition(tog):
    for total in (1, 7, 8192, 65536):
        for world in (1, 2, 3, 8):
            parts = [tog.distributed.shard(total, r, world) for r in range(world)]
            assert parts[0][0] == 0
            assert sum(c for _, c in parts) == total
            for (o1, c1), (o2, _) in zip(parts, parts[1:]):
                assert o1 + c1 == o2
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    with pytest.raises(ValueError):
        tog.distributed.shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_stats(tog, oracle, offset, count):
    prob, opts = tog.Problems.config_quadrotor(B=count, offset=offset)
    n_active, cost, cmax = 0.0, 0.0, 0.0
    for b in range(count):
        s = oracle.OracleSolver(prob, opts, b)
        s.solve()
        st = s.get("stats")
        n_active += 1.0 if not (int(st[tog.abi.STAT_FLAGS]) & tog.abi.TRAJ_AL_CONVERGED) else 0.0
        cost += st[tog.abi.STAT_J]
        cmax = max(cmax, st[tog.abi.STAT_C_MAX])
    return [n_active, cost, cmax]


def _worker(rank, world, port, total, q):
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import __graft_entry__

    tog = __graft_entry__.load_package()
    oracle = __graft_entry__.load_oracle()
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    off, cnt = tog.distributed.shard(total, rank, world)
    stats = torch.tensor(_shard_stats(tog, oracle, off, cnt), dtype=torch.float64)
    gathered = torch.zeros(3 * world, dtype=torch.float64)
    red = tog.distributed.reduce_stats(stats, gathered, dist)
    rate, steps, elapsed = tog.distributed.job_rate(10.0 * (rank + 1), 1.0 + rank, dist)
    if rank == 0:
        q.put((red.tolist(), rate, steps, elapsed))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_stats_match_single_process(tog, oracle):
    import torch.multiprocessing as mp

    total, world = 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    red, rate, steps, elapsed = q.get()
    want = _shard_stats(tog, oracle, 0, total)
    assert red[0] == want[0]
    assert red[1] == pytest.approx(want[1], rel=1e-12)
    assert red[2] == want[2]
    assert steps == 30.0 and elapsed == 2.0 and rate == 15.0
