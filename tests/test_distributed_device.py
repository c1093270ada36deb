"""The multi-rank path on the device.

* World 1 over RCCL (``nccl``) on a dedicated stream: ``tog_batch_stats_device`` writes
  [n_active, Σ J, max c_max] into a torch tensor and ``distributed.reduce_stats`` all-gathers it,
  stream-ordered — exactly bench.py's per-step exchange. The reduced values must equal the host-side
  ``tog_batch_stats`` and the step counts must equal a run without the collective.
* World 2 over gloo with a device handle per rank (both ranks on GPU 0: the pool's boxes have one
  GPU): each rank solves its contiguous shard on the device and the gathered statistics equal a
  single-process device solve of the whole batch.

Every rank runs in its own spawned process; at most 2 processes use the GPU at once.
"""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_world1(port, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    import ctypes

    import torch
    import torch.distributed as dist

    import __graft_entry__

    tog = __graft_entry__.load_package()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ts = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(ts)
    prob, opts = tog.Problems.config_quadrotor(B=256)
    solver = tog.AbstractSolverFor(prob, opts, device=0, stream=ts.cuda_stream)
    h = solver.handle
    stats = torch.zeros(3, dtype=torch.float64, device="cuda:0")
    gathered = torch.zeros(3, dtype=torch.float64, device="cuda:0")
    h.solve_init(tog.abi.MODE_AL)
    out = []
    for _ in range(6):
        h.solve_step(1)
        tog.abi.check(h.lib, h.lib.tog_batch_stats_device(h.h, ctypes.c_void_p(stats.data_ptr())))
        red = tog.distributed.reduce_stats(stats, gathered, dist)  # RCCL, stream-ordered
        red_host = red.cpu().numpy().copy()  # waits on the stream
        out.append((red_host.tolist(), h.batch_stats().tolist()))
    steps = h.total_steps()
    # the same steps without the collective, on the handle's own stream (with the same host stats
    # readbacks: the line-search round schedule follows the last n_active read on the host)
    s2 = tog.AbstractSolverFor(prob, opts, device=0)
    s2.handle.solve_init(tog.abi.MODE_AL)
    for _ in range(6):
        s2.handle.solve_step(1)
        s2.handle.batch_stats()
    q.put((out, steps, s2.handle.total_steps(), s2.handle.batch_stats().tolist()))
    dist.destroy_process_group()


def test_rccl_world1_stream_ordered_stats(tog):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_rccl_world1, args=(_free_port(), q))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0
    out, steps, steps2, final2 = q.get()
    for red, host in out:
        assert red == host  # gathered == tog_batch_stats, no host sync in between
    assert steps == steps2 and out[-1][1] == final2


def _device_shard_stats(tog, offset, count):
    prob, opts = tog.Problems.config_quadrotor(B=count, offset=offset)
    solver = tog.AbstractSolverFor(prob, opts, device=0)
    h = solver.handle
    h.solve(tog.abi.MODE_AL)
    return h.batch_stats().tolist(), h.total_steps()


def _gloo_device_worker(rank, world, port, total, q):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    import __graft_entry__

    tog = __graft_entry__.load_package()
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    off, cnt = tog.distributed.shard(total, rank, world)
    st, steps = _device_shard_stats(tog, off, cnt)
    st[0] = float(st[0])
    stats = torch.tensor(st, dtype=torch.float64)
    gathered = torch.zeros(3 * world, dtype=torch.float64)
    red = tog.distributed.reduce_stats(stats, gathered, dist)
    rate, steps_all, _ = tog.distributed.job_rate(float(steps), 1.0 + rank, dist)
    if rank == 0:
        q.put((red.tolist(), steps_all))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_device_shards_match_single_process(tog):
    import torch.multiprocessing as mp

    total, world = 64, 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_device_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    red, steps_all = q.get()
    want, steps = _device_shard_stats(tog, 0, total)
    assert red[0] == want[0] == 0.0  # every trajectory finished
    assert red[1] == pytest.approx(want[1], rel=1e-12)  # Σ J: per-shard partial sums, reassociated
    assert red[2] == want[2]
    assert steps_all == steps
