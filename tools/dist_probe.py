"""Probe: per-step cost of the multi-rank bench path (stats exchange over RCCL) at world size 1.
Run on the GPU box: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=... python tools/dist_probe.py"""
import ctypes, os, sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import torch.distributed as dist
import __graft_entry__ as g

pkg = g.load_package()
abi = pkg.abi
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
stream = torch.cuda.current_stream().cuda_stream
print("torch current stream handle", stream, flush=True)
prob, opts = pkg.Problems.config_quadrotor(B=8192)
mode = os.environ.get("PROBE_STREAM", "torch")
solver = pkg.AbstractSolverFor(prob, opts, stream=stream if mode == "torch" else None)
h = solver.handle
stats_t = torch.zeros(3, dtype=torch.float64, device="cuda:0")
gathered = torch.zeros(3, dtype=torch.float64, device="cuda:0")
h.solve_init(abi.MODE_AL)
h.solve_step(2)
h.synchronize()


def run(label, stats, gather, steps=5):
    torch.cuda.synchronize(); h.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        h.solve_step(1)
        if stats:
            abi.check(h.lib, h.lib.tog_batch_stats_device(h.h, ctypes.c_void_p(stats_t.data_ptr())))
        if gather:
            pkg.distributed.reduce_stats(stats_t, gathered, dist)
    h.synchronize(); torch.cuda.synchronize()
    print(f"{label:28s} {1e3 * (time.perf_counter() - t) / steps:8.3f} ms/step", flush=True)


run("plain", False, False)
run("stats kernel", True, False)
run("all_gather", False, True)
run("stats + all_gather", True, True)
run("plain again", False, False)
h.profile(True)
run("plain, profiling", False, False)
run("stats+gather, profiling", True, True)
dist.destroy_process_group()
