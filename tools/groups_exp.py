"""Experiment: split the per-GPU batch into G independent handles (own HIP streams) and step them
round-robin, so kernels of different groups can overlap on the GPU. Prints it/s per G."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
abi = pkg.abi
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
steps, warm = 10, 2
for G in [int(g) for g in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "4"])]:
    hs = []
    for g in range(G):
        prob, opts = pkg.Problems.config_quadrotor(B=B // G, offset=g * (B // G))
        s = pkg.AbstractSolverFor(prob, opts)
        hs.append(s)
    for s in hs:
        s.handle.solve_init(abi.MODE_AL)
        s.handle.solve_step(warm)
    for s in hs:
        s.handle.synchronize()
    t0s = [s.handle.total_steps() for s in hs]
    t = time.perf_counter()
    for _ in range(steps):
        for s in hs:
            s.handle.solve_step(1)
    for s in hs:
        s.handle.synchronize()
    dt = time.perf_counter() - t
    done = sum(s.handle.total_steps() - t0 for s, t0 in zip(hs, t0s))
    print(f"G={G} B={B} it/s={done / dt:.0f} ms/step={1e3 * dt / steps:.3f}", flush=True)
    del hs
