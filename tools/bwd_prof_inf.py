"""k_backward section breakdown for the infeasible maze (GPU box). Build first (here):
    python tools/prof_inf_build.py
then on the box:
    TOG_LIBRARY=ab_var/prof_inf/libtog.so python tools/bwd_prof_inf.py [steps] [B]
Sections (BPROF ids in the patched k_backward): 0 the knot's [A|B], x, u loads; 1 the cost + AL expansion;
2 Q.x/Q.u and the [A B]'S products; 3 regularisation, isposdef test and LU; 4 the gains solve; 5 K/d store,
S update and ΔV (charged to the next knot's start); 6 the epilogue."""
import ctypes
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import __graft_entry__  # noqa: E402

NAMES = ["[A|B], x, u loads", "expansion (cost + AL rows)", "Q.x/Q.u, [A B]'S products", "Quu_reg, isposdef, LU",
         "gains solve", "K/d store, S update, dV", "epilogue"]
pkg = __graft_entry__.load_package()
abi = pkg.abi
lib = abi.load_library()
read = lib.tog_bwd_prof_read
read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
prob, opts = pkg.Problems.config_quadrotor_maze_infeasible(B=B)
s = pkg.AbstractSolverFor(prob, opts.opts_al)
h = s.handle
h.slack_controls()  # infeasible.jl:63-80, as bench.py
h.solve_init(abi.MODE_AL)
h.solve_step(1)
h.synchronize()
buf = (ctypes.c_ulonglong * 32)()
read(buf)
h.solve_step(steps)
h.synchronize()
assert read(buf) == 32
tot = sum(buf[:7])
knots = B * steps * (prob.N - 1)
print(f"B={B} steps={steps}: cycles per wave-knot = {tot / knots:.0f} (shader clock, summed over lane 0 of each wave)")
for nm, v in zip(NAMES, buf[:7]):
    print(f"{nm:34s} {100.0 * v / max(tot, 1):6.2f}%  {v / knots:9.0f} cyc/wave-knot")
