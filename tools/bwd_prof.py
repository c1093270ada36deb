"""Backward-kernel section breakdown (GPU box). Build the timed variant first:
    tools/ab_build.sh prof -DTOG_BWD_PROF
    TOG_LIBRARY=build_ab/prof/libtog.so python tools/bwd_prof.py [steps]
Runs the bench workload (config 3) for a few AL-iLQR steps and prints each knot-loop section's share
of the summed shader-clock cycles (tog_bwd_team.hpp BPROF markers)."""
import ctypes
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import __graft_entry__  # noqa: E402

NAMES = ["terminal knot", "expansion record loads", "S [A B], Q.ux", "QR Q.uu", "QR Q.xx",
         "regularise + cond", "gains solve", "K/d store, s, tmp1", "chol_minus", "S-update operands",
         "QR S-update", "epilogue", "-", "-", "-", "-", "-", "[A B] loads",
         "-", "-"]
pkg = __graft_entry__.load_package()
abi = pkg.abi
lib = abi.load_library()
read = lib.tog_bwd_prof_read
read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
prob, opts = pkg.Problems.config_quadrotor(B=B)
s = pkg.AbstractSolverFor(prob, opts)
s.handle.solve_init(abi.MODE_AL)
s.handle.solve_step(1)
s.handle.synchronize()
buf = (ctypes.c_ulonglong * 32)()
read(buf)
s.handle.solve_step(steps)
s.handle.synchronize()
assert read(buf) in (20, 32)
tot = sum(buf)
waves = (B + 3) // 4
print(f"B={B} steps={steps}: cycles per wave-knot = {tot / (waves * steps * (prob.N - 1)):.0f}")
for nm, v in zip(NAMES, buf):
    print(f"{nm:40s} {100.0 * v / tot:6.2f}%  {v / 1e9:10.3f} Gcyc  {v / (waves * steps * (prob.N - 1)):9.0f} cyc/wave-knot")
