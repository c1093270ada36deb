"""Section breakdown of the two-wave tail backward kernel (k_bwd_duo, tog_bwd_duo.hpp DPROF markers).
Build the timed variant first:
    tools/ab_quad.sh prof -DTOG_BWD_PROF
    TOG_LIBRARY=ab_libs/prof/libtog.so python tools/duo_prof.py [steps] [trio|duo]
Runs config 3 at B=1 (the convergence-tail configuration) for a few AL-iLQR steps and prints each wave's
sections in shader-clock cycles (s_memtime) per knot."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import __graft_entry__  # noqa: E402

KIND = sys.argv[2] if len(sys.argv) > 2 else "quad"
if KIND == "quad":  # tog_bwd_quad.hpp's DPROF ids
    NAMES = {0: "A: knot start", 1: "A: QR [Q.xx; S A] (rows released)", 2: "A: wait K, tmp1",
             3: "A: top operands Q.xx + tmp1 K", 4: "A: wait B2b", 5: "A: bottom operands + QR S-update",
             25: "A: wait B3",
             6: "B: loads, QR [Q.uu; S B], Q.x/Q.u", 7: "B: regularise + cond", 8: "B: wait Q.ux",
             9: "B: gains, K/d, s, dV", 10: "B: wait B2b", 11: "B: S A, S B rows (with waits)", 12: "B: wait B3",
             13: "C: Q.ux", 14: "C: tmp1 rows (with waits)", 15: "C: wait B2b", 16: "C: wait B3",
             17: "D: wait Q.uu", 18: "D: chol_minus rows (with waits)", 19: "D: chol_minus tail",
             26: "D: wait B2b", 27: "D: wait B3"}
    WAVES = {"A": [0, 1, 2, 3, 4, 5, 25], "B": [6, 7, 8, 9, 10, 11, 12], "C": [13, 14, 15, 16],
             "D": [17, 18, 19, 26, 27]}
elif KIND == "trio":  # tog_bwd_trio.hpp's DPROF ids
    NAMES = {0: "A: knot start", 2: "A: QR [Q.xx; S A] (rows released)", 6: "A: wait B2b",
             7: "A: S-update operands", 8: "A: QR S-update (rows released)", 9: "A: wait B3",
             13: "B: loads, QR [Q.uu; S B], Q.x/Q.u", 15: "B: regularise + cond", 14: "B: wait Q.ux",
             16: "B: gains, K/d, s, dV", 17: "B: wait B2b", 11: "B: S A, S B rows (with waits)",
             18: "B: wait B3",
             1: "C: Q.ux", 3: "C: wait Q.uu", 4: "C: tmp1 + chol_minus rows (with waits)",
             5: "C: chol_minus tail", 12: "C: wait B2b", 19: "C: wait B3"}
    WAVES = {"A": [0, 2, 6, 7, 8, 9], "B": [13, 15, 14, 16, 17, 11, 18], "C": [1, 3, 4, 5, 12, 19]}
else:  # tog_bwd_duo.hpp's
    NAMES = {0: "A: S A", 1: "A: wait B1", 2: "A: QR [Q.xx; S A]", 19: "A: (kmin)", 3: "A: wait B2a",
             4: "A: tmp1", 5: "A: chol_minus", 6: "A: wait B2b", 7: "A: S-update operands",
             8: "A: QR S-update", 9: "A: wait B3",
             10: "B: loads, Q.x/Q.u, S B", 11: "B: wait B1 / S A, S B rows", 12: "B: Q.ux",
             13: "B: QR [Q.uu; S B]", 14: "B: wait B2a", 15: "B: regularise + cond",
             16: "B: gains, K/d, s, dV", 17: "B: wait B2b", 18: "B: idle until B3"}
    WAVES = {"A": list(range(10)) + [19], "B": list(range(10, 19))}
pkg = __graft_entry__.load_package()
abi = pkg.abi
lib = abi.load_library()
read = lib.tog_bwd_prof_read
read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
prob, opts = pkg.Problems.config_quadrotor(B=1)
s = pkg.AbstractSolverFor(prob, opts)
h = s.handle
h.solve_init(abi.MODE_AL)
h.solve_step(3)
h.synchronize()
buf = (ctypes.c_ulonglong * 32)()
read(buf)
t0 = time.perf_counter()
h.solve_step(steps)
h.synchronize()
wall = time.perf_counter() - t0
assert read(buf) in (20, 32)
S = h.get(abi.FIELD_STATS)[0]
knots = steps * (prob.N - 1)
print(f"B=1 steps={steps} knots={knots} wall {1e3 * wall / steps:.3f} ms/step "
      f"(restarts in last step {int(S[abi.STAT_BP_RESTARTS])})")
for wname, ids in WAVES.items():
    tot = sum(buf[i] for i in ids)
    print(f"wave {wname}: {tot / knots:.1f} cyc/knot")
    for i in ids:
        print(f"  {NAMES.get(i, '-'):40s} {100.0 * buf[i] / max(tot, 1):6.2f}%  {buf[i] / knots:9.1f} cyc/knot")
# the tail rollouts (k_ls_spec_tail2), per solver step
T2 = {20: "rollout A: dynamics (per ring group)", 21: "rollout A: wait for B", 22: "rollout B: stage costs, stores",
      23: "rollout B: staging", 24: "rollout B: wait for A"}
tot2 = sum(buf[i] for i in T2)
print(f"tail rollouts: {tot2 / steps:.0f} cyc/step (both waves)")
for i, nm in T2.items():
    print(f"  {nm:40s} {buf[i] / steps:12.0f} cyc/step")
