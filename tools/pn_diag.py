"""Diagnostic: device AL phase (ALTRO, projected_newton off) vs oracle on the batched car problem,
then device PN from the device AL iterate vs oracle PN from the oracle AL iterate."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import __graft_entry__ as g
from test_projected_newton import car_batch, car_al_opts, rel

tog = g.load_package()
orc = g.load_oracle()
prob = car_batch(tog, 3, seed=11)
al = car_al_opts(tog, tol=1e-2)
opts = tog.ALTROSolverOptions(opts_al=al)
gp = prob.copy()
solver = tog.solve_b(gp, opts)
for b in range(prob.B):
    o = orc.OracleSolver(prob, opts, b=b)
    steps = o.solve()
    print(b, "AL rel X", rel(gp._X[b], o.get("X")), "rel U", rel(gp._U[b], o.get("U")), "steps", steps,
          solver.stats["iterations_total"][b], "cmax", o.max_violation(), solver.stats["c_max"][b])
