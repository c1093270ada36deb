"""Canned problems (``TrajectoryOptimization.Problems``, src/problems.jl:14-24) and the
BASELINE.json benchmark configurations with their synthetic batched inputs
(SURVEY.md §8(d)). Every constructor cites the reference file it restates."""
from __future__ import annotations

import math

import numpy as np

from .problem import (BoundConstraint, CircleConstraints, Constraints, Dynamics, LQRCost, LQRCostTerminal,
                      LQRObjective, Objective, Problem, discretize_model, infeasible_problem,
                      SphereConstraints, goal_constraint, rk3, rk4)
from .solvers import ALTROSolverOptions, AugmentedLagrangianSolverOptions, iLQRSolverOptions

HOVER = 0.5 * 9.81 / 4.0


def doubleintegrator(U0=None, seed=0):
    """problems/doubleintegrator.jl:1-31 (config 1)."""
    model_d = rk3(Dynamics.doubleintegrator)
    n, m = 2, 1
    Q, Qf, R = np.eye(n), np.eye(n), 0.1 * np.eye(m)
    x0, xf = np.array([0.0, 0.0]), np.array([1.0, 0.0])
    N, dt = 21, 0.1
    if U0 is None:
        U0 = 0.001 * np.random.default_rng(seed).random((N - 1, m))
    obj = LQRObjective(Q, R, Qf, xf, N)
    bnd = BoundConstraint(n, m, u_max=1.5, u_min=-1.5, trim=True)
    goal = goal_constraint(xf)
    cons = Constraints(N)
    for k in range(N - 1):
        cons[k] += bnd
    cons[N - 1] += goal
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def cartpole(constrained=True, x0=None, U0=None):
    """problems/cartpole.jl:1-28. ``constrained=False`` gives config 2's unconstrained problem."""
    model_d = rk3(Dynamics.cartpole)
    n, m = 4, 1
    Q, Qf, R = 1e-2 * np.eye(n), 100.0 * np.eye(n), 1e-1 * np.eye(m)
    xf = np.array([0.0, math.pi, 0.0, 0.0])
    N, tf = 101, 5.0
    dt = tf / (N - 1)
    if x0 is None:
        x0 = np.zeros(n)
    if U0 is None:
        U0 = 0.01 * np.ones((N - 1, m))
    obj = LQRObjective(Q, R, Qf, xf, N)
    cons = Constraints(N)
    if constrained:
        bnd = BoundConstraint(n, m, u_min=-3.0, u_max=3.0)
        goal = goal_constraint(xf)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += goal
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def quadrotor_test(constraints="goal+bounds", x0=None, U0=None, integration="rk4"):
    """test/quadrotor_tests.jl:4-84: rk4, N=101, dt=0.05, Q=R=1e-2 I, Qf=1000 I.
    constraints in {"none", "goal", "goal+bounds", "goal+bounds+obs"}."""
    model_d = rk4(Dynamics.quadrotor) if integration == "rk4" else rk3(Dynamics.quadrotor)
    n, m = 13, 4
    Q, R, Qf = 1e-2 * np.eye(n), 1e-2 * np.eye(m), 1000.0 * np.eye(n)
    q0 = np.array([1.0, 0.0, 0.0, 0.0])
    if x0 is None:
        x0 = np.zeros(n)
        x0[3:7] = q0
    xf = np.zeros(n)
    xf[0:3] = [0.0, 50.0, 0.0]
    xf[3:7] = q0
    N, dt = 101, 0.05
    if U0 is None:
        U0 = HOVER * np.ones((N - 1, m))
    obj = LQRObjective(Q, R, Qf, xf, N)
    goal = goal_constraint(xf)
    bnd = BoundConstraint(n, m, u_min=0.0, u_max=15.0, trim=True)
    if constraints == "none":
        con = []
    elif constraints == "goal":
        con = [goal]
    elif constraints == "goal+bounds":
        con = [bnd, goal]
    elif constraints == "goal+bounds+obs":
        r_quad, r_sphere = 1.0, 3.0
        spheres = [(0.0, 10.0, 0.0, r_sphere + r_quad), (0.0, 20.0, 0.0, r_sphere + r_quad),
                   (0.0, 30.0, 0.0, r_sphere + r_quad)]
        con = [bnd, SphereConstraints(n, m, spheres, "obs"), goal]
    else:
        raise ValueError(constraints)
    cons = Constraints(con, N) if con else Constraints(N)
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def quad_obs(N=101, x0=None, U0=None):
    """problems/quad_obs.jl:1-89 "as written" (the sphere radius argument is
    z+r_quad, and the file initialises the other problem's controls, so U starts at 0)."""
    model_d = rk3(Dynamics.quadrotor)
    n, m = 13, 4
    q0 = np.array([1.0, 0.0, 0.0, 0.0])
    if x0 is None:
        x0 = np.zeros(n)
        x0[0:3] = [0.0, 0.0, 10.0]
        x0[3:7] = q0
    xf = np.zeros(n)
    xf[0:3] = [0.0, 60.0, 10.0]
    xf[3:7] = q0
    Q = 1e-3 * np.eye(n)
    Q[3:7, 3:7] = 1e-3 * np.eye(4)
    R = 1e-2 * np.eye(m)
    Qf = 1.0 * np.eye(n)
    u_min, u_max = 0.0, 50.0
    x_max = np.full(n, np.inf)
    x_min = np.full(n, -np.inf)
    x_max[0:3] = [25.0, np.inf, 20.0]
    x_min[0:3] = [-25.0, -np.inf, 0.0]
    bnd_u = BoundConstraint(n, m, u_min=u_min, u_max=u_max)
    bnd = BoundConstraint(n, m, u_min=u_min, u_max=u_max, x_min=x_min, x_max=x_max)
    xf_U = xf.copy()
    xf_L = xf.copy()
    xf_U[3:7] = np.inf
    xf_L[3:7] = -np.inf
    xf_U[7:10] = 0.0
    xf_L[7:10] = 0.0
    bnd_xf = BoundConstraint(n, m, x_min=xf_L, x_max=xf_U)
    tf = 5.0
    dt = tf / (N - 1)
    obj = LQRObjective(Q, R, Qf, xf, N)
    r_quad = 2.0
    cyl = [(0.0, 10.0, 3.0), (10.0, 30.0, 3.0), (-13.0, 25.0, 2.0), (5.0, 50.0, 4.0)]
    sph = [(0.0, 40.0, 5.0, 2.0), (-5.0, 15.0, 3.0, 1.0), (10.0, 20.0, 7.0, 2.0)]
    cyl_con = CircleConstraints(n, m, [(c[0], c[1], c[2] + r_quad) for c in cyl], "cylinders")
    sph_con = SphereConstraints(n, m, [(s[0], s[1], s[2], s[2] + r_quad) for s in sph], "spheres")  # A.6
    cons = Constraints(N)
    cons[0] += bnd_u
    for k in range(1, N - 1):
        cons[k] += bnd + cyl_con + sph_con
    cons[N - 1] += bnd_xf
    if U0 is None:
        U0 = np.zeros((N - 1, m))
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def car_sqrt_bp(constrained=False):
    """test/sqrt_bp_tests.jl:1-16 / :46-56: car, rk4, N=31, dt=0.15, U=ones, Q=R=1e-3 I,
    Qf=100 I, xf=[0,1,0]; constrained adds bounds ±5 and the goal."""
    model_d = rk4(Dynamics.car)
    n, m = 3, 2
    Q, R, Qf = 1e-3 * np.eye(n), 1e-3 * np.eye(m), 100.0 * np.eye(n)
    x0, xf = np.zeros(n), np.array([0.0, 1.0, 0.0])
    N, dt = 31, 0.15
    obj = LQRObjective(Q, R, Qf, xf, N)
    cons = Constraints(N)
    if constrained:
        bnd = BoundConstraint(n, m, u_min=-5.0, u_max=5.0, trim=True)
        cons = Constraints([bnd, goal_constraint(xf)], N)
    return Problem(model_d, obj, np.ones((N - 1, m)), constraints=cons, x0=x0, N=N, dt=dt)


def pendulum(integration="rk3", U0=None, model=None, stage_constraints=()):
    """problems/pendulum.jl:1-35: rk3, N=31, dt=0.15, Q=R=Qf=1e-3 I, xf=[π,0], |u|<=3 at
    k<N, goal at N, U=ones. ``model``: another continuous model with the pendulum's n, m (e.g. a
    user plugin of the same dynamics)."""
    model_d = discretize_model(model or Dynamics.pendulum, integration)
    n, m = 2, 1
    Q, R = 1e-3 * np.eye(n), 1e-3 * np.eye(m)
    x0, xf = np.zeros(n), np.array([math.pi, 0.0])
    N, dt = 31, 0.15
    if U0 is None:
        U0 = np.ones((N - 1, m))
    cons = Constraints(N)
    bnd = BoundConstraint(n, m, u_min=-3.0, u_max=3.0)
    for k in range(N - 1):
        cons[k] += bnd
        for c in stage_constraints:
            cons[k] += c
    cons[N - 1] += goal_constraint(xf)
    obj = LQRObjective(Q, R, Q, xf, N)
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def car_parallel_park(U0=None):
    """test/car_tests.jl:4-32: car, rk3, N=101, dt=0.1, Q=R=1e-2 I, Qf=1000 I, x0=0, xf=[0,1,0],
    U=ones, unconstrained (iLQR with cost_tolerance=1e-5)."""
    model_d = rk3(Dynamics.car)
    n, m = 3, 2
    Q, R, Qf = 1e-2 * np.eye(n), 1e-2 * np.eye(m), 1000.0 * np.eye(n)
    x0, xf = np.zeros(n), np.array([0.0, 1.0, 0.0])
    N, dt = 101, 0.1
    if U0 is None:
        U0 = np.ones((N - 1, m))
    obj = LQRObjective(Q, R, Qf, xf, N)
    return Problem(model_d, obj, U0, x0=x0, xf=xf, N=N, dt=dt)


def car_obstacles(U0=None, u_max=1.5, B=1):
    """test/projected_newton_test.jl:1-27 (the projected Newton tests' problem; test/altro_tests.jl:1-21
    is the same with ``Dynamics.car_costfun``, which this snapshot does not define): car, rk4, N=51,
    tf=3, Q=R=Qf=1e-2 I, xf=[0,1,0]; knot 1: u_min; knots 2..N-1: x in [-0.5,0.5]x[-0.01,1.01],
    u in [0.1,-2]..u_max, two planar obstacles; knot N: goal; U = ones."""
    model_d = rk4(Dynamics.car)
    n, m, N = 3, 2, 51
    dt = 3.0 / (N - 1)
    Q, R, Qf = 0.01 * np.eye(n), 0.01 * np.eye(m), 0.01 * np.eye(n)
    xf = np.array([0.0, 1.0, 0.0])
    obj = LQRObjective(Q, R, Qf, xf, N)
    bnd = BoundConstraint(n, m, x_min=[-0.5, -0.01, -math.inf], x_max=[0.5, 1.01, math.inf], u_min=[0.1, -2.0],
                          u_max=u_max)
    bnd1 = BoundConstraint(n, m, u_min=[0.1, -2.0])
    obs1 = CircleConstraints(n, m, [[0.2, 0.6, 0.25]], label="obstacle1")
    obs2 = CircleConstraints(n, m, [[-0.5, 0.5, 0.4]], label="obstacle2")
    cons = Constraints(N)
    cons[0] += bnd1
    for k in range(1, N - 1):
        cons[k] += bnd
        cons[k] += obs1
        cons[k] += obs2
    cons[N - 1] += goal_constraint(xf)
    if U0 is None:
        U0 = np.ones((N - 1, m))
    U0 = np.asarray(U0, dtype=np.float64)
    if B > 1 and U0.ndim == 2:
        U0 = np.broadcast_to(U0, (B,) + U0.shape).copy()
    B = U0.shape[0] if U0.ndim == 3 else B
    x0 = np.zeros((B, n)) if B > 1 else np.zeros(n)
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


# ---------------------------------------------------------------------------- BASELINE configs

def dynamics_bias(model, x):
    """``RigidBodyDynamics.dynamics_bias(state)`` at x = [q; v] (the libtog host evaluation of the
    same model code the kernels run; RBD models only)."""
    from . import abi
    x = np.ascontiguousarray(x, dtype=np.float64)
    if x.shape != (model.n,):
        raise ValueError(f"x must have length {model.n}")
    tau = np.zeros(model.m)
    lib = abi.load_library()
    abi.check(lib, lib.tog_dynamics_bias(model.model_id, x.ctypes.data_as(abi._dp), tau.ctypes.data_as(abi._dp)))
    return tau


def hold_trajectory(n, m, N, model, q):
    """dynamics/kuka.jl:117-132: U0[:, k] = dynamics_bias at configuration q, zero velocity.
    Returns (N, m) like the reference's m x N matrix (only the first N-1 columns are used)."""
    q = np.asarray(q, dtype=np.float64)
    nq = model.n // 2
    if len(q) > m:
        raise ValueError(f"system must be fully actuated to hold an arbitrary position ({len(q)} should be > {m})")
    x = np.zeros(model.n)
    x[:nq] = q[:nq]
    return np.tile(dynamics_bias(model, x), (N, 1))


def kuka(x0=None, U0=None, N=51, tf=5.0):
    """examples/kuka_iiwa/Kuka iiwa.ipynb cells 7-15: x0 = 0, xf[1:2] = pi/2, Q = diag(1x7, 100x7),
    Qf = 1000 I, R = 1e-2 I, N = 51, tf = 5, rk3, terminal goal constraint, U0 = hold trajectory."""
    model_d = rk3(Dynamics.kuka)
    n, m = 14, 7
    if x0 is None:
        x0 = np.zeros(n)
    xf = np.zeros(n)
    xf[0] = math.pi / 2
    xf[1] = math.pi / 2
    Q = np.diag(np.r_[np.ones(7), 100.0 * np.ones(7)])
    Qf = 1000.0 * np.eye(n)
    R = 1e-2 * np.eye(m)
    dt = tf / (N - 1)
    if U0 is None:
        U0 = hold_trajectory(n, m, N, Dynamics.kuka, np.asarray(x0)[:7])[: N - 1]
    obj = LQRObjective(Q, R, Qf, xf, N)
    cons = Constraints(N)
    cons[N - 1] += goal_constraint(xf)
    return Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)


def kuka_options():
    """The notebook's solver options (Kuka iiwa.ipynb cell 11)."""
    opts_ilqr = iLQRSolverOptions(iterations=300)
    return AugmentedLagrangianSolverOptions(opts_uncon=opts_ilqr, iterations=20, cost_tolerance=1.0e-6,
                                            cost_tolerance_intermediate=1.0e-5, constraint_tolerance=1.0e-3,
                                            penalty_scaling=50.0, penalty_initial=0.01)


def _per_traj_rng(seed0, B, fn):
    return np.stack([fn(np.random.default_rng(seed0 + b)) for b in range(B)])


def config_cartpole(B=1024, offset=0):
    """Config 2: cartpole swing-up, unconstrained iLQR, U0[b] = 0.01 + 0.5 N(0,1) (seed 1000+b)."""
    N, m = 101, 1
    U0 = _per_traj_rng(1000 + offset, B, lambda r: 0.01 + 0.5 * r.standard_normal((N - 1, m)))
    prob = cartpole(constrained=False, x0=np.zeros((B, 4)), U0=U0)
    return prob, iLQRSolverOptions()


def config_quadrotor(B=8192, offset=0):
    """Config 3: quadrotor point-to-point, AL-iLQR with u in [0,15] + goal, square-root BP.
    U0 = hover + 0.1 N(0,1), x0[1:3] += N(0,1) (seed 2000+b)."""
    N, n, m = 101, 13, 4

    def gen(r):
        x0 = np.zeros(n)
        x0[3] = 1.0
        x0[0:3] += r.standard_normal(3)
        U0 = HOVER + 0.1 * r.standard_normal((N - 1, m))
        return np.concatenate([x0, U0.ravel()])

    Z = _per_traj_rng(2000 + offset, B, gen)
    x0 = Z[:, :n]
    U0 = Z[:, n:].reshape(B, N - 1, m)
    prob = quadrotor_test("goal+bounds", x0=x0, U0=U0)
    opts_ilqr = iLQRSolverOptions(cost_tolerance=1e-5, square_root=True)
    opts_al = AugmentedLagrangianSolverOptions(opts_uncon=opts_ilqr, constraint_tolerance=1e-3,
                                               cost_tolerance=1e-5, cost_tolerance_intermediate=1e-4)
    return prob, opts_al


def config_quadrotor_tv(B=8192, offset=0):
    """Config 3 with a time-varying Objective (src/objective.jl:15-29): knot k's stage cost is
    LQRCost(Q w_k, R v_k, xf), w_k rising 0.5 -> 2.0 and v_k falling 2.0 -> 1.0 along the horizon (100 stage
    costs and the terminal one); the starts and options are config 3's. The bench's per-knot-cost line."""
    prob, opts = config_quadrotor(B=B, offset=offset)
    st, term = prob.obj.stage, prob.obj.terminal
    N = prob.N
    costs = []
    for k in range(N - 1):
        w = 0.5 + 1.5 * k / (N - 2)
        v = 2.0 - 1.0 * k / (N - 2)
        costs.append(LQRCost(w * st.Q, v * st.R, prob.xf))
    obj = Objective(costs + [LQRCostTerminal(term.Q, prob.xf)])
    p = Problem(prob.model, obj, prob._U.copy(), constraints=prob.constraints, x0=prob.x0.copy(), xf=prob.xf,
                N=N, dt=prob.dt)
    return p, opts


def config_quad_maze(B=8192, offset=0, N=201):
    """Config 4 (per GPU shard): quad_obs with N=201, dt=0.025; x0[1:3] ~ U([-5,5]x[-3,0]x[8,12]),
    U0 = hover + 0.1 N (seed 3000+b)."""
    n, m = 13, 4

    def gen(r):
        x0 = np.zeros(n)
        x0[3] = 1.0
        x0[0:3] = [r.uniform(-5, 5), r.uniform(-3, 0), r.uniform(8, 12)]
        U0 = HOVER + 0.1 * r.standard_normal((N - 1, m))
        return np.concatenate([x0, U0.ravel()])

    Z = _per_traj_rng(3000 + offset, B, gen)
    prob = quad_obs(N=N, x0=Z[:, :n], U0=Z[:, n:].reshape(B, N - 1, m))
    return prob, AugmentedLagrangianSolverOptions()


def config_kuka(B=4096, offset=0):
    """Config 5: Kuka iiwa (n=14, m=7, N=51), AL-iLQR with the terminal goal and the notebook's options;
    x0[1:7] ~ U(-0.2, 0.2) (seed 4000+b), U0 = the hold trajectory at x0 (the notebook's own
    initialisation, Kuka iiwa.ipynb cell 15). SURVEY §8(d) proposed hold + 0.1 N(0,1): with link 7's
    3e-4 kg m^2 inertia that open-loop rollout diverges within ~10 knots, so the batch differs by x0."""
    N, n, m = 51, 14, 7
    x0 = np.zeros((B, n))
    for b in range(B):
        x0[b, :7] = np.random.default_rng(4000 + offset + b).uniform(-0.2, 0.2, 7)
    U0 = np.stack([hold_trajectory(n, m, N, Dynamics.kuka, x0[b, :7])[: N - 1] for b in range(B)])
    return kuka(x0=x0, U0=U0, N=N), kuka_options()


def config_doubleintegrator(B=1):
    """Config 1: double integrator block move, ALTRO defaults."""
    prob = doubleintegrator()
    return prob, ALTROSolverOptions()


def interp_rows(N, tf, X):
    """``interp_rows(N, tf, X)`` (src/utils.jl:5-15): each row of X (n, N1) through a cubic spline
    on range(0, tf, N1), sampled on range(0, tf, N). The reference uses Interpolations.jl's
    ``CubicSplineInterpolation`` (BSpline(Cubic(Line(OnGrid())))) — not installed here; its Line
    boundary condition is the natural spline (zero second derivative at both ends), restated with
    scipy. Used only to build initial guesses."""
    from scipy.interpolate import CubicSpline

    X = np.asarray(X, dtype=np.float64)
    t1 = np.linspace(0.0, tf, X.shape[1])
    t2 = np.linspace(0.0, tf, N)
    return np.stack([CubicSpline(t1, X[i], bc_type="natural")(t2) for i in range(X.shape[0])])


def quadrotor_maze(N=101, waypoints=None):
    """problems/quadrotor_maze.jl:1-114: quadrotor (rk3) through 38 cylinders, u in [0, 50],
    x/z box, terminal box on position/velocity; initial controls hover, initial *state* guess
    interp_rows of 7 way-points — an infeasible start (ALTRO solves it via slack controls)."""
    model_d = rk3(Dynamics.quadrotor)
    n, m = 13, 4
    q0 = np.array([1.0, 0.0, 0.0, 0.0])
    x0 = np.zeros(n)
    x0[0:3] = [0.0, 0.0, 10.0]
    x0[3:7] = q0
    xf = np.zeros(n)
    xf[0:3] = [0.0, 60.0, 10.0]
    xf[3:7] = q0
    Q = 1e-3 * np.eye(n)
    Q[3:7, 3:7] = 1e-2 * np.eye(4)
    R = 1e-4 * np.eye(m)
    Qf = 1000.0 * np.eye(n)
    r_quad, r_cyl = 2.0, 2.0
    cyl = []
    for i in np.linspace(-25, -10, 5):
        cyl.append((i, 10.0, r_cyl))
    for i in np.linspace(10, 25, 5):
        cyl.append((i, 10.0, r_cyl))
    for i in np.linspace(-5, 5, 4):
        cyl.append((i, 30.0, r_cyl))
    for i in np.linspace(-25, -10, 5):
        cyl.append((i, 50.0, r_cyl))
    for i in np.linspace(10, 25, 5):
        cyl.append((i, 50.0, r_cyl))
    for i in np.linspace(10 + 2 * r_cyl, 50 - 2 * r_cyl, 10):
        cyl.append((-25.0, i, r_cyl))
    for i in np.linspace(10 + 2 * r_cyl, 50 - 2 * r_cyl, 10):
        cyl.append((25.0, i, r_cyl))
    maze = CircleConstraints(n, m, [(cx, cy, r + r_quad) for (cx, cy, r) in cyl], "maze")
    x_max = np.full(n, np.inf)
    x_min = np.full(n, -np.inf)
    x_max[0:3] = [25.0, np.inf, 20.0]
    x_min[0:3] = [-25.0, -np.inf, 0.0]
    bnd1 = BoundConstraint(n, m, u_min=0.0, u_max=50.0)
    bnd2 = BoundConstraint(n, m, u_min=0.0, u_max=50.0, x_min=x_min, x_max=x_max)
    xU, xL = xf.copy(), xf.copy()
    xU[3:7], xL[3:7] = np.inf, -np.inf
    xU[7:10], xL[7:10] = 0.0, 0.0
    bnd_xf = BoundConstraint(n, m, x_min=xL, x_max=xU)
    tf = 5.0
    dt = tf / (N - 1)
    cons = Constraints(N)
    cons[0] += bnd1
    stage = bnd2 + maze
    for k in range(1, N - 1):
        cons[k] = stage
    cons[N - 1] += bnd_xf
    obj = LQRObjective(Q, R, Qf, xf, N)
    U0 = HOVER * np.ones((N - 1, m))
    prob = Problem(model_d, obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=dt)
    prob.X = _maze_guess(N, tf, x0, xf, waypoints)
    return prob


_MAZE_WAYPOINTS = np.array([[0, -12.5, -20, -12.5, 0], [15, 20, 30, 40, 45], [10, 10, 10, 10, 10]], dtype=float)


def _maze_guess(N, tf, x0, xf, waypoints=None):
    """X_guess of problems/quadrotor_maze.jl:107-114 through interp_rows: (N, n)."""
    Xg = np.zeros((len(x0), 7))
    Xg[:, 0] = x0
    Xg[:, 6] = xf
    Xg[0:3, 1:6] = _MAZE_WAYPOINTS if waypoints is None else waypoints
    Xg[3:7, :] = np.array([1.0, 0.0, 0.0, 0.0])[:, None]
    return interp_rows(N, tf, Xg).T


def maze_altro_options():
    """test/infeasible_tests.jl:57-76 (the reference's quadrotor_maze case)."""
    il = iLQRSolverOptions(iterations=300)
    al = AugmentedLagrangianSolverOptions(opts_uncon=il, iterations=40, cost_tolerance=1e-5,
                                          cost_tolerance_intermediate=1e-4, constraint_tolerance=1e-3,
                                          penalty_scaling=10.0, penalty_initial=1.0)
    return ALTROSolverOptions(resolve_feasible_problem=False, opts_al=al, R_inf=0.001)


def quadrotor_maze_iros_options():
    """The ALTRO options of the reference's IROS 2019 quadrotor maze demo
    (examples/IROS_2019/quadrotor_maze.jl:8-34): AL to 1e-4 (projected_newton_tolerance), then projected
    Newton's feasible projection to 1e-8, R_inf = 1e-8, no resolve. The reference publishes 85.8 s and a final
    violation of 9.63e-9 for one solve (examples/quadrotor/Quadrotor Maze.ipynb, cell 3)."""
    il = iLQRSolverOptions(iterations=300)
    al = AugmentedLagrangianSolverOptions(opts_uncon=il, iterations=40, cost_tolerance=1e-5,
                                          cost_tolerance_intermediate=1e-4, constraint_tolerance=1e-8,
                                          penalty_scaling=10.0, penalty_initial=1.0)
    opts = ALTROSolverOptions(opts_al=al, R_inf=1e-8, resolve_feasible_problem=False,
                              projected_newton=True, projected_newton_tolerance=1e-4)
    opts.opts_pn.feasibility_tolerance = 1e-8
    opts.opts_pn.solve_type = "feasible"
    return opts


def quadrotor_maze_batch(B, offset=0, jitter=0.5):
    """B copies of ``quadrotor_maze()`` whose state guesses are the five interior way-points of
    problems/quadrotor_maze.jl:104-113 jittered by N(0, jitter^2) per coordinate (seed 5000+offset+b; jitter 0
    gives the reference's own guess), hover controls."""
    p0 = quadrotor_maze()
    N = p0.N
    Xs = _per_traj_rng(5000 + offset, B, lambda r: _maze_guess(
        N, 5.0, p0.x0[0], p0.xf, _MAZE_WAYPOINTS + jitter * r.standard_normal(_MAZE_WAYPOINTS.shape)).ravel())
    p0b = Problem(p0.model, p0.obj, np.broadcast_to(p0.U, (B, N - 1, 4)).copy(), constraints=p0.constraints,
                  x0=np.tile(p0.x0[0], (B, 1)), xf=p0.xf, N=N, dt=p0.dt)
    p0b.X = Xs.reshape(B, N, 13)
    return p0b


def config_quadrotor_maze_infeasible(B=1024, offset=0):
    """The quadrotor_maze infeasible-start AL phase (ALTRO with a state guess) as a batch: the five
    interior way-points of problems/quadrotor_maze.jl jittered by N(0, 0.5^2) per coordinate (seed
    5000+b), hover controls; returns the *infeasible* problem (slack controls still to be filled
    by ``slack_controls``) and the ALTRO options."""
    p0b = quadrotor_maze_batch(B, offset)
    opts = maze_altro_options()
    return infeasible_problem(p0b, opts.R_inf), opts


# --------------------------------------------------------------------- user models (plugins)
# Model(f!, n, m) (src/model.jl:103-131) with user dynamics compiled into a libtog plugin
# (csrc/tog_plugin.hpp). The unicycle below is not among the built-in dynamics.
UNICYCLE_F = """
const double cv = 0.1, cw = 0.2;
xd[0] = x[3] * cos_(x[2]);
xd[1] = x[3] * sin_(x[2]);
xd[2] = x[4];
xd[3] = u[0] - cv * x[3];
xd[4] = u[1] - cw * x[4];
"""


# user constraint functions of the unicycle: fid 0 a disc obstacle at (1, 0.5), r = 0.3; fid 1 the
# traction limit a v <= 1 (a control-dependent row)
UNICYCLE_CON = """
if (fid == 0) {
  const T dx = x[0] - 1.0, dy = x[1] - 0.5;
  c[0] = -((dx * dx + dy * dy) - 0.09);
} else {
  c[0] = u[0] * x[3] - 1.0;
}
"""


def unicycle_model():
    """The unicycle with first-order actuators as a user model: x = [px, py, θ, v, ω], u = [a, α],
    with the user constraint functions UNICYCLE_CON."""
    from .problem import user_model

    return user_model(UNICYCLE_F, 5, 2, name="Unicycle", con_body=UNICYCLE_CON)


def unicycle_constraints(n=5, m=2):
    """UserConstraint rows of the unicycle's con(): the obstacle (fid 0) and the traction limit (fid 1),
    with host restatements for max_violation(prob)."""
    from .problem import UserConstraint

    obs = UserConstraint(n, m, 1, fid=0, label="obstacle",
                         host=lambda x, u: np.array([-((x[0] - 1.0) ** 2 + (x[1] - 0.5) ** 2 - 0.09)]))
    trac = UserConstraint(n, m, 1, fid=1, label="traction", host=lambda x, u: np.array([u[0] * x[3] - 1.0]))
    return obs, trac


def unicycle(model=None, B=1, offset=0, N=51, dt=0.1, user_constraints=False):
    """Drive the unicycle from rest at the origin to xf = (2, 1, 0, 0, 0): rk3, LQR objective
    (Q = 1e-2 I, R = 1e-1 I, Qf = 100 I), |u| <= 2 at every stage knot, goal at N. U0 = 0.1 N(0,1)
    (seed 6000+b)."""
    model_d = rk3(model or unicycle_model())
    n, m = 5, 2
    xf = np.array([2.0, 1.0, 0.0, 0.0, 0.0])
    U0 = _per_traj_rng(6000 + offset, B, lambda r: 0.1 * r.standard_normal((N - 1, m)))
    cons = Constraints(N)
    bnd = BoundConstraint(n, m, u_min=-2.0, u_max=2.0)
    extra = unicycle_constraints(n, m) if user_constraints else ()
    for k in range(N - 1):
        cons[k] += bnd
        for c in extra:
            cons[k] += c
    cons[N - 1] += goal_constraint(xf)
    obj = LQRObjective(1e-2 * np.eye(n), 1e-1 * np.eye(m), 100.0 * np.eye(n), xf, N)
    return Problem(model_d, obj, U0 if B > 1 else U0[0], constraints=cons, x0=np.zeros((B, n)) if B > 1 else np.zeros(n),
                   xf=xf, N=N, dt=dt)
