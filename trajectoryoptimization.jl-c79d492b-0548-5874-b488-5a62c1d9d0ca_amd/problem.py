"""Host-side mirror of the reference's problem definition layer (L0 in SURVEY.md §1):
``Model``/``rk3``/``rk4`` (src/model.jl), ``QuadraticCost``/``LQRCost`` (src/cost.jl),
``Objective``/``LQRObjective`` (src/objective.jl), ``BoundConstraint``/``goal_constraint``
(src/constraints.jl), ``Constraints`` (src/constraint_sets.jl) and ``Problem``
(src/problem.jl).

These are plain data holders: they are marshalled into ``tog_problem_desc`` (include/tog.h)
and every computation runs in libtog.so on the GPU. The small ``evaluate``/``jacobian``
helpers on constraints exist for the reference's own unit assertions
(test/constraint_tests.jl) and for ``max_violation(prob)``, which the reference evaluates
on the host after a solve (src/problem.jl:242-267).

Julia → Python naming: a trailing ``!`` becomes ``_b`` (``solve!`` → ``solve_b``), 1-based
knot ``k`` becomes 0-based ``k-1``; trajectories are numpy arrays ``X[N, n]`` (one trajectory)
or ``X[B, N, n]`` (a batch), which is exactly the C-ABI memory layout.
"""
from __future__ import annotations

import copy as _copy
import math
import pathlib
from dataclasses import dataclass, field

import numpy as np

from . import abi

# ----------------------------------------------------------------------------- models


@dataclass
class Model:
    """``AnalyticalModel{Nominal, Continuous|Discrete}`` (src/model.jl:36-74).

    Either one of the canned dynamics built into libtog (``Dynamics.*``) or a user model
    ``Model(f!, n, m)`` (src/model.jl:103-131) compiled into a plugin (``user_model`` /
    ``Model.from_plugin``, csrc/tog_plugin.hpp). A discrete model carries its integrator
    (``rk3``/``rk4``, src/model.jl:642-644).
    """

    model_id: int
    n: int
    m: int
    name: str
    integration: int | None = None  # None = Continuous; abi.RK3 / abi.RK4 = Discrete
    slack: int = 0  # add_slack_controls: the last `slack` (= n) controls are infeasible slacks
    plugin: "UserModelPlugin | None" = None  # model_id == abi.MODEL_USER
    min_time: bool = False  # add_min_time_controls: x = [x; τ], u = [u; h], dt_k = h_k² (last state / control)

    @staticmethod
    def from_plugin(path, name: str | None = None) -> "Model":
        """A user model from a compiled plugin (``tog_model_load``); n, m come from the plugin."""
        plug = UserModelPlugin.load(path)
        return Model(abi.MODEL_USER, plug.n, plug.m, name or pathlib.Path(path).stem, plugin=plug)

    @property
    def discrete(self) -> bool:
        return self.integration is not None


def discretize_model(model: Model, discretizer: str = "rk3", dt: float = 1.0) -> Model:
    """``discretize_model(model, :rk3|:rk4)`` (src/model.jl:607-615)."""
    if model.discrete:
        raise ValueError("model is already discrete")
    key = discretizer.lstrip(":")
    integs = {"rk3": abi.RK3, "rk4": abi.RK4, "midpoint": abi.MIDPOINT, "rk3_implicit": abi.RK3_IMPLICIT,
              "midpoint_implicit": abi.MIDPOINT_IMPLICIT}
    if key not in integs:
        raise ValueError(f"Integration not defined: {discretizer!r}")  # src/model.jl:659
    builtin_implicit = model.plugin is None and model.model_id in (abi.MODEL_QUADROTOR, abi.MODEL_KUKA)
    if integs[key] in (abi.RK3_IMPLICIT, abi.MIDPOINT_IMPLICIT) and model.n > 4 and not builtin_implicit:
        # the device instantiates the implicit Newton step for n <= 4, the built-in quadrotor and the Kuka
        # arm (ModelTraits::implicit_ok, csrc/tog_device.hpp), decided by model id as the runtime does
        raise NotImplementedError(f"implicit integration {discretizer!r} is built for models with n <= 4, "
                                  "the quadrotor and the Kuka arm")
    return Model(model.model_id, model.n, model.m, model.name, integs[key], plugin=model.plugin)


def midpoint(model: Model, dt: float = 1.0) -> Model:
    """``midpoint(model)`` (src/model.jl:642, src/integration.jl:26-33)."""
    return discretize_model(model, "midpoint", dt)


def midpoint_implicit(model: Model, dt: float = 1.0) -> Model:
    """``midpoint_implicit(model)`` (src/model.jl:647, src/integration.jl:44-73): x+ solves
    g = x+ - x - dt f((x + x+)/2) = 0 by Newton iterations to ||g|| <= 1e-12."""
    return discretize_model(model, "midpoint_implicit", dt)


def rk3_implicit(model: Model, dt: float = 1.0) -> Model:
    """``rk3_implicit(model)`` (src/model.jl:646, src/integration.jl:171-205), including the
    reference's aliasing of its three stage buffers (see csrc/tog_device.hpp implicit_step)."""
    return discretize_model(model, "rk3_implicit", dt)


def add_slack_controls(model: Model) -> Model:
    """``add_slack_controls(model)`` (src/model.jl:761-779): a discrete model with n extra controls,
    x+ = f_d(x, u[1:m]) + u[m+1:m+n]; its Jacobian is [∇f | I]. The device evaluates it as
    ``Infeasible<M>`` (csrc/tog_device.hpp)."""
    if not model.discrete:
        raise ValueError("add_slack_controls needs a discrete model")
    if model.slack:
        raise ValueError("model already has slack controls")
    return Model(model.model_id, model.n, model.m + model.n, model.name + "_inf", model.integration, model.n,
                 plugin=model.plugin)


def rk3(model: Model, dt: float = 1.0) -> Model:
    return discretize_model(model, "rk3", dt)


def rk4(model: Model, dt: float = 1.0) -> Model:
    return discretize_model(model, "rk4", dt)


class UserModelPlugin:
    """A loaded user-model plugin (``tog_model_load``, include/tog.h). Kept alive by every
    ``Model`` built on it; freed (``tog_model_free``) when the last reference goes."""

    _cache: dict = {}

    def __init__(self, path, ptr, n, m):
        self.path, self.ptr, self.n, self.m = str(path), ptr, n, m

    @classmethod
    def load(cls, path):
        path = str(pathlib.Path(path).resolve())
        if path in cls._cache:
            return cls._cache[path]
        import ctypes as C

        lib = abi.load_library()
        h = C.c_void_p()
        abi.check(lib, lib.tog_model_load(path.encode(), C.byref(h)))
        n, m = C.c_int32(), C.c_int32()
        abi.check(lib, lib.tog_model_dims(h, C.byref(n), C.byref(m)))
        plug = cls(path, h.value, n.value, m.value)
        cls._cache[path] = plug  # a plugin stays loaded for the life of the process (kernels registered)
        return plug


_PLUGIN_TEMPLATE = """// generated by user_model() (problem.py): Model(f!, n, m) as a libtog plugin
#include "{hdr}"

struct {name} {{
  static constexpr int n = {n}, m = {m}, id = TOG_MODEL_USER;
  template <class T>
  __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {{
    using namespace tog;
{body}
  }}{con}
}};

TOG_PLUGIN({name})
"""

_CON_TEMPLATE = """
  static constexpr bool has_con = true;
  template <class T>
  __host__ __device__ __forceinline__ static void con(int fid, T* c, const T* x, const T* u) {{
    using namespace tog;
{body}
  }}
"""


def _prune_stale_plugins(out_dir: pathlib.Path, hh: str):
    """Remove generated plugins built against other libtog headers (their .hip records the hash):
    tog_model_load / tog_generic_cost_load would refuse them anyway."""
    for hip in out_dir.glob("gen_*.hip"):
        try:
            first = hip.read_text().split("\n", 1)[0]
        except OSError:
            continue
        if first != f"// libtog header hash {hh}":
            hip.with_suffix(".so").unlink(missing_ok=True)
            hip.unlink(missing_ok=True)


def user_model(f_body: str, n: int, m: int, name: str = "UserModel", build_dir=None, con_body: str | None = None) -> Model:
    """``Model(f!, n, m)`` (src/model.jl:103-131) for user dynamics: ``f_body`` is the body of
    ``f(T* xd, const T* x, const T* u)`` in C++ over the scalar type ``T`` (double in rollouts,
    dual numbers in the Jacobian kernel, as ForwardDiff differentiates the Julia f!). Use
    ``sin_``, ``cos_``, ``sqrt_``, ``inv_``. ``con_body`` (optional) is the body of the user
    constraint functions ``con(int fid, T* c, const T* x, const T* u)`` that ``UserConstraint``
    rows evaluate. The plugin is compiled once with hipcc for gfx950
    (cached by the hash of its source under ``csrc/plugins/``) and loaded with ``tog_model_load``."""
    import hashlib
    import subprocess

    csrc = pathlib.Path(__file__).resolve().parent / "csrc"
    out_dir = pathlib.Path(build_dir) if build_dir else csrc / "plugins"
    out_dir.mkdir(parents=True, exist_ok=True)
    body = "\n".join("    " + ln for ln in f_body.strip().splitlines())
    con = ""
    if con_body:
        con = _CON_TEMPLATE.format(body="\n".join("    " + ln for ln in con_body.strip().splitlines()))
    src = _PLUGIN_TEMPLATE.format(hdr=str(csrc / "tog_plugin.hpp"), name=name, n=int(n), m=int(m), body=body,
                                  con=con)
    hh = abi.header_hash()  # the plugin is compiled against (and cached under) libtog's header text
    src = f"// libtog header hash {hh}\n" + src
    key = hashlib.sha1(src.encode()).hexdigest()[:12]
    so = out_dir / f"gen_{name}_{key}.so"
    if not so.exists():
        _prune_stale_plugins(out_dir, hh)
        hip = out_dir / f"gen_{name}_{key}.hip"
        hip.write_text(src)
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-fPIC",
               f"-DTOG_HEADER_HASH=0x{hh}LL", "-shared", "-o", str(so), str(hip)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            hip.unlink(missing_ok=True)  # no broken source left in the plugin directory
            raise ValueError(f"user model {name!r} does not compile:\n{r.stderr[-4000:]}")
    model = Model.from_plugin(so, name)
    if (model.n, model.m) != (int(n), int(m)):
        raise ValueError("plugin dimensions do not match")
    return model


class Dynamics:
    """``TrajectoryOptimization.Dynamics`` canned models (src/dynamics.jl:23-32)."""

    doubleintegrator = Model(abi.MODEL_DOUBLE_INTEGRATOR, 2, 1, "doubleintegrator")  # double_integrator.jl
    cartpole = Model(abi.MODEL_CARTPOLE, 4, 1, "cartpole")  # dynamics/cartpole.jl:9-36
    quadrotor = Model(abi.MODEL_QUADROTOR, 13, 4, "quadrotor")  # dynamics/quadrotor.jl:10-71
    car = Model(abi.MODEL_CAR, 3, 2, "car")  # dynamics/car.jl:3-8
    pendulum = Model(abi.MODEL_PENDULUM, 2, 1, "pendulum")  # dynamics/pendulum.jl:3-12
    # Model(urdf_kuka) dynamics/kuka.jl:137 -> src/model.jl:394-447 (RBD, tables include/tog_kuka.h)
    kuka = Model(abi.MODEL_KUKA, 14, 7, "kuka")


# ----------------------------------------------------------------------------- costs


def _mat(a, shape):
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 0:
        a = a * np.eye(shape[0])
    return np.array(a.reshape(shape), dtype=np.float64)


class QuadraticCost:
    """``QuadraticCost(Q, R, H, q, r, c)`` (src/cost.jl:112-131):
    1/2 x'Qx + 1/2 u'Ru + u'Hx + q'x + r'u + c (times dt for stage costs)."""

    def __init__(self, Q, R=None, H=None, q=None, r=None, c=0.0):
        Q = np.asarray(Q, dtype=np.float64)
        n = Q.shape[0]
        if R is None:  # QuadraticCost(Q, q, c) terminal form
            R = np.zeros((0, 0))
        R = np.asarray(R, dtype=np.float64)
        m = R.shape[0]
        self.Q = _mat(Q, (n, n))
        self.R = _mat(R, (m, m)) if m else np.zeros((0, 0))
        self.H = np.zeros((m, n)) if H is None else _mat(H, (m, n))
        self.q = np.zeros(n) if q is None else np.asarray(q, dtype=np.float64).reshape(n).copy()
        self.r = np.zeros(m) if r is None else np.asarray(r, dtype=np.float64).reshape(m).copy()
        self.c = float(c)
        if m and not _isposdef(self.R) and not getattr(self, "_padded", False):
            import warnings

            warnings.warn("R is not positive definite")
        if not _ispossemidef(self.Q):
            raise ValueError("Q must be positive semi-definite")

    def sizes(self):
        return self.Q.shape[0], self.R.shape[0]

    # reference formulas (src/cost.jl:171-198), host side for the KAT tests only
    def stage_cost(self, x, u=None, dt=None):
        x = np.asarray(x, dtype=np.float64)
        if u is None:
            return 0.5 * x @ self.Q @ x + self.q @ x + self.c
        u = np.asarray(u, dtype=np.float64)
        J = 0.5 * x @ self.Q @ x + 0.5 * u @ self.R @ u + self.q @ x + self.r @ u + self.c + u @ self.H @ x
        return J * (1.0 if dt is None else dt)

    def copy(self):
        return _copy.deepcopy(self)


def _isposdef(A):
    try:
        np.linalg.cholesky(0.5 * (A + A.T))
        return np.allclose(A, A.T)
    except np.linalg.LinAlgError:
        return False


def _ispossemidef(A):
    return bool(np.all(np.linalg.eigvalsh(0.5 * (A + A.T)) >= -1e-12 * max(1.0, np.abs(A).max())))


def LQRCost(Q, R, xf) -> QuadraticCost:
    """``LQRCost(Q, R, xf)`` (src/cost.jl:151-157)."""
    Q = np.asarray(Q, dtype=np.float64)
    xf = np.asarray(xf, dtype=np.float64)
    R = np.asarray(R, dtype=np.float64)
    return QuadraticCost(Q, R, np.zeros((R.shape[0], Q.shape[0])), -Q @ xf, np.zeros(R.shape[0]), 0.5 * xf @ Q @ xf)


def LQRCostTerminal(Qf, xf) -> QuadraticCost:
    """``LQRCostTerminal(Qf, xf)`` (src/cost.jl:165-169)."""
    Qf = np.asarray(Qf, dtype=np.float64)
    xf = np.asarray(xf, dtype=np.float64)
    return QuadraticCost(Qf, None, None, -Qf @ xf, None, 0.5 * xf @ Qf @ xf)


class GenericCost:
    """``GenericCost(ℓ, ℓf, n, m)`` / ``GenericCost(ℓ, ℓf, grad, hess, n, m)`` (src/cost.jl:239-287) from a
    compiled cost plugin (``tog_generic_cost_load``, csrc/tog_cost_plugin.hpp). ``stage_cost`` and
    ``cost_expansion`` (src/cost.jl:324-345) run on the device: the plugin's kernel evaluates ℓ with
    ForwardDiff's gradient and Hessian (auto_expansion_function, src/cost.jl:289-322), or the user's
    analytic expansion. Points are batched: x (n,) or (count, n), u (m,) or (count, m). As in the
    reference, a GenericCost is not a solver cost (its stage_cost has no dt method, src/cost.jl:324)."""

    _cache: dict = {}

    def __init__(self, path, device: int = 0):
        import ctypes as C

        path = str(pathlib.Path(path).resolve())
        lib = abi.load_library()
        if path not in GenericCost._cache:  # a plugin stays loaded for the life of the process
            h = C.c_void_p()
            abi.check(lib, lib.tog_generic_cost_load(path.encode(), C.byref(h)))
            n, m = C.c_int32(), C.c_int32()
            abi.check(lib, lib.tog_generic_cost_dims(h, C.byref(n), C.byref(m)))
            GenericCost._cache[path] = (h.value, n.value, m.value)
        self.ptr, self.n, self.m = GenericCost._cache[path]
        self.path, self.device = path, int(device)

    def sizes(self):
        return self.n, self.m

    def expand(self, X, U=None):
        """Batched ℓ and expansion: returns (J (count,), Expansion with leading dim count). With U None
        the terminal cost ℓf and its (xx, x) expansion; u, uu, ux are then empty."""
        import ctypes as C

        from .solvers import Expansion

        lib = abi.load_library()
        n, m = self.n, self.m
        X = np.ascontiguousarray(np.atleast_2d(np.asarray(X, dtype=np.float64)))
        if X.shape[1] != n:
            raise ValueError(f"x has {X.shape[1]} entries, the cost has n = {n}")
        cnt = X.shape[0]
        term = U is None
        J = np.zeros(cnt)
        Ex = np.zeros((cnt, n))
        Exx = np.zeros((cnt, n, n))  # stored column-major per point: Exx[p].T is the matrix
        if term:
            Eu, Euu, Eux = np.zeros((cnt, 0)), np.zeros((cnt, 0, 0)), np.zeros((cnt, n, 0))
            nul = C.cast(None, C.POINTER(C.c_double))
            abi.check(lib, lib.tog_generic_cost_expand(self.ptr, self.device, 1, abi.as_dp(X), nul, cnt, abi.as_dp(J),
                                                       abi.as_dp(Ex), nul, abi.as_dp(Exx), nul, nul))
        else:
            U = np.ascontiguousarray(np.atleast_2d(np.asarray(U, dtype=np.float64)))
            if U.shape != (cnt, m):
                raise ValueError(f"u must have shape ({cnt}, {m})")
            Eu, Euu, Eux = np.zeros((cnt, m)), np.zeros((cnt, m, m)), np.zeros((cnt, n, m))
            abi.check(lib, lib.tog_generic_cost_expand(self.ptr, self.device, 0, abi.as_dp(X), abi.as_dp(U), cnt,
                                                       abi.as_dp(J), abi.as_dp(Ex), abi.as_dp(Eu), abi.as_dp(Exx),
                                                       abi.as_dp(Euu), abi.as_dp(Eux)))
        t = lambda a: np.ascontiguousarray(a.swapaxes(-1, -2))  # column-major per point -> row-major
        return J, Expansion(Ex, Eu, t(Exx), t(Euu), t(Eux))

    def stage_cost(self, x, u=None):
        """``stage_cost(cost, x, u)`` / ``stage_cost(cost, xN)`` (src/cost.jl:324-325)."""
        J, _ = self.expand(x, u)
        return float(J[0]) if np.ndim(x) == 1 else J

    def cost_expansion(self, E, x, u=None):
        """``cost_expansion!(E, cost, x, u)`` / ``cost_expansion!(S, cost, xN)`` (src/cost.jl:327-345):
        fills E.x, E.u, E.xx, E.uu, E.ux (E.xx, E.x for the terminal form) in place."""
        _, e = self.expand(x, u)
        single = np.ndim(x) == 1
        fields = ("x", "xx") if u is None else ("x", "u", "xx", "uu", "ux")
        for f in fields:
            v = getattr(e, f)
            getattr(E, f)[...] = v[0] if single else v
        return None

    def copy(self):
        """``copy(cost::GenericCost)`` (src/cost.jl:347)."""
        return GenericCost(self.path, self.device)


_COST_TEMPLATE = """// generated by generic_cost() (problem.py): GenericCost(ℓ, ℓf, n, m) as a libtog cost plugin
#include "{hdr}"

struct {name} {{
  static constexpr int n = {n}, m = {m};
  template <class T>
  __host__ __device__ __forceinline__ static T stage(const T* x, const T* u) {{
    using namespace tog;
{stage}
  }}
  template <class T>
  __host__ __device__ __forceinline__ static T terminal(const T* x) {{
    using namespace tog;
{term}
  }}
}};

TOG_COST_PLUGIN({name})
"""


def generic_cost(stage_body: str, terminal_body: str, n: int, m: int, name: str = "UserCost", build_dir=None,
                 device: int = 0) -> GenericCost:
    """``GenericCost(ℓ, ℓf, n, m)`` (src/cost.jl:279-287) from C++ source: ``stage_body`` is the body of
    ``T stage(const T* x, const T* u)`` and ``terminal_body`` of ``T terminal(const T* x)`` over the scalar
    type T (double, or the second-order dual numbers of the expansion kernel). Compiled once with hipcc
    for gfx950 (cached by the hash of its source under ``csrc/plugins/``)."""
    import hashlib
    import subprocess

    csrc = pathlib.Path(__file__).resolve().parent / "csrc"
    out_dir = pathlib.Path(build_dir) if build_dir else csrc / "plugins"
    out_dir.mkdir(parents=True, exist_ok=True)
    ind = lambda b: "\n".join("    " + ln for ln in b.strip().splitlines())
    src = _COST_TEMPLATE.format(hdr=str(csrc / "tog_cost_plugin.hpp"), name=name, n=int(n), m=int(m),
                                stage=ind(stage_body), term=ind(terminal_body))
    hh = abi.header_hash()  # the plugin is compiled against (and cached under) libtog's header text
    src = f"// libtog header hash {hh}\n" + src
    key = hashlib.sha1(src.encode()).hexdigest()[:12]
    so = out_dir / f"gen_{name}_{key}.so"
    if not so.exists():
        _prune_stale_plugins(out_dir, hh)
        hip = out_dir / f"gen_{name}_{key}.hip"
        hip.write_text(src)
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-fPIC",
               f"-DTOG_HEADER_HASH=0x{hh}LL", "-shared", "-o", str(so), str(hip)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            hip.unlink(missing_ok=True)  # no broken source left in the plugin directory
            raise ValueError(f"generic cost {name!r} does not compile:\n{r.stderr[-4000:]}")
    cost = GenericCost(so, device)
    if (cost.n, cost.m) != (int(n), int(m)):
        raise ValueError("plugin dimensions do not match")
    return cost


class Objective:
    """``Objective(costs)`` (src/objective.jl:15-29): one cost per knot, the last the terminal cost.
    Knots 1..N-1 may share one QuadraticCost (the form every config uses) or carry their own
    (a time-varying objective: ``stage_table`` goes to the device as tog_problem_desc.stage_costs,
    DevProblem::kc); ``stage`` is knot 1's cost."""

    def __init__(self, cost, cost_terminal=None, N=None):
        if isinstance(cost, list):
            costs = list(cost) + ([cost_terminal] if cost_terminal is not None else [])
        else:
            if N is None:
                raise ValueError("N required")
            term = cost if cost_terminal is None else cost_terminal
            costs = [cost] * (N - 1) + [term]
        self.cost = costs
        stage = costs[0]
        self.varying = any(c is not stage and not _same_cost(c, stage) for c in costs[:-1])
        if self.varying:
            sz = stage.sizes()
            if not all(isinstance(c, QuadraticCost) and c.sizes() == sz for c in costs[:-1]):
                raise ValueError("a time-varying objective's stage costs must be QuadraticCosts of one size")
        self.stage = stage
        self.terminal = costs[-1]

    def __len__(self):
        return len(self.cost)

    def __getitem__(self, k):
        return self.cost[k]

    def stage_table(self, m=None):
        """The (N-1, nc) per-knot rows [Q; R; H; q; r; c] (matrices column-major) of a time-varying
        objective, None when every stage knot shares one cost."""
        if not self.varying:
            return None
        rows = []
        for c in self.cost[:-1]:
            n = c.Q.shape[0]
            R = c.R if c.R.size else np.zeros((m, m))
            mm = R.shape[0]
            H = c.H if c.H.size else np.zeros((mm, n))
            r = c.r if c.r.size else np.zeros(mm)
            rows.append(np.concatenate([c.Q.ravel(order="F"), R.ravel(order="F"), H.ravel(order="F"), c.q, r,
                                        [c.c]]))
        return np.stack(rows)

    def map_stage(self, f):
        """A new Objective with f applied to each stage cost (knots sharing a cost keep sharing one)."""
        memo = {}
        out = []
        for c in self.cost[:-1]:
            if id(c) not in memo:
                memo[id(c)] = f(c)
            out.append(memo[id(c)])
        return out


def _same_cost(a, b):
    return all(np.array_equal(getattr(a, f), getattr(b, f)) for f in ("Q", "R", "H", "q", "r")) and a.c == b.c


def LQRObjective(Q, R, Qf, xf, N) -> Objective:
    """``LQRObjective(Q, R, Qf, xf, N)`` (src/objective.jl:102-114)."""
    Q = np.asarray(Q, dtype=np.float64)
    R = np.asarray(R, dtype=np.float64)
    Qf = np.asarray(Qf, dtype=np.float64)
    xf = np.asarray(xf, dtype=np.float64)
    ell = QuadraticCost(Q, R, np.zeros((R.shape[0], Q.shape[0])), -Q @ xf, np.zeros(R.shape[0]), 0.5 * xf @ Q @ xf)
    ellN = QuadraticCost(Qf, None, None, -Qf @ xf, None, 0.5 * xf @ Qf @ xf)
    return Objective([ell] * (N - 1) + [ellN])


# ----------------------------------------------------------------------------- constraints


class _Constraint:
    inequality = True
    label = "con"

    def __add__(self, other):
        return ConstraintSet([self]) + other

    def __radd__(self, other):
        return ConstraintSet(list(other)) + self


class BoundConstraint(_Constraint):
    """``BoundConstraint(n, m; x_min, x_max, u_min, u_max, trim=true)`` (src/constraints.jl:155-188).
    Constraint vector order ``[x_max; u_max; x_min; u_min]``; ``trim=true`` drops the infinite bounds,
    ``trim=false`` keeps every row (an infinite bound then evaluates to -Inf and the AL terms to NaN, as
    in the reference). At the terminal knot the untrimmed rows are x_max and x_min (the reference's
    untrimmed ``x_all`` mask, ``[trues(n); falses(m); trues(m); falses(m)]``, has the wrong length unless
    n == m; its evident intent is taken)."""

    label = "bound"

    def __init__(self, n, m, x_min=-math.inf, x_max=math.inf, u_min=-math.inf, u_max=math.inf, trim=True):
        self.n, self.m = n, m
        self.u_max, self.u_min = _validate_bounds(u_max, u_min, m)
        self.x_max, self.x_min = _validate_bounds(x_max, x_min, n)
        self.trim = bool(trim)
        if self.trim:
            self.active = dict(x_max=np.isfinite(self.x_max), u_max=np.isfinite(self.u_max),
                               x_min=np.isfinite(self.x_min), u_min=np.isfinite(self.u_min))
        else:
            self.active = dict(x_max=np.ones(n, bool), u_max=np.ones(m, bool), x_min=np.ones(n, bool),
                               u_min=np.ones(m, bool))

    def length(self, kind="stage"):
        a = self.active
        if kind == "stage":
            return int(sum(v.sum() for v in a.values()))
        return int(a["x_max"].sum() + a["x_min"].sum())

    def evaluate(self, x, u=None):  # src/constraints.jl:212-227
        a = self.active
        x = np.asarray(x, dtype=np.float64)
        if u is None:
            return np.concatenate([(x - self.x_max)[a["x_max"]], (self.x_min - x)[a["x_min"]]])
        u = np.asarray(u, dtype=np.float64)[: self.m]  # u[con.inds[2]] (constraint_sets.jl:106-110)
        return np.concatenate([(x - self.x_max)[a["x_max"]], (u - self.u_max)[a["u_max"]],
                               (self.x_min - x)[a["x_min"]], (self.u_min - u)[a["u_min"]]])

    def jacobian(self, x, u=None):  # src/constraints.jl:229-237
        n, m = self.n, self.m
        jac = np.vstack([np.eye(n + m), -np.eye(n + m)])
        a = self.active
        if u is None:
            sel = np.concatenate([a["x_max"], np.zeros(m, bool), a["x_min"], np.zeros(m, bool)])
            return jac[sel][:, :n]
        sel = np.concatenate([a["x_max"], a["u_max"], a["x_min"], a["u_min"]])
        return jac[sel]

    def to_abi(self, m=None):
        # an infeasible problem's controls are [u; slack]: the bound keeps the model's m
        # (update_constraint_set_jacobians, constraint_sets.jl:135-150), so the rows are those of the model
        # controls, trimmed or not (the device's build_rows and the oracle's con_init skip the slack entries)
        pad = np.full(0 if m is None else m - self.m, np.inf)
        data = np.concatenate([self.x_max, self.x_min, self.u_max, pad, self.u_min, -pad])
        return (abi.CON_BOUND, 0 if self.trim else 1, data)


class InfeasibleConstraint(_Constraint):
    """``infeasible_constraints(n, m)`` (src/constraints.jl:306-314): Constraint{Equality} on the
    slack controls, c = u[m+1:m+n], ∇c = [0 0 I]. Stage only."""

    inequality = False
    label = "infeasible"

    def __init__(self, n, m):
        self.n, self.m = n, m

    def length(self, kind="stage"):
        return self.n if kind == "stage" else 0

    def evaluate(self, x, u=None):
        if u is None:
            return np.zeros(0)
        return np.asarray(u, dtype=np.float64)[self.m: self.m + self.n].copy()

    def jacobian(self, x, u=None):
        J = np.zeros((self.n, 2 * self.n + self.m))
        J[:, self.n + self.m:] = np.eye(self.n)
        return J

    def to_abi(self, m=None):
        return (abi.CON_INFEASIBLE, 0, np.zeros(1))


def infeasible_constraints(n, m):
    return InfeasibleConstraint(n, m)


def _validate_bounds(mx, mn, n):  # src/constraints.jl:276-296
    if np.isscalar(mn):
        mn = np.ones(n) * mn
    if np.isscalar(mx):
        mx = np.ones(n) * mx
    mx = np.asarray(mx, dtype=np.float64).copy()
    mn = np.asarray(mn, dtype=np.float64).copy()
    if len(mx) != len(mn):
        raise ValueError("u_max and u_min must have equal length")
    if not np.all(mx >= mn):
        raise ValueError("u_max must be greater than u_min")
    if len(mx) != n:
        raise ValueError(f"limit of length {len(mx)} doesn't match expected length of {n}")
    return mx, mn


class GoalConstraint(_Constraint):
    """``goal_constraint(xf)`` (src/constraints.jl:299-304): terminal equality x_N - xf."""

    inequality = False
    label = "goal"

    def __init__(self, xf):
        self.xf = np.asarray(xf, dtype=np.float64).copy()

    def length(self, kind="stage"):
        return 0 if kind == "stage" else len(self.xf)

    def evaluate(self, x, u=None):
        return np.asarray(x, dtype=np.float64) - self.xf if u is None else np.zeros(0)

    def to_abi(self):
        return (abi.CON_GOAL, len(self.xf), self.xf)  # count: the goal rows x[1:count] - xf (inds, constraints.jl:303)


def goal_constraint(xf):
    return GoalConstraint(xf)


class UserConstraint(_Constraint):
    """``Constraint{Inequality|Equality}(c!, n, m, p, label)`` with a user function
    (src/constraints.jl:85-89; Jacobian by ForwardDiff, src/model.jl:460-489). The function is
    the user model plugin's ``con(fid, c, x, u)`` (csrc/tog_plugin.hpp): it runs on the device,
    its Jacobian over [x; u] by dual numbers. ``where``: "stage" (knots 1..N-1), "terminal" (knot
    N, u = 0) or "both". ``host`` (optional): a numpy restatement ``f(x, u) -> c`` used only by
    the host-side ``max_violation(prob)``."""

    _WHERE = {"stage": 0, "terminal": 1, "both": 2}

    def __init__(self, n, m, p, fid=0, equality=False, where="stage", label="user", host=None):
        if not 1 <= p <= 16:
            raise ValueError("user constraint: 1 <= p <= 16 outputs")
        if where not in self._WHERE:
            raise ValueError(f"where must be one of {sorted(self._WHERE)}")
        self.n, self.m, self.p, self.fid = n, m, int(p), int(fid)
        self.inequality = not equality
        self.where, self.label, self.host = where, label, host

    def length(self, kind="stage"):
        if kind == "stage":
            return self.p if self.where in ("stage", "both") else 0
        return self.p if self.where in ("terminal", "both") else 0

    def evaluate(self, x, u=None):
        kind = "stage" if u is not None else "terminal"
        if self.length(kind) == 0:
            return np.zeros(0)
        if self.host is None:
            return np.full(self.p, np.nan)
        return np.asarray(self.host(np.asarray(x), np.zeros(self.m) if u is None else np.asarray(u)),
                          dtype=np.float64)

    def to_abi(self):
        return (abi.CON_USER, self.p, np.array([self.fid, 0.0 if self.inequality else 1.0,
                                                 self._WHERE[self.where]], dtype=np.float64))


def circle_constraint(x, x0, y0=None, r=None):
    """``circle_constraint(x, x0, y0, r)`` / ``(x, c, r)`` (src/utils.jl:140-144); c <= 0 is feasible."""
    if r is None:
        c, r = x0, y0
        x0, y0 = c[0], c[1]
    return -((x[0] - x0) ** 2 + (x[1] - y0) ** 2 - r ** 2)


def sphere_constraint(x, x0, y0, z0=None, r=None):
    """``sphere_constraint`` (src/utils.jl:150-156)."""
    if z0 is None:  # (x, c, r)
        c, r = x0, y0
        x0, y0, z0 = c[0], c[1], c[2]
    return -((x[0] - x0) ** 2 + (x[1] - y0) ** 2 + (x[2] - z0) ** 2 - r ** 2)


class CircleConstraints(_Constraint):
    """A ``Constraint{Inequality}`` whose rows are ``circle_constraint(x, xc, yc, r)`` — the
    reference's cylinder-obstacle idiom (problems/quad_obs.jl:53-62). Stage only."""

    label = "circles"

    def __init__(self, n, m, circles, label="circles"):
        self.circles = np.asarray(circles, dtype=np.float64).reshape(-1, 3)
        self.label = label

    def length(self, kind="stage"):
        return len(self.circles) if kind == "stage" else 0

    def evaluate(self, x, u=None):
        if u is None:
            return np.zeros(0)
        return np.array([circle_constraint(x, c[0], c[1], c[2]) for c in self.circles])

    def to_abi(self):
        return (abi.CON_CIRCLES, len(self.circles), self.circles.ravel())


class SphereConstraints(_Constraint):
    """Rows ``sphere_constraint(x, xc, yc, zc, r)`` (test/quadrotor_tests.jl:68-74,
    problems/quad_obs.jl:64-69). Stage only."""

    label = "spheres"

    def __init__(self, n, m, spheres, label="spheres"):
        self.spheres = np.asarray(spheres, dtype=np.float64).reshape(-1, 4)
        self.label = label

    def length(self, kind="stage"):
        return len(self.spheres) if kind == "stage" else 0

    def evaluate(self, x, u=None):
        if u is None:
            return np.zeros(0)
        return np.array([sphere_constraint(x, s[0], s[1], s[2], s[3]) for s in self.spheres])

    def to_abi(self):
        return (abi.CON_SPHERES, len(self.spheres), self.spheres.ravel())


class ConstraintSet(list):
    """``ConstraintSet`` (src/constraint_sets.jl:1): an ordered list of constraints."""

    def __add__(self, other):
        out = ConstraintSet(self)
        if isinstance(other, (list, tuple)):
            out.extend(other)
        else:
            out.append(other)
        return out

    __iadd__ = __add__

    def num_constraints(self, kind="stage"):
        return sum(c.length(kind) for c in self)


class Constraints:
    """``Constraints`` per-knot constraint sets (src/constraint_sets.jl:157-206)."""

    def __init__(self, C=None, N=None, C_term=None):
        if isinstance(C, int) and N is None:  # Constraints(N)
            N, C = C, None
        if N is None:
            raise ValueError("N required")
        if C is None:
            self.C = [ConstraintSet() for _ in range(N)]
        elif C_term is None:
            self.C = [ConstraintSet(C) for _ in range(N)]
        else:
            self.C = [ConstraintSet(C) for _ in range(N - 1)] + [ConstraintSet(C_term)]

    def __len__(self):
        return len(self.C)

    def __getitem__(self, k):
        return self.C[k]

    def __setitem__(self, k, v):
        self.C[k] = v if isinstance(v, ConstraintSet) else ConstraintSet(v if isinstance(v, list) else [v])

    def is_constrained(self):
        return any(len(c) > 0 for c in self.C)

    def num_constraints(self):
        N = len(self.C)
        return [c.num_constraints("stage" if k < N - 1 else "terminal") for k, c in enumerate(self.C)]

    def copy(self):
        return Constraints([], N=len(self.C)) if not self.C else _copy_constraints(self)


def _copy_constraints(cons):
    out = Constraints(len(cons.C))
    out.C = [ConstraintSet(c) for c in cons.C]
    return out


# ----------------------------------------------------------------------------- problem


class Problem:
    """``Problem{T,Discrete}`` (src/problem.jl:37-113).

    ``x0`` may be a vector (one trajectory) or an array ``(B, n)``; ``U0`` a list of N-1
    control vectors, an array ``(N-1, m)`` or a batch ``(B, N-1, m)``. ``X`` starts as NaN
    (``empty_state``, src/problem.jl:232), which makes the solvers roll out first.
    """

    def __init__(self, model: Model, obj: Objective, U0=None, X0=None, *, constraints: Constraints | None = None,
                 x0=None, xf=None, N=None, dt=None, tf=None, integration=None):
        if not model.discrete:
            if integration is None:
                raise ValueError("a continuous model needs integration=:rk3/:rk4 (DIRCOL is out of scope)")
            model = discretize_model(model, integration)
        N = len(obj) if N is None else N
        if len(obj) != N:
            raise ValueError("objective length must equal N")
        N, tf, dt = _validate_time(N, tf, dt)
        self.model = model
        self.obj = obj
        self.constraints = constraints if constraints is not None else Constraints(N)
        if len(self.constraints) != N:
            raise ValueError("constraints length must equal N")
        n, m = model.n, model.m
        x0 = np.zeros(n) if x0 is None else np.asarray(x0, dtype=np.float64)
        self.batched = x0.ndim == 2
        B = x0.shape[0] if self.batched else 1
        self.x0 = x0.reshape(B, n).copy()
        self.xf = np.zeros(n) if xf is None else np.asarray(xf, dtype=np.float64).copy()
        self.N, self.dt, self.tf = N, dt, tf
        self._X = np.full((B, N, n), np.nan)
        self._U = np.zeros((B, N - 1, m))
        if U0 is not None:
            initial_controls_b(self, U0)
        if X0 is not None:
            initial_states_b(self, X0)

    # ---- shapes
    @property
    def B(self):
        return self._X.shape[0]

    def size(self):
        return self.model.n, self.model.m, self.N

    @property
    def X(self):
        return self._X if self.batched else self._X[0]

    @X.setter
    def X(self, v):
        self._X[...] = np.asarray(v, dtype=np.float64).reshape(self._X.shape)

    @property
    def U(self):
        return self._U if self.batched else self._U[0]

    @U.setter
    def U(self, v):
        self._U[...] = np.asarray(v, dtype=np.float64).reshape(self._U.shape)

    def copy(self):
        p = _copy.copy(self)
        p.constraints = _copy_constraints(self.constraints)
        p.x0 = self.x0.copy()
        p.xf = self.xf.copy()
        p._X = self._X.copy()
        p._U = self._U.copy()
        return p

    def is_constrained(self):
        return self.constraints.is_constrained()

    # ---- marshalling to the C ABI
    def build_desc(self, tf_min: bool = False) -> abi.DescBuilder:
        """The C ABI's tog_problem_desc. ``tf_min``: mark a tf = 0 problem TOG_PROB_TF_MIN (the original
        problem handed to tog_solve_altro, which builds minimum_time_problem itself)."""
        n, m, N = self.model.n, self.model.m, self.N
        stage, term = self.obj.stage, self.obj.terminal
        sets, knot_set, keys = [], [], {}
        for k in range(N):
            cs = self.constraints[k]
            if len(cs) == 0:
                knot_set.append(-1)
                continue
            key = tuple(id(c) for c in cs) + (k == N - 1,)
            if key not in keys:
                keys[key] = len(sets)
                sets.append([c.to_abi(m) if isinstance(c, (BoundConstraint, InfeasibleConstraint)) else c.to_abi()
                             for c in cs])
            knot_set.append(keys[key])
        R = stage.R if stage.R.size else np.zeros((m, m))
        flags = (abi.PROB_INFEASIBLE if self.model.slack else 0) | (abi.PROB_MIN_TIME if self.model.min_time else 0)
        if tf_min and not self.model.min_time:
            flags |= abi.PROB_TF_MIN
        return abi.DescBuilder(self.model.model_id, self.model.integration, n, m, N, self.dt, stage.Q, R, stage.H,
                               stage.q, stage.r, stage.c, term.Q, term.q, term.c, sets, knot_set, batch=self.B,
                               flags=flags, user_model=self.model.plugin.ptr if self.model.plugin else None,
                               R_min_time=getattr(self, "R_min_time", 0.0), stage_costs=self.obj.stage_table(m))


def _validate_time(N, tf, dt):
    """``_validate_time`` (src/problem.jl:169-220) for the fixed-time case."""
    if N is None and dt is None and tf is None:
        raise ValueError("Must specify at least 2: N, dt, or tf")
    if isinstance(tf, str) and tf.lstrip(":") == "min":
        tf = 0.0
    if tf == 0:  # minimum time (src/problem.jl:174-178): dt is the initial time step guess
        if dt is None or not dt > 0:
            raise ValueError("a minimum-time problem needs the initial dt")
        if N is None:
            raise ValueError("a minimum-time problem needs N")
        return N, 0.0, dt
    if tf is not None:
        if dt is None and N is not None:
            dt = tf / (N - 1)
        elif dt is not None and N is None:
            N = int(round(tf / dt)) + 1
            dt = tf / (N - 1)
        elif dt is not None and N is not None and dt != tf / (N - 1):
            raise ValueError("Specified time step, number of knot points, and final time do not agree")
    else:
        if dt is None or not dt > 0:
            raise ValueError("dt must be positive for a non-minimum-time problem")
        if N is None:
            N = 51
        tf = dt * (N - 1)
    if N < 0:
        raise ValueError(f"{N} is not a valid entry for N")
    if not dt > 0:
        raise ValueError("dt must be strictly positive")
    return N, tf, dt


def initial_controls_b(prob: Problem, U0):
    """``initial_controls!(prob, U0)`` (src/problem.jl:149-150)."""
    U0 = np.asarray(U0, dtype=np.float64)
    N, m = prob.N, prob.model.m
    if U0.ndim == 2:
        U0 = U0[: N - 1]
        prob._U[...] = U0[None, :, :]
    else:
        prob._U[...] = U0[:, : N - 1, :]


def initial_states_b(prob: Problem, X0):
    """``initial_states!(prob, X0)`` (src/problem.jl:153-154)."""
    X0 = np.asarray(X0, dtype=np.float64)
    prob._X[...] = X0 if X0.ndim == 3 else X0[None]


def set_x0_b(prob: Problem, x0):
    prob.x0[...] = np.asarray(x0, dtype=np.float64)


def max_violation(prob: Problem) -> float:
    """``max_violation(prob)`` (src/problem.jl:242-267), host side, per trajectory max over
    the batch (returns an array for a batched problem)."""
    out = []
    N = prob.N
    for b in range(prob.B):
        c_max = 0.0
        if prob.is_constrained():
            X, U = prob._X[b], prob._U[b]
            for k in range(N):
                cs = prob.constraints[k]
                term = k == N - 1
                vals_e, vals = [], []
                for c in cs:
                    v = c.evaluate(X[k]) if term else c.evaluate(X[k], U[k])
                    if len(v) == 0:
                        continue
                    vals.append(v)
                    if not c.inequality:
                        vals_e.append(v)
                if not vals:
                    continue
                allc = np.concatenate(vals)
                max_e = np.max(np.abs(np.concatenate(vals_e))) if vals_e else 0.0
                max_i = np.max(np.maximum(allc, 0.0))
                c_max = max(c_max, max(max_e, max_i))
        out.append(c_max)
    return out[0] if not prob.batched else np.array(out)


# ----------------------------------------------------------------------------- infeasible start


def infeasible_problem(prob: Problem, R_inf: float = 1.0) -> Problem:
    """``infeasible_problem(prob, R_inf)`` (src/solvers/altro/infeasible.jl:2-33).

    Slack controls u_inf (n per knot) make any state trajectory dynamically feasible:
    the model becomes ``add_slack_controls`` (x+ = f_d(x,u) + u_inf), the stage cost gets
    ``R_inf*I/dt`` on u_inf (zero-padded r and H), and every stage constraint set becomes
    ``update_constraint_set_jacobians`` order — non-bound constraints first, then the bounds
    (constraint_sets.jl:135-150) — followed by ``infeasible_constraints`` (u_inf = 0).
    The terminal set is kept. The state trajectory X is kept; the slack controls are filled on
    the device by ``slack_controls`` (infeasible.jl:63-80) when the solver is set up.
    """
    n, m, N = prob.model.n, prob.model.m, prob.N
    term = prob.obj.terminal

    def cost_inf(stage):
        R = np.zeros((m + n, m + n))
        R[:m, :m] = stage.R
        R[m:, m:] = R_inf * np.eye(n) / prob.dt
        H = np.vstack([stage.H, np.zeros((n, n))])
        r = np.concatenate([stage.r, np.zeros(n)])
        return QuadraticCost(stage.Q, R, H, stage.q, r, stage.c)

    obj = Objective(prob.obj.map_stage(cost_inf), term.copy())
    con_inf = infeasible_constraints(n, m)
    cons = Constraints(N)
    constrained = prob.is_constrained()
    memo = {}
    for k in range(N - 1):
        cs = prob.constraints[k]
        key = tuple(id(c) for c in cs)
        if key not in memo:  # knots sharing a set keep sharing one (same rows, one device copy)
            others = [c for c in cs if not isinstance(c, BoundConstraint)] if constrained else []
            bnds = [c for c in cs if isinstance(c, BoundConstraint)] if constrained else []
            memo[key] = ConstraintSet(others + bnds + [con_inf])
        cons.C[k] = memo[key]
    cons.C[N - 1] = ConstraintSet(prob.constraints[N - 1]) if constrained else ConstraintSet()
    p = Problem(add_slack_controls(prob.model), obj, constraints=cons, x0=prob.x0 if prob.batched else prob.x0[0],
                xf=prob.xf, N=N, dt=prob.dt)
    p._U[:, :, :m] = prob._U
    p._U[:, :, m:] = 0.0
    p._X[...] = prob._X
    return p


# ----------------------------------------------------------------------------- minimum time


def add_min_time_controls(model: Model) -> Model:
    """``add_min_time_controls(model)`` (src/solvers/altro/minimum_time.jl:83-104): state [x; τ],
    control [u; h], x+ = f_d(x, u, h²), τ+ = h (the device's MinTime<M>)."""
    if not model.discrete:
        raise ValueError("add_min_time_controls needs a discrete model")
    if model.min_time:
        raise ValueError("model already has a time-step control")
    # (user plugin models too: each plugin instantiates MinTime<M>, csrc/tog_plugin.hpp). An infeasible-start
    # model (altro_problem's infeasible + minimum-time case, altro_methods.jl:98-124) keeps its slacks:
    # u = [u; s; h], the device's MinTime<Infeasible<M>>
    if model.slack and model.plugin is not None:
        raise NotImplementedError("minimum time of an infeasible-start user plugin model is not built")
    return Model(model.model_id, model.n + 1, model.m + 1, model.name + "_mt", model.integration, model.slack,
                 plugin=model.plugin, min_time=True)


class MinTimeEquality(_Constraint):
    """``mintime_equality(n, m)`` (minimum_time.jl:106-124): h_k - τ_k = 0 (τ_k is h_{k-1})."""

    inequality = False
    label = "min_time_eq"

    def length(self, kind="stage"):
        return 1 if kind == "stage" else 0

    def evaluate(self, x, u=None):
        return np.zeros(0) if u is None else np.array([u[-1] - x[-1]])

    def to_abi(self):
        return (abi.CON_MIN_TIME_EQ, 1, np.zeros(1))


def mintime_constraints(prob: Problem, dt_max: float = 1.0, dt_min: float = 1.0e-3) -> Constraints:
    """``mintime_constraints(prob, dt_max, dt_min)`` (minimum_time.jl:125-141): at every knot the
    bounds are removed, combined with √dt_min <= h <= √dt_max (``combine``, constraints.jl:195-203; τ
    unbounded) and appended after the other constraints (``update_constraint_set_jacobians``), then
    h_k = τ_k at the knots 1 < k < N."""
    n, m, N = prob.model.n, prob.model.m, prob.N
    cons = Constraints(N)
    eq = MinTimeEquality()
    memo = {}
    for k in range(N):
        cs = prob.constraints[k]
        key = (tuple(id(c) for c in cs), k == 0, k == N - 1)
        if key not in memo:
            others = [c for c in cs if not isinstance(c, BoundConstraint)]
            bnds = [c for c in cs if isinstance(c, BoundConstraint)]
            b = bnds[0] if bnds else BoundConstraint(n, m)
            # combine(bnd, mt_bnd) (constraints.jl:195-203) sizes the result by the bound's own (n, m): an
            # infeasible problem's bound keeps the model's m, so its √dt bounds land on u[m+1], the first
            # slack control, and h stays unbounded (the reference's behaviour, reproduced as written)
            bnd2 = BoundConstraint(n + 1, len(b.u_max) + 1, x_min=np.append(b.x_min, -math.inf),
                                   x_max=np.append(b.x_max, math.inf), u_min=np.append(b.u_min, math.sqrt(dt_min)),
                                   u_max=np.append(b.u_max, math.sqrt(dt_max)))
            memo[key] = ConstraintSet(others + [bnd2] + ([eq] if 0 < k < N - 1 else []))
        cons.C[k] = memo[key]
    return cons


def minimum_time_problem(prob: Problem, R_min_time: float = 1.0, dt_max: float = 1.0, dt_min: float = 1.0e-3) -> Problem:
    """``minimum_time_problem(prob, R_min_time, dt_max, dt_min)`` (minimum_time.jl:2-34): the model
    ``add_min_time_controls``, the objective MinTimeCost (the quadratic costs zero-padded to the
    augmented sizes plus R_min_time h², on the device), ``mintime_constraints``,
    U = [U; √dt], X = [X; √dt], x0 = [x0; 0]."""
    n, m, N = prob.model.n, prob.model.m, prob.N
    term = prob.obj.terminal

    def pad(A, r, c):
        out = np.zeros((r, c))
        A = np.asarray(A, dtype=np.float64)
        if A.size:
            out[:A.shape[0], :A.shape[1]] = A
        return out

    def cost_mt(stage):
        R = stage.R if stage.R.size else np.zeros((m, m))
        st = QuadraticCost.__new__(QuadraticCost)
        st._padded = True  # MinTimeCost's base cost on [x; τ], [u; h]: R is singular by construction
        st.__init__(pad(stage.Q, n + 1, n + 1), pad(R, m + 1, m + 1), pad(stage.H, m + 1, n + 1),
                    np.append(stage.q, 0.0), np.append(stage.r if stage.r.size else np.zeros(m), 0.0), stage.c)
        return st

    tm = QuadraticCost(pad(term.Q, n + 1, n + 1), None, None, np.append(term.q, 0.0), None, term.c)
    obj = Objective(prob.obj.map_stage(cost_mt), tm)
    x0 = np.hstack([prob.x0, np.zeros((prob.B, 1))])
    p = Problem(add_min_time_controls(prob.model), obj, constraints=mintime_constraints(prob, dt_max, dt_min),
                x0=x0 if prob.batched else x0[0], xf=np.append(prob.xf, 0.0), N=N, dt=prob.dt)
    p.tf = 0.0
    p.R_min_time = float(R_min_time)
    p._U[:, :, :m] = prob._U
    p._U[:, :, m] = math.sqrt(prob.dt)
    p._X[:, :, :n] = prob._X
    p._X[:, :, n] = math.sqrt(prob.dt)
    return p


def total_time(prob: Problem):
    """``total_time(prob)`` (minimum_time.jl:64-73): Σ h_k² for a minimum-time problem (its h comes
    back from the solve in ``prob.h``), else dt (N - 1)."""
    if prob.tf == 0.0:
        tt = np.sum(np.asarray(prob.h) ** 2, axis=-1)
        return tt if prob.batched else float(tt[0])
    return prob.dt * (prob.N - 1)


def line_trajectory(x0, xf, N):
    """``line_trajectory(x0, xf, N)`` (src/solvers/altro/infeasible.jl:82-90): (N, n) with
    x_k = (xf - x0)/N * t_k, t = range(0, N, length=N), first/last rows pinned to x0/xf."""
    x0 = np.asarray(x0, dtype=np.float64)
    xf = np.asarray(xf, dtype=np.float64)
    t = np.linspace(0.0, N, N)
    slope = (xf - x0) / N
    X = np.array([slope * t[k] for k in range(N)])
    X[0] = x0
    X[-1] = xf
    return X
