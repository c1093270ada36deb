"""MI355X-native batched iLQR / AL-iLQR hot path of TrajectoryOptimization.jl.

Public surface mirrors the reference's exports (src/TrajectoryOptimization.jl:29-125) for the
hot path: models + ``rk3``/``rk4``, costs/objectives, bound/goal/obstacle constraints,
``Problem``, the solver option structs and ``solve_b`` (= ``solve!``) / ``solve``, plus the
step-level entry points (``rollout_b``, ``jacobian_b``, ``backwardpass_b``, ``forwardpass_b``,
``cost``). Compute runs in ``csrc/libtog.so`` (hand-written HIP for gfx950) through the C ABI in
``include/tog.h``.

The directory name is not a Python identifier; ``__graft_entry__.load_package()`` imports it
under the alias ``trajopt_amd``.
"""
from . import abi
from .problem import (BoundConstraint, CircleConstraints, Constraints, ConstraintSet, Dynamics, GoalConstraint,
                      LQRCost, LQRCostTerminal, LQRObjective, Model, Objective, Problem, QuadraticCost,
                      SphereConstraints, circle_constraint, discretize_model, goal_constraint, initial_controls_b,
                      initial_states_b, max_violation, midpoint, midpoint_implicit, rk3, rk3_implicit, rk4, set_x0_b, sphere_constraint, add_slack_controls,
                      InfeasibleConstraint, infeasible_constraints, infeasible_problem, line_trajectory, user_model,
                      UserModelPlugin, UserConstraint, add_min_time_controls,
                      minimum_time_problem, mintime_constraints, total_time, MinTimeEquality, GenericCost, generic_cost)
from .solvers import (Expansion, AbstractSolver, AbstractSolverFor, ALTROSolver, ALTROSolverOptions, AugmentedLagrangianSolver,
                      AugmentedLagrangianSolverOptions, iLQRSolver, iLQRSolverOptions, ProjectedNewtonSolver,
                      ProjectedNewtonSolverOptions, PosDefException, ProjectedNewtonError, solve, solve_b, solver_name, to_tog_options,
                      to_tog_pn_options)
from .steps import backwardpass_b, cost, cost_expansion_b, forwardpass_b, jacobian_b, rollout_b, update_constraints_b
from . import problems as Problems
from . import distributed

__all__ = [
    "abi", "BoundConstraint", "CircleConstraints", "Constraints", "ConstraintSet", "Dynamics", "GoalConstraint",
    "LQRCost", "LQRCostTerminal", "LQRObjective", "Model", "Objective", "Problem", "QuadraticCost",
    "SphereConstraints", "circle_constraint", "discretize_model", "goal_constraint", "initial_controls_b",
    "initial_states_b", "max_violation", "midpoint", "midpoint_implicit", "rk3", "rk3_implicit", "rk4", "set_x0_b", "sphere_constraint", "AbstractSolver",
    "AbstractSolverFor", "ALTROSolver", "ALTROSolverOptions", "AugmentedLagrangianSolver",
    "AugmentedLagrangianSolverOptions", "iLQRSolver", "iLQRSolverOptions", "solve", "solve_b", "solver_name",
    "to_tog_options", "Expansion", "backwardpass_b", "cost", "cost_expansion_b", "update_constraints_b", "forwardpass_b", "jacobian_b", "rollout_b",
    "Problems", "add_slack_controls", "InfeasibleConstraint", "infeasible_constraints", "infeasible_problem",
    "line_trajectory", "ProjectedNewtonSolver", "ProjectedNewtonSolverOptions", "to_tog_pn_options",
    "GenericCost", "generic_cost", "PosDefException", "ProjectedNewtonError",
]
