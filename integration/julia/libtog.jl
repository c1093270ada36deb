# libtog.jl — TrajectoryOptimization.jl solver plugin over libtog's C ABI (include/tog.h).
#
# Drop-in for the reference's solver plugin contract (docs/src/solvers.md:25-47, src/solvers.jl:47-108):
#   BatchediLQRSolverOptions{T} <: AbstractSolverOptions{T}   (mutable, @with_kw defaults)
#   BatchediLQRSolver{T}        <: AbstractSolver{T}          (fields `opts`, `stats::Dict{Symbol,Any}`)
#   AbstractSolver(prob, opts), solve!(prob, solver), reset!, copy, size
# so the reference's generic `solve!(prob, opts)` (src/solvers.jl:91-94) and `solve(prob, opts)`
# (:104-108) dispatch to the HIP kernels with no other change. A Vector{<:Problem} of the same problem
# with different x0 / U0 is one batched solve (B trajectories on the GPU at once).
#
# Include it from src/TrajectoryOptimization.jl after `include("solvers.jl")` (it uses Problem, Model,
# Objective, QuadraticCost, BoundConstraint, Constraint, Dynamics, iLQRSolverOptions,
# AugmentedLagrangianSolverOptions and @with_kw from the module). UNTESTED: the build image has no
# Julia. tests/c/test_capi_config3.c fills tog_problem_desc for BASELINE config 3 exactly as
# tog_desc below does and is checked bit for bit against the Python path on the GPU.

using Parameters
using LinearAlgebra: PosDefException

const libtog = get(ENV, "TOG_LIB", "libtog.so")

# ------------------------------------------------------------------------ include/tog.h mirrors
const TOG_ABI_VERSION = Int32(4)    # include/tog.h; checked against tog_version() at first use
const TOG_OK = Int32(0)
const TOG_RK3, TOG_RK4, TOG_MIDPOINT, TOG_RK3_IMPLICIT, TOG_MIDPOINT_IMPLICIT = Int32.(0:4)
const TOG_CON_BOUND, TOG_CON_GOAL, TOG_CON_CIRCLES, TOG_CON_SPHERES, TOG_CON_INFEASIBLE, TOG_CON_USER,
      TOG_CON_MIN_TIME_EQ = Int32.(0:6)
const TOG_PROB_INFEASIBLE, TOG_PROB_MIN_TIME, TOG_PROB_TF_MIN = Int32(1), Int32(2), Int32(4)
const TOG_MODE_ILQR, TOG_MODE_AL = Int32(0), Int32(1)
const TOG_FIELD_X, TOG_FIELD_U, TOG_FIELD_RHO, TOG_FIELD_STATS = Int32(0), Int32(1), Int32(16), Int32(15)
const TOG_NSTATS = 14
const TOG_PN_NSTATS = 7
const TOG_STAT_J, TOG_STAT_ITERATIONS, TOG_STAT_C_MAX, TOG_STAT_AL_ITER, TOG_STAT_TOTAL_STEPS,
      TOG_STAT_FLAGS = 0, 3, 7, 8, 9, 12
const TOG_TRAJ_COST_INCREASED = Int32(1 << 3)
const TOG_TRAJ_SQRT_PD_FAIL = Int32(1 << 6)     # lowrankdowndate! PosDefException (the trajectory stopped)
const TOG_TRAJ_PN_ERROR = Int32(1 << 11)        # _projection_linesearch!'s MethodError (projected_newton.jl:273-277)
const TOG_FIELD_HIST_INNER, TOG_FIELD_HIST_OUTER, TOG_FIELD_HIST_COUNT = Int32(18), Int32(19), Int32(20)
const TOG_PN_C_MAX, TOG_PN_J, TOG_PN_STEPS = 1, 2, 6
const TOG_MODEL_USER = Int32(100)

struct TogConstraint
    type::Int32
    count::Int32
    data::Ptr{Float64}
end
struct TogConstraintSet
    n_con::Int32
    con::Ptr{TogConstraint}
end
struct TogProblemDesc
    model::Int32; integrator::Int32; n::Int32; m::Int32; N::Int32; flags::Int32
    batch::Int64; dt::Float64
    Q::Ptr{Float64}; R::Ptr{Float64}; H::Ptr{Float64}; q::Ptr{Float64}; r::Ptr{Float64}; c::Float64
    Qf::Ptr{Float64}; qf::Ptr{Float64}; cf::Float64
    n_sets::Int32; reserved1::Int32
    sets::Ptr{TogConstraintSet}; knot_set::Ptr{Int32}
    user_model::Ptr{Cvoid}
    R_min_time::Float64
    stage_costs::Ptr{Float64}   # NULL, or the (nc, N-1) per-knot [Q; R; H; q; r; c] of a time-varying Objective
end
# Layout pins (tests/test_julia_layout.py checks these numbers, and the field lists below, against
# include/tog.h compiled by gcc): sizeof and field offsets of the mirrored structs. tog_check_layout()
# asserts them in Julia at first use.
const TOG_LAYOUT = (tog_constraint = 16, tog_constraint_set = 16, tog_problem_desc = 160, tog_options = 200,
                    tog_pn_options = 24, tog_altro_options = 280, tog_altro_result = 96)
const TOG_DESC_OFFSETS = (0, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64, 72, 80, 88, 96, 104, 112, 116, 120,
                          128, 136, 144, 152)

mutable struct TogOptions          # field order = tog_options
    cost_tolerance::Float64; gradient_norm_tolerance::Float64
    iterations::Int32; dJ_counter_limit::Int32; square_root::Int32; bp_reg_type::Int32
    gradient_type::Int32; iterations_linesearch::Int32
    line_search_lower_bound::Float64; line_search_upper_bound::Float64
    bp_reg_increase_factor::Float64; bp_reg_max::Float64; bp_reg_min::Float64; bp_reg_fp::Float64
    max_cost_value::Float64; max_state_value::Float64; max_control_value::Float64
    al_cost_tolerance::Float64; al_cost_tolerance_intermediate::Float64
    al_gradient_norm_tolerance::Float64; al_gradient_norm_tolerance_intermediate::Float64
    constraint_tolerance::Float64; dual_min::Float64; dual_max::Float64; penalty_max::Float64
    penalty_initial::Float64; penalty_scaling::Float64; al_iterations::Int32; kickout_max_penalty::Int32
    function TogOptions()
        o = new()
        ccall((:tog_default_options, libtog), Cvoid, (Ref{TogOptions},), o)
        return o
    end
end

"The same fields, immutable (inline inside tog_altro_options)."
struct TogOptionsI
    cost_tolerance::Float64; gradient_norm_tolerance::Float64
    iterations::Int32; dJ_counter_limit::Int32; square_root::Int32; bp_reg_type::Int32
    gradient_type::Int32; iterations_linesearch::Int32
    line_search_lower_bound::Float64; line_search_upper_bound::Float64
    bp_reg_increase_factor::Float64; bp_reg_max::Float64; bp_reg_min::Float64; bp_reg_fp::Float64
    max_cost_value::Float64; max_state_value::Float64; max_control_value::Float64
    al_cost_tolerance::Float64; al_cost_tolerance_intermediate::Float64
    al_gradient_norm_tolerance::Float64; al_gradient_norm_tolerance_intermediate::Float64
    constraint_tolerance::Float64; dual_min::Float64; dual_max::Float64; penalty_max::Float64
    penalty_initial::Float64; penalty_scaling::Float64; al_iterations::Int32; kickout_max_penalty::Int32
end
TogOptionsI(o::TogOptions) = TogOptionsI((getfield(o, f) for f in fieldnames(TogOptions))...)
struct TogPNOptions                # = tog_pn_options
    n_steps::Int32; solve_type::Int32; active_set_tolerance::Float64; feasibility_tolerance::Float64
end
mutable struct TogAltroOptions     # = tog_altro_options
    opts_al::TogOptionsI
    R_inf::Float64; R_minimum_time::Float64; dt_max::Float64; dt_min::Float64
    projected_newton_tolerance::Float64
    dynamically_feasible_projection::Int32; resolve_feasible_problem::Int32; projected_newton::Int32
    max_steps::Int32
    opts_pn::TogPNOptions
    function TogAltroOptions()
        a = new()
        ccall((:tog_default_altro_options, libtog), Cvoid, (Ref{TogAltroOptions},), a)
        return a
    end
end

mutable struct TogAltroResult      # = tog_altro_result
    inner_capacity::Int32; keep_handle::Int32
    stats::Ptr{Float64}; stats_resolve::Ptr{Float64}; stats_pn::Ptr{Float64}
    hist_inner::Ptr{Float64}; hist_outer::Ptr{Float64}; hist_count::Ptr{Float64}; hist_pn::Ptr{Float64}
    time::Float64; time_al::Float64; time_pn::Float64
    handle::Ptr{Cvoid}
end

const TOG_CHECKED = Ref(false)
"ABI version and struct layouts, once per session."
function tog_check_layout()
    TOG_CHECKED[] && return nothing
    v = ccall((:tog_version, libtog), Int32, ())
    v == TOG_ABI_VERSION || error("libtog ABI version $v, this binding expects $TOG_ABI_VERSION")
    sizeof(TogConstraint) == TOG_LAYOUT.tog_constraint || error("tog_constraint layout")
    sizeof(TogConstraintSet) == TOG_LAYOUT.tog_constraint_set || error("tog_constraint_set layout")
    sizeof(TogProblemDesc) == TOG_LAYOUT.tog_problem_desc || error("tog_problem_desc layout")
    Tuple(Int(fieldoffset(TogProblemDesc, i)) for i = 1:fieldcount(TogProblemDesc)) == TOG_DESC_OFFSETS ||
        error("tog_problem_desc field offsets")
    sizeof(TogOptionsI) == TOG_LAYOUT.tog_options || error("tog_options layout")
    sizeof(TogPNOptions) == TOG_LAYOUT.tog_pn_options || error("tog_pn_options layout")
    sizeof(TogAltroOptions) == TOG_LAYOUT.tog_altro_options || error("tog_altro_options layout")
    sizeof(TogAltroResult) == TOG_LAYOUT.tog_altro_result || error("tog_altro_result layout")
    TOG_CHECKED[] = true
    return nothing
end

togcheck(rc) = rc == TOG_OK ? nothing :
    error("libtog: ", unsafe_string(ccall((:tog_last_error, libtog), Cstring, ())))

# ------------------------------------------------------------------------ models
# The canned Dynamics models the library compiles in (tog_model_id). A discretised model keeps its
# continuous dynamics function in info[:fc] (discretize_model, src/model.jl:607-615), which is the
# identity the binding matches on.
tog_builtin_models() = ((Dynamics.doubleintegrator, Int32(0)), (Dynamics.cartpole, Int32(1)),
                        (Dynamics.quadrotor, Int32(2)), (Dynamics.car, Int32(3)),
                        (Dynamics.pendulum, Int32(4)), (Dynamics.kuka, Int32(5)))

# Model(f!, n, m) with user dynamics: register the compiled libtog plugin of the same f! (a C++
# template over the scalar type built against csrc/tog_plugin.hpp, INTEGRATION.md)
struct TogModel
    ptr::Ptr{Cvoid}
    n::Int
    m::Int
end
const TOG_USER_MODELS = IdDict{Function,TogModel}()
function tog_register_model(model::Model, plugin_path::AbstractString)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    togcheck(ccall((:tog_model_load, libtog), Int32, (Cstring, Ref{Ptr{Cvoid}}), plugin_path, h))
    n, m = Ref{Int32}(0), Ref{Int32}(0)
    togcheck(ccall((:tog_model_dims, libtog), Int32, (Ptr{Cvoid}, Ref{Int32}, Ref{Int32}), h[], n, m))
    (n[] == model.n && m[] == model.m) || throw(ArgumentError("plugin dimensions differ from the model's"))
    TOG_USER_MODELS[model.f] = TogModel(h[], n[], m[])
end

"Model id, user plugin and problem flags of a discrete model (base model, add_slack_controls or add_min_time_controls)."
function tog_model_id(model::Model)
    fc = get(model.info, :fc, model.f)
    for (mc, id) in tog_builtin_models()
        if fc === mc.f
            flags = Int32(0)
            model.m == mc.m + mc.n && (flags |= TOG_PROB_INFEASIBLE)        # add_slack_controls
            (model.n == mc.n + 1 && model.m == mc.m + 1) && (flags |= TOG_PROB_MIN_TIME)  # add_min_time_controls
            return id, C_NULL, flags
        end
    end
    if haskey(TOG_USER_MODELS, fc)
        tm = TOG_USER_MODELS[fc]
        flags = model.m == tm.m + tm.n ? TOG_PROB_INFEASIBLE : Int32(0)
        return TOG_MODEL_USER, tm.ptr, flags
    end
    throw(ArgumentError("model has no libtog kernels: use a Dynamics model or tog_register_model(model, plugin)"))
end

function tog_integrator(model::Model)
    s = get(model.info, :integration, :none)
    s == :rk3 && return TOG_RK3
    s == :rk4 && return TOG_RK4
    s == :midpoint && return TOG_MIDPOINT
    s == :rk3_implicit && return TOG_RK3_IMPLICIT
    s == :midpoint_implicit && return TOG_MIDPOINT_IMPLICIT
    throw(ArgumentError("integration $s has no libtog kernel (rk3, rk4, midpoint, rk3_implicit, midpoint_implicit)"))
end

# ------------------------------------------------------------------------ constraints
# BoundConstraint and goal_constraint are read from their own fields; a Constraint{S} whose function is
# an arbitrary closure (circle/sphere obstacles, problems/quad_obs.jl:59-78) cannot be introspected, so
# the binding builds those itself and records their rows here.
const TOG_CONSTRAINTS = IdDict{Function,Tuple{Int32,Int32,Vector{Float64}}}()

"Circle obstacles on x[1:2] (circle_constraint, src/utils.jl:140-144): circles = [(x0, y0, r), ...]."
function tog_circle_constraint(n::Int, m::Int, circles; label::Symbol=:circles)
    cs = [(Float64(c[1]), Float64(c[2]), Float64(c[3])) for c in circles]
    c!(v, x, u) = (for (i, c) in enumerate(cs); v[i] = circle_constraint(x, c[1], c[2], c[3]); end)
    con = Constraint{Inequality}(c!, n, m, length(cs), label)
    TOG_CONSTRAINTS[con.c] = (TOG_CON_CIRCLES, Int32(length(cs)), Float64[v for c in cs for v in c])
    return con
end

"Sphere obstacles on x[1:3] (sphere_constraint, src/utils.jl:150-156): spheres = [(x0, y0, z0, r), ...]."
function tog_sphere_constraint(n::Int, m::Int, spheres; label::Symbol=:spheres)
    ss = [(Float64(s[1]), Float64(s[2]), Float64(s[3]), Float64(s[4])) for s in spheres]
    c!(v, x, u) = (for (i, s) in enumerate(ss); v[i] = sphere_constraint(x, s[1], s[2], s[3], s[4]); end)
    con = Constraint{Inequality}(c!, n, m, length(ss), label)
    TOG_CONSTRAINTS[con.c] = (TOG_CON_SPHERES, Int32(length(ss)), Float64[v for s in ss for v in s])
    return con
end

"Rows of one constraint for tog_constraint: (type, count, data)."
function tog_constraint_spec(con, n::Int, m::Int)
    if con isa BoundConstraint
        # [x_max; x_min; u_max; u_min]; count 0: ±Inf entries trimmed by the library (trim=true,
        # src/constraints.jl:173-181), 1: every row kept (trim=false: an untrimmed constraint has every
        # entry of `active.all` set)
        untrimmed = all(con.active.all) && !all(isfinite, [con.x_max; con.x_min; con.u_max; con.u_min])
        return TOG_CON_BOUND, Int32(untrimmed ? 1 : 0), Float64[con.x_max; con.x_min; con.u_max; con.u_min]
    elseif con isa Constraint && haskey(TOG_CONSTRAINTS, con.c)
        return TOG_CONSTRAINTS[con.c]
    elseif con isa Constraint{Equality} && con.label == :goal && hasfield(typeof(con.c), :xf)
        xf = getfield(con.c, :xf)            # goal_constraint(xf) (src/constraints.jl:299-304) captures xf
        return TOG_CON_GOAL, Int32(length(xf)), Vector{Float64}(xf)
    elseif con isa Constraint{Equality} && con.label == :infeasible
        return TOG_CON_INFEASIBLE, Int32(0), Float64[]     # infeasible_constraints (src/constraints.jl:306-314)
    elseif con isa Constraint{Equality} && con.label == :min_time_eq
        return TOG_CON_MIN_TIME_EQ, Int32(0), Float64[]    # mintime_equality (minimum_time.jl:106-124)
    end
    throw(ArgumentError("constraint $(con.label) has no libtog rows: build it with tog_circle_constraint / " *
                        "tog_sphere_constraint, or as a TOG_CON_USER row of a registered plugin"))
end

# ------------------------------------------------------------------------ Problem -> tog_problem_desc
"A tog_problem_desc and every array it points into (kept alive while the handle lives)."
mutable struct TogDesc
    desc::Base.RefValue{TogProblemDesc}
    keep::Vector{Any}
end

# knot 1's stage cost, the terminal cost, and whether knots 2..N-1 carry costs of their own (a
# time-varying Objective, src/objective.jl:15-29: marshalled as tog_problem_desc.stage_costs)
function stage_and_terminal_costs(obj::Objective, N::Int)
    ℓ = obj.cost[1]
    ℓ isa QuadraticCost || throw(ArgumentError("libtog evaluates QuadraticCost / LQRCost objectives"))
    varying = false
    for k = 2:N-1
        c = obj.cost[k]
        c isa QuadraticCost || throw(ArgumentError("libtog evaluates QuadraticCost stage costs"))
        varying |= !(c === ℓ || (c.Q == ℓ.Q && c.R == ℓ.R && c.H == ℓ.H && c.q == ℓ.q && c.r == ℓ.r && c.c == ℓ.c))
    end
    ℓN = obj.cost[N]
    ℓN isa QuadraticCost || throw(ArgumentError("terminal cost must be a QuadraticCost"))
    return ℓ, ℓN, varying
end

# the (nc, N-1) column-major table of tog_problem_desc.stage_costs: per knot [vec(Q); vec(R); vec(H); q; r; c]
stage_cost_table(obj::Objective, N::Int) =
    reduce(hcat, [vcat(vec(Matrix{Float64}(c.Q)), vec(Matrix{Float64}(c.R)), vec(Matrix{Float64}(c.H)),
                       Vector{Float64}(c.q), Vector{Float64}(c.r), Float64(c.c)) for c in obj.cost[1:N-1]])

"""
    tog_desc(prob::Problem; batch=1, R_min_time=0.0) -> TogDesc

Marshal `prob` into the C descriptor: model id and problem flags, integrator, N, dt, the LQR/quadratic
stage and terminal cost (column-major copies), and the per-knot ConstraintSets flattened to
tog_constraint entries in the order of the knot's constraint vector (labels in insertion order,
src/constraint_sets.jl:64-94). Knots whose ConstraintSet is the same object share one table entry.
"""
function tog_desc(prob::Problem; batch::Integer=1, R_min_time::Real=0.0, tf_min::Bool=false)
    tog_check_layout()
    model = prob.model
    n, m, N = model.n, model.m, prob.N
    id, user, flags = tog_model_id(model)
    keep = Any[]
    mat(A, r, c) = (a = Matrix{Float64}(reshape(collect(A), r, c)); push!(keep, a); a)
    vec_(v) = (a = Vector{Float64}(collect(v)); push!(keep, a); a)
    ℓ, ℓN, varying = stage_and_terminal_costs(prob.obj, N)
    table = varying ? stage_cost_table(prob.obj, N) : Matrix{Float64}(undef, 0, 0)
    push!(keep, table)
    Q = mat(ℓ.Q, n, n); R = mat(ℓ.R, m, m); H = mat(ℓ.H, m, n); q = vec_(ℓ.q); r = vec_(ℓ.r)
    Qf = mat(ℓN.Q, n, n); qf = vec_(ℓN.q)
    # constraint sets: one entry per distinct ConstraintSet object
    set_ids = IdDict{Any,Int32}()
    sets = TogConstraintSet[]
    knot_set = fill(Int32(-1), N)
    for k = 1:N
        C = prob.constraints.C[k]
        isempty(C) && continue
        if !haskey(set_ids, C)
            cons = TogConstraint[]
            for con in C
                t, cnt, data = tog_constraint_spec(con, n, m)
                push!(keep, data)
                push!(cons, TogConstraint(t, cnt, isempty(data) ? Ptr{Float64}(C_NULL) : pointer(data)))
            end
            push!(keep, cons)
            push!(sets, TogConstraintSet(Int32(length(cons)), pointer(cons)))
            set_ids[C] = Int32(length(sets) - 1)
        end
        knot_set[k] = set_ids[C]
    end
    push!(keep, sets); push!(keep, knot_set)
    tf_min && (flags |= TOG_PROB_TF_MIN)   # tf = 0: tog_solve_altro builds minimum_time_problem
    d = TogProblemDesc(id, tog_integrator(model), Int32(n), Int32(m), Int32(N), flags, Int64(batch),
                       Float64(prob.dt), pointer(Q), pointer(R), pointer(H), pointer(q), pointer(r),
                       Float64(ℓ.c), pointer(Qf), pointer(qf), Float64(ℓN.c), Int32(length(sets)), Int32(0),
                       isempty(sets) ? Ptr{TogConstraintSet}(C_NULL) : pointer(sets), pointer(knot_set),
                       user, Float64(R_min_time), varying ? pointer(table) : Ptr{Float64}(C_NULL))
    return TogDesc(Ref(d), keep)
end

"Live fields of iLQRSolverOptions / AugmentedLagrangianSolverOptions (ilqr_solver.jl:7-81, augmented_lagrangian_solver.jl:8-66)."
function tog_options(opts::AbstractSolverOptions)
    o = TogOptions()
    if opts isa AugmentedLagrangianSolverOptions
        al, il = opts, opts.opts_uncon
        o.al_cost_tolerance = al.cost_tolerance
        o.al_cost_tolerance_intermediate = al.cost_tolerance_intermediate
        o.al_gradient_norm_tolerance = al.gradient_norm_tolerance
        o.al_gradient_norm_tolerance_intermediate = al.gradient_norm_tolerance_intermediate
        o.constraint_tolerance = al.constraint_tolerance
        o.dual_min = al.dual_min; o.dual_max = al.dual_max; o.penalty_max = al.penalty_max
        o.penalty_initial = al.penalty_initial; o.penalty_scaling = al.penalty_scaling
        o.al_iterations = al.iterations; o.kickout_max_penalty = al.kickout_max_penalty
    else
        il = opts::iLQRSolverOptions
    end
    o.cost_tolerance = il.cost_tolerance
    o.gradient_norm_tolerance = il.gradient_norm_tolerance
    o.iterations = il.iterations
    o.dJ_counter_limit = il.dJ_counter_limit
    o.square_root = il.square_root
    il.bp_reg_type in (:control, :state) || throw(ArgumentError("bp_reg_type must be :control or :state"))
    o.bp_reg_type = il.bp_reg_type == :control ? 0 : 1
    gt = (todorov = 0, feedforward = 1, ℓ2 = 2, ℓinf = 3)
    haskey(gt, il.gradient_type) || throw(ArgumentError("gradient_type $(il.gradient_type)"))
    o.gradient_type = gt[il.gradient_type]
    o.iterations_linesearch = il.iterations_linesearch
    o.line_search_lower_bound = il.line_search_lower_bound
    o.line_search_upper_bound = il.line_search_upper_bound
    o.bp_reg_increase_factor = il.bp_reg_increase_factor
    o.bp_reg_max = il.bp_reg_max; o.bp_reg_min = il.bp_reg_min; o.bp_reg_fp = il.bp_reg_fp
    o.max_cost_value = il.max_cost_value; o.max_state_value = il.max_state_value
    o.max_control_value = il.max_control_value
    return o
end

# ------------------------------------------------------------------------ the solver plugin
"""
    BatchediLQRSolverOptions{T}(; opts=AugmentedLagrangianSolverOptions{T}(), device=0, max_steps=0)

iLQR (`opts::iLQRSolverOptions`) or AL-iLQR (`opts::AugmentedLagrangianSolverOptions`) on the GPU.
`max_steps` caps the batch steps (0: run until every trajectory has finished; each trajectory stops
at its own iteration limits).
"""
@with_kw mutable struct BatchediLQRSolverOptions{T} <: AbstractSolverOptions{T}
    opts::AbstractSolverOptions{T} = AugmentedLagrangianSolverOptions{T}()
    device::Int = 0
    max_steps::Int = 0
end

mutable struct BatchediLQRSolver{T} <: AbstractSolver{T}
    opts::BatchediLQRSolverOptions{T}
    stats::Dict{Symbol,Any}
    handle::Ptr{Cvoid}
    desc::TogDesc
    n::Int
    m::Int
    N::Int
    B::Int
end

function _tog_create(desc::TogDesc, opts::BatchediLQRSolverOptions)
    o = tog_options(opts.opts)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    togcheck(ccall((:tog_create, libtog), Int32, (Ref{TogProblemDesc}, Ref{TogOptions}, Int32, Ref{Ptr{Cvoid}}),
                   desc.desc, o, opts.device, h))
    return h[]
end

function _tog_solver(desc::TogDesc, opts::BatchediLQRSolverOptions{T}, n, m, N, B) where T
    s = BatchediLQRSolver{T}(opts, Dict{Symbol,Any}(), _tog_create(desc, opts), desc, n, m, N, B)
    finalizer(s -> ccall((:tog_destroy, libtog), Int32, (Ptr{Cvoid},), s.handle), s)
    return s
end

"AbstractSolver(prob, opts) (src/solvers.jl:60-62): marshal the problem, allocate the device buffers."
function AbstractSolver(prob::Problem{T,D}, opts::BatchediLQRSolverOptions{T}) where {T<:AbstractFloat,D<:DynamicsType}
    return AbstractSolver([prob], opts)
end

"A batch of B copies of one problem that differ in x0 and the initial controls."
function AbstractSolver(probs::Vector{<:Problem{T}}, opts::BatchediLQRSolverOptions{T}) where T
    p = probs[1]
    desc = tog_desc(p; batch=length(probs))
    return _tog_solver(desc, opts, p.model.n, p.model.m, p.N, length(probs))
end

"solve!(prob, solver) (src/solvers.jl:53-54): the problem's X, U are written in place."
function solve!(prob::Problem{T,D}, solver::BatchediLQRSolver{T}) where {T<:AbstractFloat,D<:DynamicsType}
    solve!([prob], solver)
    return solver
end

function solve!(probs::Vector{<:Problem{T}}, s::BatchediLQRSolver{T}) where T
    n, m, N, B = s.n, s.m, s.N, length(probs)
    B == s.B || throw(ArgumentError("the solver was built for $(s.B) trajectories"))
    x0 = Matrix{Float64}(undef, n, B)
    U = Array{Float64}(undef, m, N - 1, B)
    X = Array{Float64}(undef, n, N, B)
    for (b, p) in enumerate(probs)
        x0[:, b] = p.x0
        for k = 1:N-1; U[:, k, b] = p.U[k]; end
        for k = 1:N; X[:, k, b] = p.X[k]; end     # NaN (empty_state, src/problem.jl:232): initial rollout
    end
    togcheck(ccall((:tog_set_state, libtog), Int32, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                   s.handle, x0, U, X))
    mode = s.opts.opts isa AugmentedLagrangianSolverOptions ? TOG_MODE_AL : TOG_MODE_ILQR
    # 0: tog_solve_budget, the iteration budget x the line-search rounds of pending mode
    max_steps = s.opts.max_steps > 0 ? s.opts.max_steps : 0
    togcheck(ccall((:tog_solve, libtog), Int32, (Ptr{Cvoid}, Int32, Int32), s.handle, mode, max_steps))
    togcheck(ccall((:tog_get, libtog), Int32, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.handle, TOG_FIELD_X, X))
    togcheck(ccall((:tog_get, libtog), Int32, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.handle, TOG_FIELD_U, U))
    St = Matrix{Float64}(undef, TOG_NSTATS, B)
    togcheck(ccall((:tog_get, libtog), Int32, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.handle, TOG_FIELD_STATS, St))
    for (b, p) in enumerate(probs)
        copyto!(p.X, [X[:, k, b] for k = 1:N])
        copyto!(p.U, [U[:, k, b] for k = 1:N-1])
    end
    flags = Int32.(St[TOG_STAT_FLAGS+1, :])
    s.stats[:iterations] = Int.(St[TOG_STAT_TOTAL_STEPS+1, :])
    s.stats[:cost] = St[TOG_STAT_J+1, :]
    s.stats[:c_max] = St[TOG_STAT_C_MAX+1, :]
    s.stats[:iterations_outer] = Int.(St[TOG_STAT_AL_ITER+1, :])
    s.stats[:flags] = flags
    # the reference's exceptions, after the batch: chol_minus's PosDefException (backward_pass.jl:186-192),
    # then the cost increase (forward_pass.jl:80-82)
    any(f -> f & TOG_TRAJ_SQRT_PD_FAIL != 0, flags) && throw(PosDefException(0))
    any(f -> f & TOG_TRAJ_COST_INCREASED != 0, flags) && error("Cost increased during Forward Pass")
    return s
end

"reset!(solver) (src/solvers.jl:63-67; iLQRSolver's: ρ = dρ = 0, stats cleared, ilqr_solver.jl:146-154)."
function reset!(s::BatchediLQRSolver)
    empty!(s.stats)
    ρ = zeros(2, s.B)
    togcheck(ccall((:tog_set, libtog), Int32, (Ptr{Cvoid}, Int32, Ptr{Float64}), s.handle, TOG_FIELD_RHO, ρ))
    return nothing
end

"copy(solver) (src/solvers.jl:69-73): a new handle on the same descriptor, no shared memory."
copy(s::BatchediLQRSolver{T}) where T = _tog_solver(s.desc, deepcopy(s.opts), s.n, s.m, s.N, s.B)

"size(solver) (src/solvers.jl:75-79): (n, m, N)."
size(s::BatchediLQRSolver) = (s.n, s.m, s.N)

solver_name(::BatchediLQRSolverOptions) = "libtog batched iLQR"

# ------------------------------------------------------------------------ ALTRO
"ALTROSolverOptions (src/solvers/altro/altro_solver.jl:6-65) -> tog_altro_options."
function tog_altro_options(opts::ALTROSolverOptions)
    a = TogAltroOptions()
    a.opts_al = TogOptionsI(tog_options(opts.opts_al))
    a.R_inf = opts.R_inf; a.R_minimum_time = opts.R_minimum_time
    a.dt_max = opts.dt_max; a.dt_min = opts.dt_min
    a.projected_newton_tolerance = opts.projected_newton_tolerance
    a.dynamically_feasible_projection = opts.dynamically_feasible_projection
    a.resolve_feasible_problem = opts.resolve_feasible_problem
    a.projected_newton = opts.projected_newton
    pn = opts.opts_pn
    pn.solve_type in (:feasible, :optimal) || throw(ArgumentError("solve_type must be :feasible or :optimal"))
    a.opts_pn = TogPNOptions(Int32(pn.n_steps), Int32(pn.solve_type == :optimal ? 1 : 0), pn.active_set_tolerance,
                             pn.feasibility_tolerance)
    return a
end

"Route solve!(prob, ::ALTROSolverOptions) to libtog (false: the reference's Julia solver)."
const TOG_ALTRO = Ref(true)

"""
The solver `solve!(prob, ::ALTROSolverOptions)` returns (altro_solver.jl:70-75, altro_methods.jl:40-52):
`stats` (:time, :time_al, :time_pn), `solver_al.stats` (the AL phase's :iterations, :iterations_total,
:iterations_inner, :cost, :c_max, :penalty_max vectors; its inner solves' stats in `solver_al.stats_uncon`)
and `solver_pn.stats` (:iterations, :cost, :c_max per newton step), so callers such as
examples/IROS_2019/quadrotor_maze.jl:75-79 read them unchanged.
"""
struct TogStatsSolver{T} <: AbstractSolver{T}
    opts::AbstractSolverOptions{T}
    stats::Dict{Symbol,Any}
    stats_uncon::Vector{Dict{Symbol,Any}}
end
struct TogALTROSolver{T} <: AbstractSolver{T}
    opts::ALTROSolverOptions{T}
    stats::Dict{Symbol,Any}
    solver_al::TogStatsSolver{T}
    solver_pn::TogStatsSolver{T}
end

"record_iteration!'s vectors of one inner solve (ilqr_methods.jl:77-89) from history records r (3 x k)."
function _tog_ilqr_stats(r::AbstractMatrix{Float64})
    k = size(r, 2)
    zc = 0
    for j = 1:k; zc = r[2, j] == 0.0 ? zc + 1 : 0; end
    return Dict{Symbol,Any}(:iterations => k, :cost => r[1, :], :dJ => r[2, :], :gradient => r[3, :],
                            :dJ_zero_counter => zc)
end

"""
    solve!(prob::Problem{Float64,Discrete}, opts::ALTROSolverOptions{Float64})

The reference's ALTRO entry (src/solvers/altro/altro_methods.jl:2-53; README.md:32-67's quick start),
more specific than its `solve!(::Problem{T,Discrete}, ::ALTROSolverOptions)`, so a Float64 problem on a
libtog model reaches tog_solve_altro_ex: altro_problem (an initial state trajectory -> infeasible_problem;
tf = 0 -> minimum_time_problem), the AL solve on the GPU, projected Newton, process_results! and the feasible
resolve run in libtog (csrc/tog_altro.cpp). prob.X, prob.U are written in place; a minimum-time solve leaves
prob.U[k] = [u; u; h] as the reference's process_results! does. Returns a TogALTROSolver (the reference's
ALTROSolver fields: opts, stats, solver_al, solver_pn).
"""
function solve!(prob::Problem{Float64,Discrete}, opts::ALTROSolverOptions{Float64})
    if !TOG_ALTRO[]
        return invoke(solve!, Tuple{Problem{Float64,Discrete},ALTROSolverOptions}, prob, opts)
    end
    tog_check_layout()
    if opts.projected_newton   # altro_methods.jl:5-13 (mutates opts_al, as the reference does)
        if opts.projected_newton_tolerance >= 0
            opts.opts_al.constraint_tolerance = opts.projected_newton_tolerance
        else
            opts.opts_al.constraint_tolerance = 0
            opts.opts_al.kickout_max_penalty = true
        end
    end
    n, m, N = prob.model.n, prob.model.m, prob.N
    tf_min = prob.tf == 0.0
    desc = tog_desc(prob; batch=1, tf_min=tf_min)
    a = tog_altro_options(opts)
    x0 = Vector{Float64}(prob.x0)
    X = Matrix{Float64}(undef, n, N)
    for k = 1:N; X[:, k] = prob.X[k]; end      # all NaN (empty_state): no infeasible start
    U = Matrix{Float64}(undef, m, N - 1)
    for k = 1:N-1; U[:, k] = prob.U[k]; end
    h = Vector{Float64}(undef, N - 1)
    St, Sr = zeros(TOG_NSTATS), zeros(TOG_NSTATS)
    Spn = zeros(TOG_PN_NSTATS)
    al_it, it = opts.opts_al.iterations, opts.opts_al.opts_uncon.iterations
    cap = al_it * (it + 1) + 1
    Hin, Hout, Hcnt = zeros(3, cap), zeros(4, al_it + 1), zeros(2)
    npn = opts.projected_newton ? max(opts.opts_pn.n_steps, 0) : 0
    Hpn = fill(NaN, 2, max(npn, 1))
    GC.@preserve St Sr Spn Hin Hout Hcnt Hpn begin
        r = TogAltroResult(Int32(cap), Int32(0), pointer(St), pointer(Sr), pointer(Spn), pointer(Hin),
                           pointer(Hout), pointer(Hcnt), npn > 0 ? pointer(Hpn) : Ptr{Float64}(C_NULL),
                           0.0, 0.0, 0.0, C_NULL)
        togcheck(ccall((:tog_solve_altro_ex, libtog), Int32,
                       (Ref{TogProblemDesc}, Ref{TogAltroOptions}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                        Ptr{Float64}, Ref{TogAltroResult}),
                       desc.desc, a, Int32(0), x0, X, U, h, r))
    end
    copyto!(prob.X, [X[:, k] for k = 1:N])
    if tf_min   # process_results! (altro_methods.jl:81-85): U[k] = [u; u; h]
        for k = 1:N-1; prob.U[k] = [U[:, k]; U[:, k]; h[k]]; end
    else
        copyto!(prob.U, [U[:, k] for k = 1:N-1])
    end
    flags = Int32(St[TOG_STAT_FLAGS+1]) | Int32(Sr[TOG_STAT_FLAGS+1])
    flags & TOG_TRAJ_SQRT_PD_FAIL != 0 && throw(PosDefException(0))   # backward_pass.jl:186-192
    flags & TOG_TRAJ_COST_INCREASED != 0 && error("Cost increased during Forward Pass")  # forward_pass.jl:80-82
    # solver_al.stats (augmented_lagrangian_methods.jl:79-97); an unconstrained problem's AL phase keeps
    # only its inner records (the AL solver's own records need constraints)
    n_in, n_out = Int(Hcnt[1]), Int(Hcnt[2])
    it_in = Int.(Hout[1, 1:n_out])
    uncon = Dict{Symbol,Any}[]
    o = 0
    for k in it_in
        push!(uncon, _tog_ilqr_stats(Hin[:, o+1:o+k]))
        o += k
    end
    sal = Dict{Symbol,Any}(:iterations => n_out, :iterations_total => sum(it_in), :iterations_inner => it_in,
                           :cost => Hout[2, 1:n_out], :c_max => Hout[3, 1:n_out], :penalty_max => Hout[4, 1:n_out],
                           :flags => flags)
    spn = Dict{Symbol,Any}(:iterations => 0, :cost => Float64[], :c_max => Float64[])
    if opts.projected_newton
        k = Int(Spn[TOG_PN_STEPS+1])
        spn = Dict{Symbol,Any}(:iterations => k, :cost => Hpn[1, 1:k], :c_max => Hpn[2, 1:k])
        Int32(St[TOG_STAT_FLAGS+1]) & TOG_TRAJ_PN_ERROR != 0 &&   # projected_newton.jl:273-277
            error("projected Newton: line search did not reduce the violation")
    end
    stats = Dict{Symbol,Any}(:time => r.time, :time_al => r.time_al, :time_pn => r.time_pn)
    return TogALTROSolver{Float64}(opts, stats, TogStatsSolver{Float64}(opts.opts_al, sal, uncon),
                                   TogStatsSolver{Float64}(opts.opts_pn, spn, Dict{Symbol,Any}[]))
end
