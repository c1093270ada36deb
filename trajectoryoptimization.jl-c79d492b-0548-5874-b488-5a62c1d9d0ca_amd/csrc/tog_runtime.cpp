// tog_runtime.cpp — C ABI (include/tog.h) over the HIP kernels. Host code only: device buffers,
// problem marshalling (tog_problem_desc -> DevProblem + constraint rows), launch sequencing.
//
// Ownership: the handle owns every device buffer; callers own host arrays. One host thread per
// handle; handles are independent (one per GPU for multi-GPU runs).
#include <cmath>
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include <dlfcn.h>

#include "tog_plugin.hpp"
#include "tog_cost_plugin.hpp"

using namespace tog;

namespace tog {
const ModelOps* ops_double_integrator();
const ModelOps* ops_cartpole();
const ModelOps* ops_quadrotor();
const ModelOps* ops_car();
const ModelOps* ops_pendulum();
const ModelOps* ops_kuka();
const ModelOps* ops_kuka_implicit();
// add_slack_controls(model) variants (infeasible start, src/model.jl:761-779)
const ModelOps* ops_inf_double_integrator();
const ModelOps* ops_inf_cartpole();
const ModelOps* ops_inf_quadrotor();
const ModelOps* ops_inf_car();
const ModelOps* ops_inf_pendulum();
const ModelOps* ops_inf_kuka();
// add_min_time_controls(model) variants (minimum time, src/solvers/altro/minimum_time.jl:83-104)
const ModelOps* ops_mt_pendulum();
const ModelOps* ops_mtinf_pendulum();
const ModelOps* ops_mtinf_car();
const ModelOps* ops_mtinf_double_integrator();
const ModelOps* ops_mtinf_cartpole();
const ModelOps* ops_mtinf_quadrotor();
const ModelOps* ops_mtinf_kuka();
const ModelOps* ops_mt_car();
const ModelOps* ops_mt_double_integrator();
const ModelOps* ops_mt_quadrotor();
const ModelOps* ops_mt_cartpole();
const ModelOps* ops_mt_kuka();
}  // namespace tog

static thread_local std::string g_err;

// active trajectories at or below which tog_solve_step runs the latency-sized kernel variants
// (DevBuffers::tail): 2048 trajectories = 512 team waves, at most one per SIMD
static constexpr double TAIL_ACTIVE = 2048.0;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Host watchdog of the blocking readbacks: wait for `ev` polling, and give up after TOG_WATCHDOG_S seconds
// (default 600) with TOG_ERR_DEVICE, so that a kernel that never finishes (e.g. a lost LDS hand-off in the
// tail backward kernel, whose waits are unbounded for speed, tog_bwd_quad.hpp) is reported instead of
// blocking the caller forever. The device queue itself stays hung: the process should exit.
static int wait_event(hipEvent_t ev, const char* what) {
  static const double limit = getenv("TOG_WATCHDOG_S") ? atof(getenv("TOG_WATCHDOG_S")) : 600.0;
  const auto t0 = std::chrono::steady_clock::now();
  unsigned polls = 0;
  while (true) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return TOG_OK;
    if (e != hipErrorNotReady) return fail(TOG_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    if (++polls > 64) {  // (first a short spin: a check usually completes within microseconds)
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit)
        return fail(TOG_ERR_DEVICE, std::string(what) + ": the device did not finish within TOG_WATCHDOG_S = " +
                                        std::to_string(limit) + " s (a hung kernel?)");
      std::this_thread::sleep_for(std::chrono::microseconds(polls < 1000 ? 2 : 200));
    }
  }
}

#define HIPCHECK(expr)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(TOG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct tog_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int model = 0, integ = 0, n = 0, m = 0, N = 0, pmax = 0, nrows = 0, nq = 0;
  long long B = 0;
  double last_active = -1.0;  // n_active of the last host stats readback (-1: none yet)
  int mode = TOG_MODE_ILQR;
  tog_options opts;
  DevProblem hostP;
  DevProblem* dP = nullptr;
  int* d_knot_off = nullptr;
  int* d_knot_cnt = nullptr;
  int* d_knot_nx = nullptr;
  ConRow* d_rows = nullptr;
  DevBuffers buf = {};
  const ModelOps* ops = nullptr;
  int bwd_team = 0;  // backward pass on column-per-lane teams (else one wave per trajectory, LDS)
  double* d_scratch = nullptr;  // B doubles (J_prev / J_out staging)
  double* d_scratch2 = nullptr; // B doubles
  int* d_iscratch = nullptr;    // B ints
  double* d_stats = nullptr;    // 3 doubles
  int* d_act_list = nullptr;    // B ints: the active trajectories of a compacted tail step
  int* d_act_count = nullptr;
  std::vector<void*> allocs;
  // live per-kernel timing (tog_profile)
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<int> ev_kind;  // kernel id per recorded (start, end) pair
  size_t ev_used = 0;
  // tog_create_multi: a handle over several devices owns one plain handle per device, each with a
  // contiguous slice [part_off[i], part_off[i+1]) of the batch; every entry point fans out
  std::vector<tog_handle*> parts;
  std::vector<long long> part_off;
  // second stream + fork/join events: the forward pass overlaps the decided trajectories' commit
  // with the second speculative round (tog_kernels.hpp forward_i)
  StreamPair sp = {nullptr, nullptr, nullptr};
  // projected Newton workspace, allocated by the first tog_solve_pn (tog_pn.hpp)
  PNBuffers pn = {};
  bool pn_alloc = false, pn_opt_alloc = false;
  // solver_pn.stats histories of the last tog_solve_pn: (2, n_steps, B) [cost, c_max], records per trajectory
  std::vector<double> pn_hist;
  std::vector<int32_t> pn_hist_rec;
  int pn_hist_steps = -1;
  // asynchronous stopping check (tog_batch_stats_begin / _end): pinned landing buffer + completion event
  double* h_stats = nullptr;
  hipEvent_t stats_ev = nullptr;
  bool stats_pending = false;
  // tog_history_enable's allocations (DevBuffers::hist_in / hist_out point into them while recording is on)
  double *hist_in_alloc = nullptr, *hist_out_alloc = nullptr;
  int hist_cap_alloc = 0, hist_ocap_alloc = 0;
  hipEvent_t sync_ev = nullptr;  // tog_synchronize's watchdog wait
};

static hipEvent_t next_event(tog_handle* h) {
  if (h->ev_used == h->ev_pool.size()) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    h->ev_pool.push_back(e);
  }
  return h->ev_pool[h->ev_used++];
}

// launch `fn` bracketed by timing events when profiling is on
template <class F>
static void timed(tog_handle* h, int kind, F&& fn) {
  if (!h->profiling) {
    fn();
    return;
  }
  hipEvent_t a = next_event(h), b = next_event(h);
  (void)hipEventRecord(a, h->stream);
  fn();
  (void)hipEventRecord(b, h->stream);
  h->ev_kind.push_back(kind);
}

// a loaded GenericCost plugin (tog_generic_cost_load)
struct tog_generic_cost {
  using expand_fn = int (*)(int, const double*, const double*, long long, double*, double*, double*, double*,
                            double*, double*, void*);
  void* so;
  int n, m;
  expand_fn ex;
};

// a loaded user model plugin (tog_model_load)
struct tog_model {
  void* so;
  const tog::ModelOps* ops;
  const tog::ModelOps* ops_inf;
  const tog::ModelOps* ops_mt;  // MinTime<M> (add_min_time_controls)
};

static const ModelOps* ops_for(int model, bool infeasible, bool min_time, const tog_model* user, int integ) {
  if (model == TOG_MODEL_KUKA && !infeasible && !min_time && (integ == TOG_RK3_IMPLICIT || integ == TOG_MIDPOINT_IMPLICIT))
    return ops_kuka_implicit();
  if (min_time && infeasible) {  // minimum_time_problem(infeasible_problem(prob))
    switch (model) {
      case TOG_MODEL_PENDULUM: return ops_mtinf_pendulum();
      case TOG_MODEL_CAR: return ops_mtinf_car();
      case TOG_MODEL_DOUBLE_INTEGRATOR: return ops_mtinf_double_integrator();
      case TOG_MODEL_CARTPOLE: return ops_mtinf_cartpole();
      case TOG_MODEL_QUADROTOR: return ops_mtinf_quadrotor();
      case TOG_MODEL_KUKA: return ops_mtinf_kuka();
    }
    return nullptr;
  }
  if (min_time) {
    if (model == TOG_MODEL_USER) return user ? user->ops_mt : nullptr;
    switch (model) {
      case TOG_MODEL_PENDULUM: return ops_mt_pendulum();
      case TOG_MODEL_CAR: return ops_mt_car();
      case TOG_MODEL_DOUBLE_INTEGRATOR: return ops_mt_double_integrator();
      case TOG_MODEL_QUADROTOR: return ops_mt_quadrotor();
      case TOG_MODEL_CARTPOLE: return ops_mt_cartpole();
      case TOG_MODEL_KUKA: return ops_mt_kuka();
    }
    return nullptr;
  }
  if (model == TOG_MODEL_USER) return user ? (infeasible ? user->ops_inf : user->ops) : nullptr;
  if (infeasible) {
    switch (model) {
      case TOG_MODEL_DOUBLE_INTEGRATOR: return ops_inf_double_integrator();
      case TOG_MODEL_CARTPOLE: return ops_inf_cartpole();
      case TOG_MODEL_QUADROTOR: return ops_inf_quadrotor();
      case TOG_MODEL_CAR: return ops_inf_car();
      case TOG_MODEL_PENDULUM: return ops_inf_pendulum();
      case TOG_MODEL_KUKA: return ops_inf_kuka();
    }
    return nullptr;
  }
  switch (model) {
    case TOG_MODEL_DOUBLE_INTEGRATOR: return ops_double_integrator();
    case TOG_MODEL_CARTPOLE: return ops_cartpole();
    case TOG_MODEL_QUADROTOR: return ops_quadrotor();
    case TOG_MODEL_CAR: return ops_car();
    case TOG_MODEL_PENDULUM: return ops_pendulum();
    case TOG_MODEL_KUKA: return ops_kuka();
  }
  return nullptr;
}

// upper Cholesky (dpotrf 'U') of a symmetric matrix; returns false if not PD
static bool host_chol_upper(const double* A, int n, double* U) {
  for (int i = 0; i < n * n; i++) U[i] = 0.0;
  for (int j = 0; j < n; j++) {
    double s = A[j + n * j];
    for (int k = 0; k < j; k++) s -= U[k + n * j] * U[k + n * j];
    if (!(s > 0.0)) return false;
    const double ujj = sqrt(s);
    U[j + n * j] = ujj;
    for (int c = j + 1; c < n; c++) {
      double t = A[j + n * c];
      for (int k = 0; k < j; k++) t -= U[k + n * j] * U[k + n * c];
      U[j + n * c] = t / ujj;
    }
  }
  return true;
}

// Flatten the ordered constraint sets into per-knot rows (src/constraint_sets.jl:64-131).
static int build_rows(const tog_problem_desc* d, int slack, int pcap, int has_con, std::vector<ConRow>& rows,
                      std::vector<int>& off, std::vector<int>& cnt) {
  const int n = d->n, m = d->m, N = d->N;
  const int mt = (d->flags & TOG_PROB_MIN_TIME) ? 1 : 0;  // h, the last control
  off.assign(N, 0);
  cnt.assign(N, 0);
  for (int k = 0; k < N; k++) {
    off[k] = (int)rows.size();
    const int si = d->knot_set ? d->knot_set[k] : -1;
    if (si < 0) continue;
    if (si >= d->n_sets) return fail(TOG_ERR_ARG, "knot_set index out of range");
    const bool term = (k == N - 1);
    const tog_constraint_set& set = d->sets[si];
    for (int c = 0; c < set.n_con; c++) {
      const tog_constraint& con = set.con[c];
      const double* D = con.data;
      switch (con.type) {
        case TOG_CON_BOUND: {
          // data = [x_max(n), x_min(n), u_max(m), u_min(m)]; order [x_max; u_max; x_min; u_min].
          // count 0: trim = true (infinite bounds dropped); 1: trim = false (every row kept). The slack
          // controls of an infeasible-start problem are never bounded: its BoundConstraint keeps the model's
          // m (update_constraint_set_jacobians, constraint_sets.jl:135-150)
          // (trimmed bounds: rows for the finite entries over all m; the infeasible minimum-time problem's
          // combined bound reaches u[1:m+1], mintime_constraints, minimum_time.jl:125-141)
          // (trim=false: the model's controls and, on a minimum-time problem, the time step h = u[m-1])
          const bool keep = (con.count == 1);
          const int mb = keep ? m - slack - mt : m;
          auto u_row = [&](int i) { return i < mb || (keep && mt && i == m - 1); };
          for (int i = 0; i < n; i++)
            if (keep || isfinite(D[i])) rows.push_back({ROW_XMAX, i, D[i], 0, 0, 0});
          if (!term)
            for (int i = 0; i < m; i++)
              if (u_row(i) && (keep || isfinite(D[2 * n + i]))) rows.push_back({ROW_UMAX, i, D[2 * n + i], 0, 0, 0});
          for (int i = 0; i < n; i++)
            if (keep || isfinite(D[n + i])) rows.push_back({ROW_XMIN, i, D[n + i], 0, 0, 0});
          if (!term)
            for (int i = 0; i < m; i++)
              if (u_row(i) && (keep || isfinite(D[2 * n + m + i]))) rows.push_back({ROW_UMIN, i, D[2 * n + m + i], 0, 0, 0});
          break;
        }
        case TOG_CON_GOAL: {  // count: rows x[1:count] - xf (the goal's inds); 0 = n
          const int ng = con.count > 0 ? con.count : n;
          if (ng > n) return fail(TOG_ERR_ARG, "goal constraint longer than the state");
          if (term)
            for (int i = 0; i < ng; i++) rows.push_back({ROW_GOAL, i, D[i], 0, 0, 0});
          break;
        }
        case TOG_CON_CIRCLES:
          if (!term)
            for (int o = 0; o < con.count; o++)
              rows.push_back({ROW_CIRCLE, 0, D[3 * o], D[3 * o + 1], 0.0, D[3 * o + 2]});
          break;
        case TOG_CON_SPHERES:
          if (!term)
            for (int o = 0; o < con.count; o++)
              rows.push_back({ROW_SPHERE, 0, D[4 * o], D[4 * o + 1], D[4 * o + 2], D[4 * o + 3]});
          break;
        case TOG_CON_INFEASIBLE:
          // infeasible_constraints(n, m) (src/constraints.jl:306-314): c = u[m+1:m+n], stage only
          if (!slack) return fail(TOG_ERR_ARG, "TOG_CON_INFEASIBLE needs a TOG_PROB_INFEASIBLE problem");
          if (!term)
            for (int i = 0; i < slack; i++) rows.push_back({ROW_USLACK, m - slack - mt + i, 0.0, 0.0, 0.0, 0.0});
          break;
        case TOG_CON_MIN_TIME_EQ:
          if (!(d->flags & TOG_PROB_MIN_TIME)) return fail(TOG_ERR_ARG, "TOG_CON_MIN_TIME_EQ needs a TOG_PROB_MIN_TIME problem");
          if (!term) rows.push_back({ROW_MT_EQ, n - 1, (double)(m - 1), 0.0, 0.0, 0.0});
          break;
        case TOG_CON_USER: {
          if (!has_con) return fail(TOG_ERR_ARG, "TOG_CON_USER needs a user model plugin that defines con()");
          const int where = (int)D[2];
          if (con.count < 1 || con.count > PUSER) return fail(TOG_ERR_ARG, "user constraint: 1 <= p <= 16");
          if ((term && where != 0) || (!term && where != 1))
            for (int i = 0; i < con.count; i++)
              rows.push_back({D[1] != 0.0 ? ROW_USER_EQ : ROW_USER_INEQ, i, D[0], (double)con.count, 0.0, 0.0});
          break;
        }
        default:
          return fail(TOG_ERR_ARG, "unknown constraint type");
      }
    }
    cnt[k] = (int)rows.size() - off[k];
    if (cnt[k] > pcap) return fail(TOG_ERR_UNSUPPORTED, "too many constraint rows at one knot (PCAP)");
    // knots with the same rows share one copy (stage knots of one ConstraintSet): the table stays
    // small enough for the backward kernel to cache it in LDS
    for (int j = 0; j < k; j++) {
      if (cnt[j] != cnt[k] || cnt[k] == 0) continue;
      if (memcmp(&rows[off[j]], &rows[off[k]], sizeof(ConRow) * cnt[k]) == 0) {
        rows.resize(off[k]);
        off[k] = off[j];
        break;
      }
    }
  }
  return TOG_OK;
}

template <class T>
static int dalloc(tog_handle* h, T** p, size_t count) {
  void* v = nullptr;
  HIPCHECK(hipMalloc(&v, count * sizeof(T) > 0 ? count * sizeof(T) : 16));
  h->allocs.push_back(v);
  *p = (T*)v;
  return TOG_OK;
}
// release one dalloc'ed buffer before the handle is destroyed (null: nothing)
static void dfree(tog_handle* h, void* v) {
  if (!v) return;
  for (size_t i = 0; i < h->allocs.size(); i++)
    if (h->allocs[i] == v) {
      (void)hipFree(v);
      h->allocs.erase(h->allocs.begin() + (long)i);
      return;
    }
}

// =============================================================================================
// k_batch_stats: [n_active, Σ J, max c_max] (input to the cross-GPU RCCL all-reduce)
// =============================================================================================
static __global__ void __launch_bounds__(1024) k_batch_stats(const TrajState* __restrict__ st, long long B, double* out) {
  __shared__ double sa[1024], sj[1024], sc[1024];
  const int t = threadIdx.x;
  double a = 0.0, j = 0.0, c = 0.0;
  for (long long b = t; b < B; b += blockDim.x) {
    a += st[b].active ? 1.0 : 0.0;
    j += st[b].J;
    c = tog_jlmax(c, st[b].c_max);  // a NaN violation propagates (Julia max), never reads as feasible
  }
  sa[t] = a;
  sj[t] = j;
  sc[t] = c;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (t < w) {
      sa[t] += sa[t + w];
      sj[t] += sj[t + w];
      sc[t] = tog_jlmax(sc[t], sc[t + w]);
    }
    __syncthreads();
  }
  if (t == 0) {
    out[0] = sa[0];
    out[1] = sj[0];
    out[2] = sc[0];
  }
}


// the active trajectories, for the compacted launches of a tail step (order immaterial: every
// trajectory's computation is independent of its slot)
static __global__ void __launch_bounds__(256) k_list_active(const TrajState* __restrict__ st, long long B, int* list,
                                                            int* count) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool a = b < B && st[b].active;
  const unsigned long long mask = __ballot(a);
  if (mask == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)mask) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(mask));
  base = __shfl(base, leader);
  if (a) list[base + __popcll(mask & ((1ull << lane) - 1))] = (int)b;
}

__global__ void k_fill(double* p, size_t count, double v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) p[i] = v;
}

static void fill(tog_handle* h, double* p, size_t count, double v) {
  if (!count) return;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, h->stream, p, count, v);
}

__global__ void k_reset_state(TrajState* st, long long B, double mu0) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  TrajState s = {};
  s.active = 1;
  (void)mu0;
  st[b] = s;
}

extern "C" {

int32_t tog_version(void) { return TOG_ABI_VERSION; }
// (internal) the error path of tog_altro.cpp: records the message for tog_last_error
int32_t tog__fail(int32_t code, const char* msg) { return fail(code, msg); }

int32_t tog_model_load(const char* path, tog_model** out) {
  if (!path || !out) return fail(TOG_ERR_ARG, "null argument");
  *out = nullptr;
  void* so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!so) return fail(TOG_ERR_ARG, std::string("cannot load model plugin: ") + dlerror());
  auto fp = reinterpret_cast<long long (*)()>(dlsym(so, "tog_plugin_fingerprint"));
  auto ops = reinterpret_cast<const ModelOps* (*)()>(dlsym(so, "tog_plugin_ops"));
  auto opi = reinterpret_cast<const ModelOps* (*)()>(dlsym(so, "tog_plugin_ops_infeasible"));
  auto opm = reinterpret_cast<const ModelOps* (*)()>(dlsym(so, "tog_plugin_ops_min_time"));
  if (!fp || !ops || !opi || !opm) {
    dlclose(so);
    return fail(TOG_ERR_ARG, "not a libtog model plugin (TOG_PLUGIN symbols missing)");
  }
  if (fp() != plugin_fingerprint()) {
    dlclose(so);
    return fail(TOG_ERR_ARG, "model plugin was built against different libtog headers");
  }
  tog_model* m = new tog_model{so, ops(), opi(), opm()};
  *out = m;
  return TOG_OK;
}

int32_t tog_model_dims(const tog_model* model, int32_t* n, int32_t* m) {
  if (!model || !n || !m) return fail(TOG_ERR_ARG, "null argument");
  *n = model->ops->n;
  *m = model->ops->m;
  return TOG_OK;
}

int32_t tog_model_free(tog_model* model) {
  if (!model) return fail(TOG_ERR_ARG, "null model");
  dlclose(model->so);
  delete model;
  return TOG_OK;
}

// GenericCost plugins (tog_cost_plugin.hpp): the plugin's kernels evaluate ℓ / ℓf with their
// ForwardDiff-style gradient and Hessian; libtog stages host buffers and checks the results' launch
int32_t tog_generic_cost_load(const char* path, tog_generic_cost** out) {
  if (!path || !out) return fail(TOG_ERR_ARG, "null argument");
  *out = nullptr;
  void* so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!so) return fail(TOG_ERR_ARG, std::string("cannot load cost plugin: ") + dlerror());
  auto fp = reinterpret_cast<long long (*)()>(dlsym(so, "tog_cost_plugin_fingerprint"));
  auto dims = reinterpret_cast<int (*)(int*, int*)>(dlsym(so, "tog_cost_plugin_dims"));
  auto ex = reinterpret_cast<tog_generic_cost::expand_fn>(dlsym(so, "tog_cost_plugin_expand"));
  if (!fp || !dims || !ex) {
    dlclose(so);
    return fail(TOG_ERR_ARG, "not a libtog cost plugin (TOG_COST_PLUGIN symbols missing)");
  }
  if (fp() != cost_plugin_fingerprint()) {
    dlclose(so);
    return fail(TOG_ERR_ARG, "cost plugin was built against different libtog headers");
  }
  tog_generic_cost* c = new tog_generic_cost{so, 0, 0, ex};
  dims(&c->n, &c->m);
  *out = c;
  return TOG_OK;
}

int32_t tog_generic_cost_dims(const tog_generic_cost* cost, int32_t* n, int32_t* m) {
  if (!cost || !n || !m) return fail(TOG_ERR_ARG, "null argument");
  *n = cost->n;
  *m = cost->m;
  return TOG_OK;
}

int32_t tog_generic_cost_expand_device(const tog_generic_cost* cost, int32_t terminal, const double* X, const double* U,
                               int64_t count, double* J, double* Ex, double* Eu, double* Exx, double* Euu,
                               double* Eux, void* hip_stream) {
  if (!cost) return fail(TOG_ERR_ARG, "null cost");
  if (count < 0) return fail(TOG_ERR_ARG, "count < 0");
  if (count == 0) return TOG_OK;
  if (!X || !J || !Ex || !Exx || (!terminal && (!U || !Eu || !Euu || !Eux)))
    return fail(TOG_ERR_ARG, "null buffer");
  if (cost->ex(terminal ? 1 : 0, X, U, count, J, Ex, Eu, Exx, Euu, Eux, hip_stream) != 0)
    return fail(TOG_ERR_DEVICE, "cost plugin launch failed");
  return TOG_OK;
}

int32_t tog_generic_cost_expand(const tog_generic_cost* cost, int32_t device, int32_t terminal, const double* X, const double* U,
                        int64_t count, double* J, double* Ex, double* Eu, double* Exx, double* Euu, double* Eux) {
  if (!cost) return fail(TOG_ERR_ARG, "null cost");
  if (count < 0) return fail(TOG_ERR_ARG, "count < 0");
  if (count == 0) return TOG_OK;
  if (!X || !J || !Ex || !Exx || (!terminal && (!U || !Eu || !Euu || !Eux)))
    return fail(TOG_ERR_ARG, "null buffer");
  const size_t n = cost->n, m = terminal ? 0 : cost->m, c = (size_t)count;
  // one device block: X | U | J | Ex | Eu | Exx | Euu | Eux
  const size_t sz[8] = {n * c, m * c, c, n * c, m * c, n * n * c, m * m * c, m * n * c};
  size_t tot = 0;
  for (size_t v : sz) tot += v;
  HIPCHECK(hipSetDevice(device));
  double* d = nullptr;
  HIPCHECK(hipMalloc(&d, tot * sizeof(double)));
  double* p[8];
  size_t o = 0;
  for (int i = 0; i < 8; i++) {
    p[i] = d + o;
    o += sz[i];
  }
  hipError_t e = hipMemcpy(p[0], X, sz[0] * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess && m) e = hipMemcpy(p[1], U, sz[1] * sizeof(double), hipMemcpyHostToDevice);
  int rc = TOG_OK;
  if (e == hipSuccess) {
    rc = cost->ex(terminal ? 1 : 0, p[0], p[1], count, p[2], p[3], p[4], p[5], p[6], p[7], nullptr);
    if (rc != 0) rc = fail(TOG_ERR_DEVICE, "cost plugin launch failed");
  }
  if (e == hipSuccess && rc == TOG_OK) e = hipDeviceSynchronize();
  double* outs[6] = {J, Ex, Eu, Exx, Euu, Eux};
  for (int i = 0; i < 6 && e == hipSuccess && rc == TOG_OK; i++)
    if (sz[i + 2]) e = hipMemcpy(outs[i], p[i + 2], sz[i + 2] * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(TOG_ERR_DEVICE, std::string("tog_cost_expand: ") + hipGetErrorString(e));
  return rc;
}

int32_t tog_generic_cost_free(tog_generic_cost* cost) {
  if (!cost) return fail(TOG_ERR_ARG, "null cost");
  dlclose(cost->so);
  delete cost;
  return TOG_OK;
}

// dynamics_bias(state) of an RBD model at x = [q; v] (RigidBodyDynamics, used by
// hold_trajectory dynamics/kuka.jl:117-132): host evaluation of the same model code the kernels run.
int tog_dynamics_bias(int32_t model, const double* x, double* tau) {
  if (!x || !tau) return TOG_ERR_ARG;
  if (model != TOG_MODEL_KUKA) return TOG_ERR_UNSUPPORTED;
  double c[7], s[7];
  Kuka::bias<double>(tau, c, s, x, x + 7);
  return TOG_OK;
}

int32_t tog_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

void tog_default_options(tog_options* o) {
  memset(o, 0, sizeof(*o));
  o->cost_tolerance = 1e-4;
  o->gradient_norm_tolerance = 1e-5;
  o->iterations = 300;
  o->dJ_counter_limit = 10;
  o->square_root = 0;
  o->bp_reg_type = 0;
  o->gradient_type = 0;
  o->iterations_linesearch = 20;
  o->line_search_lower_bound = 1e-8;
  o->line_search_upper_bound = 10.0;
  o->bp_reg_increase_factor = 1.6;
  o->bp_reg_max = 1e8;
  o->bp_reg_min = 1e-8;
  o->bp_reg_fp = 10.0;
  o->max_cost_value = 1e8;
  o->max_state_value = 1e8;
  o->max_control_value = 1e8;
  o->al_cost_tolerance = 1e-4;
  o->al_cost_tolerance_intermediate = 1e-3;
  o->al_gradient_norm_tolerance = 1e-5;
  o->al_gradient_norm_tolerance_intermediate = 1e-5;
  o->constraint_tolerance = 1e-3;
  o->dual_min = -1e8;
  o->dual_max = 1e8;
  o->penalty_max = 1e8;
  o->penalty_initial = 1.0;
  o->penalty_scaling = 10.0;
  o->al_iterations = 30;
  o->kickout_max_penalty = 0;
}

const char* tog_last_error(void) { return g_err.c_str(); }


// =============================================================================================
// Multi-device handles (tog_create_multi): the batch is split into
// contiguous slices, one plain handle (device buffers + stream) per device. Trajectories are
// independent (§8(e)), so every step-level and solve-level call is the same call on each slice;
// launches are asynchronous per device, so the devices run concurrently. Host arrays are split
// and gathered along the batch axis, which is the outermost axis of every field.
// =============================================================================================
static bool is_multi(const tog_handle* h) { return h && !h->parts.empty(); }

// doubles per trajectory of a host-side field array (tog_get / tog_set layouts)
static size_t per_traj(const tog_handle* h, int field) {
  const size_t n = h->n, m = h->m, N = h->N, P1 = h->pmax > 0 ? h->pmax : 1;
  switch (field) {
    case TOG_FIELD_X: case TOG_FIELD_XBAR: return N * n;
    case TOG_FIELD_U: case TOG_FIELD_UBAR: case TOG_FIELD_D: return (N - 1) * m;
    case TOG_FIELD_K: return (N - 1) * m * n;
    case TOG_FIELD_A: return (N - 1) * n * n;
    case TOG_FIELD_B: return (N - 1) * n * m;
    case TOG_FIELD_S: return N * n * n;
    case TOG_FIELD_SX: return N * n;
    case TOG_FIELD_DV: case TOG_FIELD_RHO: return 2;
    case TOG_FIELD_LAMBDA: case TOG_FIELD_MU: case TOG_FIELD_C: return N * P1;
    case TOG_FIELD_X0: return n;
    case TOG_FIELD_STATS: return TOG_NSTATS;
    case TOG_FIELD_Q: return N * (size_t)h->nq;
    case TOG_FIELD_HIST_INNER: return 3 * (size_t)h->buf.hcap;
    case TOG_FIELD_HIST_OUTER: return 4 * (size_t)h->buf.ocap;
    case TOG_FIELD_HIST_COUNT: return 2;
  }
  return 0;
}

extern "C++" {
template <class F>
static int32_t each_part(tog_handle* h, F&& fn) {
  for (size_t i = 0; i < h->parts.size(); i++) {
    int32_t rc = fn(h->parts[i], (size_t)h->part_off[i]);
    if (rc) return rc;
  }
  return TOG_OK;
}
}  // extern "C++"

int32_t tog_destroy(tog_handle* h) {
  if (!h) return TOG_OK;
  if (is_multi(h)) {
    for (tog_handle* p : h->parts) tog_destroy(p);
    delete h;
    return TOG_OK;
  }
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : h->allocs) (void)hipFree(p);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  if (h->sp.st2) (void)hipStreamDestroy(h->sp.st2);
  if (h->sp.fork) (void)hipEventDestroy(h->sp.fork);
  if (h->sp.join) (void)hipEventDestroy(h->sp.join);
  for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->stats_ev) (void)hipEventDestroy(h->stats_ev);
  if (h->sync_ev) (void)hipEventDestroy(h->sync_ev);
  if (h->h_stats) (void)hipHostFree(h->h_stats);
  delete h;
  return TOG_OK;
}

// Body of tog_create after argument validation: every early return (HIPCHECK, allocation, build_rows)
// leaves the partially built handle to the caller, which destroys it (streams, events, allocations).
static int32_t create_single(tog_handle* h, const tog_problem_desc* d, const tog_options* opts,
                             const ModelOps* ops, int32_t device) {
  h->device = device;
  HIPCHECK(hipSetDevice(device));
  HIPCHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  h->own_stream = true;
  HIPCHECK(hipStreamCreateWithFlags(&h->sp.st2, hipStreamNonBlocking));
  HIPCHECK(hipEventCreateWithFlags(&h->sp.fork, hipEventDisableTiming));
  HIPCHECK(hipEventCreateWithFlags(&h->sp.join, hipEventDisableTiming));
  h->model = d->model;
  h->integ = d->integrator;
  h->n = d->n;
  h->m = d->m;
  h->N = d->N;
  h->B = d->batch;
  h->opts = *opts;
  h->ops = ops;
  const int n = h->n, m = h->m, N = h->N;
  h->nq = n + m + n * n + m * m + m * n;

  std::vector<ConRow> rows;
  std::vector<int> off, cnt;
  int rc = build_rows(d, ops->slack, ops->pcap, ops->has_con, rows, off, cnt);
  if (rc) return rc;
  h->nrows = (int)rows.size();
  h->pmax = 0;
  for (int k = 0; k < N; k++) h->pmax = cnt[k] > h->pmax ? cnt[k] : h->pmax;

  DevProblem& P = h->hostP;
  memset(&P, 0, sizeof(P));
  P.n = n;
  P.m = m;
  P.N = N;
  P.pmax = h->pmax;
  P.model = d->model;
  P.integ = d->integrator;
  P.nrows = h->nrows;
  P.B = h->B;
  P.dt = d->dt;
  // the stage cost(s): one for every knot, or a time-varying Objective's table (desc->stage_costs, rows
  // [Q; R; H; q; r; c]); the device table adds each knot's square-root factors cQ, cR (DevProblem::kc)
  const int nc_in = n * n + m * m + m * n + n + m + 1, kst = 2 * n * n + 2 * m * m + m * n + n + m + 1;
  const int nk = d->stage_costs ? N - 1 : 1;
  std::vector<double> kc((size_t)nk * kst, 0.0);
  for (int k = 0; k < nk; k++) {
    double* o = kc.data() + (size_t)k * kst;
    if (d->stage_costs) {
      memcpy(o, d->stage_costs + (size_t)k * nc_in, sizeof(double) * nc_in);
    } else {
      memcpy(o, d->Q, sizeof(double) * n * n);
      memcpy(o + n * n, d->R, sizeof(double) * m * m);
      memcpy(o + n * n + m * m, d->H, sizeof(double) * m * n);
      memcpy(o + n * n + m * m + m * n, d->q, sizeof(double) * n);
      memcpy(o + n * n + m * m + m * n + n, d->r, sizeof(double) * m);
      o[nc_in - 1] = d->c;
    }
  }
  auto kQ = [&](int k) { return kc.data() + (size_t)k * kst; };
  auto kR = [&](int k) { return kQ(k) + n * n; };
  auto kH = [&](int k) { return kR(k) + m * m; };
  auto kcQ = [&](int k) { return kQ(k) + nc_in; };
  auto kcR = [&](int k) { return kcQ(k) + n * n; };
  // P's own cost fields hold knot 0's (the shared one without a table)
  memcpy(P.Q, kQ(0), sizeof(double) * n * n);
  memcpy(P.R, kR(0), sizeof(double) * m * m);
  memcpy(P.H, kH(0), sizeof(double) * m * n);
  memcpy(P.q, kH(0) + m * n, sizeof(double) * n);
  memcpy(P.r, kH(0) + m * n + n, sizeof(double) * m);
  P.c = kQ(0)[nc_in - 1];
  memcpy(P.Qf, d->Qf, sizeof(double) * n * n);
  memcpy(P.qf, d->qf, sizeof(double) * n);
  P.cf = d->cf;
  {
    bool ok = host_chol_upper(P.Qf, n, P.cQf);
    for (int k = 0; k < nk; k++) {
      double Qdt[NMAX * NMAX], Rdt[MMAX * MMAX];
      for (int i = 0; i < n * n; i++) Qdt[i] = kQ(k)[i] * P.dt;
      for (int i = 0; i < m * m; i++) Rdt[i] = kR(k)[i] * P.dt;
      ok = host_chol_upper(Qdt, n, kcQ(k)) && host_chol_upper(Rdt, m, kcR(k)) && ok;
    }
    memcpy(P.cQ, kcQ(0), sizeof(double) * n * n);
    memcpy(P.cR, kcR(0), sizeof(double) * m * m);
    P.sqrt_ok = ok ? 1 : 0;
    bool diag = true;
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++)
        if (i != j && P.Qf[i + n * j] != 0.0) diag = false;
    for (int k = 0; k < nk; k++) {
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++)
          if (i != j && kQ(k)[i + n * j] != 0.0) diag = false;
      for (int j = 0; j < m; j++)
        for (int i = 0; i < m; i++)
          if (i != j && kR(k)[i + m * j] != 0.0) diag = false;
      for (int i = 0; i < m * n; i++)
        if (kH(k)[i] != 0.0) diag = false;
    }
    // 2: diagonal with every off-diagonal entry (and H, and the factors' off-diagonals) +0.0 and
    // dt > 0, so the kernels may use literal zeros for them and stay bit-identical
    bool pz = diag && P.dt > 0.0;
    auto offdiag_pz = [&](const double* A, int kk) {
      for (int j = 0; j < kk; j++)
        for (int i = 0; i < kk; i++)
          if (i != j && (A[i + kk * j] != 0.0 || std::signbit(A[i + kk * j]))) return false;
      return true;
    };
    if (pz) pz = offdiag_pz(P.Qf, n) && (!ok || offdiag_pz(P.cQf, n));
    for (int k = 0; pz && k < nk; k++) {
      pz = offdiag_pz(kQ(k), n) && offdiag_pz(kR(k), m);
      if (pz && ok) pz = offdiag_pz(kcQ(k), n) && offdiag_pz(kcR(k), m);
      for (int i = 0; pz && i < m * n; i++)
        if (std::signbit(kH(k)[i])) pz = false;
    }
    P.diag_cost = diag ? (pz ? 2 : 1) : 0;
    h->buf.cost_diag = P.diag_cost;
    if (opts->square_root && !ok) {
      return fail(TOG_ERR_ARG, "cost Hessians must be PD for the sqrt backward pass (objective.jl:70-94)");
    }
  }
  // packed std AL expansion records: the Q.xx entries a stage row can change (row_grad's state indices)
  {
    unsigned int pat[NMAX] = {0};
    for (const ConRow& r : rows) {
      unsigned int sx = 0;
      switch (r.type) {
        case ROW_XMAX: case ROW_XMIN: case ROW_GOAL: case ROW_MT_EQ: sx = 1u << r.idx; break;
        case ROW_UMAX: case ROW_UMIN: case ROW_USLACK: break;
        case ROW_CIRCLE: sx = 3u; break;
        case ROW_SPHERE: sx = 7u; break;
        default: sx = (1u << n) - 1u;  // user rows: dense
      }
      for (int c = 0; c < n; c++)
        if (sx >> c & 1u) pat[c] |= sx;
    }
    int off = 0;
    P.qpat_max = 0;
    for (int c = 0; c < n; c++) {
      P.qpat[c] = pat[c];
      P.qoff[c] = off;
      off += __builtin_popcount(pat[c]);
      P.qpat_max = std::max(P.qpat_max, __builtin_popcount(pat[c]));
    }
    P.qpat_n = off;
    // (the expansion's pattern loop: every column within QPK pattern rows; TOG_DENSE_RECORDS=1 runs the
    // general loop, for A/B checks)
    P.qpat_on = (P.qpat_max <= QPK && getenv("TOG_DENSE_RECORDS") == nullptr) ? 1 : 0;
  }
  P.kc = nullptr;
  P.kc_stride = kst;
  P.kc_pad = 0;
  if (d->stage_costs) {
    double* dkc = nullptr;
    if ((rc = dalloc(h, &dkc, kc.size()))) return rc;
    HIPCHECK(hipMemcpy(dkc, kc.data(), sizeof(double) * kc.size(), hipMemcpyHostToDevice));
    P.kc = dkc;
  }
  P.o = *opts;
  P.R_min_time = (d->flags & TOG_PROB_MIN_TIME) ? d->R_min_time : 0.0;
  const size_t B = (size_t)h->B, P1 = (size_t)(h->pmax > 0 ? h->pmax : 1);
  // rows with a state gradient per knot (every row type but the control bounds): the knots whose
  // square-root expansion changes Q.xx (expansion records, tog_bwd_team.hpp ne_of)
  std::vector<int> nxk(N, 0);
  for (int k = 0; k < N; k++)
    for (int r = 0; r < cnt[k]; r++) {
      const int t = rows[off[k] + r].type;
      if (t != ROW_UMAX && t != ROW_UMIN) nxk[k]++;
    }
  if ((rc = dalloc(h, &h->d_knot_off, N)) || (rc = dalloc(h, &h->d_knot_cnt, N)) ||
      (rc = dalloc(h, &h->d_knot_nx, N)) || (rc = dalloc(h, &h->d_rows, rows.size() + 1)) ||
      (rc = dalloc(h, &h->dP, 1)))
    return rc;
  HIPCHECK(hipMemcpy(h->d_knot_off, off.data(), sizeof(int) * N, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(h->d_knot_cnt, cnt.data(), sizeof(int) * N, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(h->d_knot_nx, nxk.data(), sizeof(int) * N, hipMemcpyHostToDevice));
  if (!rows.empty()) HIPCHECK(hipMemcpy(h->d_rows, rows.data(), sizeof(ConRow) * rows.size(), hipMemcpyHostToDevice));
  {
    // TOG_BWD=lds forces the one-wave-per-trajectory LDS backward kernel (A/B checks)
    const char* ev = getenv("TOG_BWD");
    const bool force_lds = ev && strcmp(ev, "lds") == 0;
    // (a time-varying Objective runs the team kernels' TV variants, which read knot k's cost from the table)
    h->bwd_team = (!force_lds && !ops->min_time &&
                   team_rows_fit(off.data(), cnt.data(), rows.data(), N, n, m, (int)rows.size()))
                      ? 1 : 0;
    for (int sq = 0; sq < 2; sq++) {
      h->buf.bwd_stride2[sq] = ops->team_stride(h->pmax, sq);
      h->buf.bwd_shmem2[sq] = (int)bwd_team_shmem(h->buf.bwd_stride2[sq], ops->team_tpw, (int)rows.size(), N);
      if (h->buf.bwd_shmem2[sq] > 64 * 1024) h->bwd_team = 0;
    }
  }
  // bulk k_ls_spec: a block's LDS copy of the row tables (TOG_SPEC_RT=global: the constant-space reads)
  h->buf.rows_lds = getenv("TOG_SPEC_RT") && strcmp(getenv("TOG_SPEC_RT"), "global") == 0
                        ? 0
                        : row_tables_bytes((int)rows.size(), N);
  // k_ls_spec_tail (tail rollouts staged through LDS): admissible up to SPEC_TAIL_PMAX rows per knot
  {  // k_ls_spec_tail2 (two waves): within 64 KB of LDS; TOG_NO_SPEC_TAIL2 keeps the one-wave kernel
    const size_t b2 = sizeof(double) * (size_t)spec_tail2_doubles(n, m, h->pmax);
    h->buf.spec_tail2_shmem =
        (h->pmax <= SPEC_TAIL_PMAX && b2 <= 64 * 1024 && !getenv("TOG_NO_SPEC_TAIL2")) ? (int)b2 : 0;
  }
  h->buf.spec_tail_shmem = (h->pmax <= SPEC_TAIL_PMAX && !getenv("TOG_NO_SPEC_TAIL"))
                               ? (int)(sizeof(double) * (spec_tail_tc(n, m) * spec_tail_rec(n, m, h->pmax) + 2 * h->pmax))
                               : 0;
  P.knot_off = h->d_knot_off;
  P.knot_cnt = h->d_knot_cnt;
  P.knot_nx = h->d_knot_nx;
  P.rows = h->d_rows;
  HIPCHECK(hipMemcpy(h->dP, &P, sizeof(P), hipMemcpyHostToDevice));

  DevBuffers& b = h->buf;
  b.tv = d->stage_costs ? 1 : 0;
  b.dense_stage_knots = 0;  // a stage knot with a state row (its square-root expansion changes Q.xx)
  for (int k = 0; k + 1 < N; k++)
    if (nxk[k] > 0) b.dense_stage_knots = 1;
  if ((rc = dalloc(h, &b.x0, B * n)) || (rc = dalloc(h, &b.X, B * N * n)) || (rc = dalloc(h, &b.U, B * (N - 1) * m)) ||
      (rc = dalloc(h, &b.Xb, B * N * n)) || (rc = dalloc(h, &b.Ub, B * (N - 1) * m)) ||
      (rc = dalloc(h, &b.AB, B * (N - 1) * n * (n + m))) || (rc = dalloc(h, &b.K, B * (N - 1) * m * n)) ||
      (rc = dalloc(h, &b.d, B * (N - 1) * m)) || (rc = dalloc(h, &b.lam, B * N * P1)) ||
      (rc = dalloc(h, &b.mu, B * N * P1)) || (rc = dalloc(h, &b.C, B * N * P1)) ||
      (rc = dalloc(h, &b.Qscr, B * N * h->nq)) || (rc = dalloc(h, &b.st, B)) ||
      (rc = dalloc(h, &h->d_scratch, B)) || (rc = dalloc(h, &h->d_scratch2, B)) ||
      (rc = dalloc(h, &h->d_iscratch, B)) || (rc = dalloc(h, &h->d_stats, 4)) ||
      (rc = dalloc(h, &h->d_act_list, B)) || (rc = dalloc(h, &h->d_act_count, 1)) ||
      (rc = dalloc(h, &b.lsJ, B * 64)) || (rc = dalloc(h, &b.lsok, B * 64)) ||
      (rc = dalloc(h, &b.ls_list, 2 * B)) || (rc = dalloc(h, &b.ls_count, LS_COUNT_SLOTS)))
    return rc;
  b.Sdbg = nullptr;
  b.sdbg = nullptr;
  b.E = nullptr;
  b.ls_done = b.ls_list + B;  // (the second half of ls_list; its offset is the full batch, never a
                              //  compacted launch's slot count)
  b.act_list = nullptr;  // set only in the launch view of a compacted tail step
  b.act_count = nullptr;
  b.hist_in = nullptr;  // tog_history_enable
  b.hist_out = nullptr;
  b.hcap = 0;
  b.ocap = 0;
  if (h->bwd_team) {  // expansion records of the team backward pass (k_expand_team)
    const size_t ne = (size_t)n + m + (size_t)m * m + (size_t)n * n;
    if ((rc = dalloc(h, &b.E, B * N * ne))) return rc;
  }
  b.nc = opts->iterations_linesearch + 1 < 64 ? opts->iterations_linesearch + 1 : 64;
  if (b.nc < 1) b.nc = 1;
  b.nknots = N;
  b.jws = nullptr;
  b.jac_chain = (getenv("TOG_KUKA_JAC") && strcmp(getenv("TOG_KUKA_JAC"), "dual") == 0) ? 0 : 1;
  // staged RK3 Jacobian (the RBD model): the stage state of every (knot, partial) lane
  if (ops->jws_per_lane > 0 && d->integrator == TOG_RK3 && !getenv("TOG_JAC_UNSTAGED")) {
    const size_t lanes = B * (size_t)(N - 1) * (size_t)(ops->n + ops->m - ops->slack);
    if ((rc = dalloc(h, &b.jws, lanes * (size_t)ops->jws_per_lane))) return rc;
  }
  b.ncp = (b.nc + 7) & ~7;
  b.tail = 0;
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) cus = 0;
    b.simds = getenv("TOG_BWD_W2") ? 0 : 4 * cus;  // (TOG_BWD_W2: the 2-wave variant at every batch size, A/B)
  }
  b.ls_pend_ok = getenv("TOG_LS_NOPEND") ? 0 : 1;
  b.ls_first = LS_FIRST;
  b.cand = nullptr;
  b.ls_fb = nullptr;
  // candidate-copy line search when every trial fits the speculative window (TOG_LS=replay: the
  // replaying k_ls_commit path, for A/B checks)
  {
    const char* ev = getenv("TOG_LS");
    const bool replay = ev && strcmp(ev, "replay") == 0;
    if (!replay && opts->iterations_linesearch + 1 <= 64) {
      if ((rc = dalloc(h, &b.cand, B * (size_t)b.ncp * N * 4 * ((n + m + 3) / 4))) || (rc = dalloc(h, &b.ls_win, B)) ||
          (rc = dalloc(h, &b.ls_Jw, B)) || (rc = dalloc(h, &b.gk, B * N)) || (rc = dalloc(h, &b.ls_fb, B)))
        return rc;
    }
  }
  // reference constructor state: X = NaN, U = 0, K = d = 0, λ = 0, μ = opts.penalty_initial,
  // ρ = dρ = 0 (ilqr_solver.jl:118-144, augmented_lagrangian_solver.jl:143-169)
  fill(h, b.x0, B * n, 0.0);
  fill(h, b.X, B * N * n, NAN);
  fill(h, b.U, B * (N - 1) * m, 0.0);
  fill(h, b.Xb, B * N * n, 0.0);
  fill(h, b.Ub, B * (N - 1) * m, 0.0);
  fill(h, b.AB, B * (N - 1) * n * (n + m), 0.0);
  fill(h, b.K, B * (N - 1) * m * n, 0.0);
  fill(h, b.d, B * (N - 1) * m, 0.0);
  fill(h, b.lam, B * N * P1, 0.0);
  fill(h, b.mu, B * N * P1, h->opts.penalty_initial);  // init_constraint_trajectories
  fill(h, b.C, B * N * P1, 0.0);
  hipLaunchKernelGGL(k_reset_state, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, h->stream, b.st, (long long)B, h->opts.penalty_initial);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}

int32_t tog_create(const tog_problem_desc* d, const tog_options* opts, int32_t device, tog_handle** out) {
  if (!d || !opts || !out) return fail(TOG_ERR_ARG, "null argument");
  *out = nullptr;
  if (d->flags & ~(int32_t)(TOG_PROB_INFEASIBLE | TOG_PROB_MIN_TIME)) return fail(TOG_ERR_ARG, "unknown problem flags");
  if (opts->gradient_type < 0 || opts->gradient_type > 3)
    return fail(TOG_ERR_ARG, "gradient_type must be 0 (:todorov), 1 (:feedforward), 2 (:ℓ2) or 3 (:ℓinf)");
  if ((d->flags & TOG_PROB_MIN_TIME) && opts->square_root)
    return fail(TOG_ERR_UNSUPPORTED, "minimum time: MinTimeCost has no square-root expansion (std backward pass)");
  const ModelOps* ops = ops_for(d->model, (d->flags & TOG_PROB_INFEASIBLE) != 0, (d->flags & TOG_PROB_MIN_TIME) != 0,
                                d->user_model, d->integrator);
  if (!ops) return fail(TOG_ERR_UNSUPPORTED, "model not built");
  if (d->n != ops->n || d->m != ops->m) return fail(TOG_ERR_ARG, "n, m do not match the model");
  if (d->N < 2) return fail(TOG_ERR_ARG, "N must be >= 2");
  if (d->batch < 1) return fail(TOG_ERR_ARG, "batch must be >= 1");
  if (!(d->dt > 0)) return fail(TOG_ERR_ARG, "dt must be strictly positive");  // src/problem.jl:66-68
  if (d->integrator != TOG_RK3 && d->integrator != TOG_RK4 && d->integrator != TOG_MIDPOINT &&
      d->integrator != TOG_RK3_IMPLICIT && d->integrator != TOG_MIDPOINT_IMPLICIT)
    return fail(TOG_ERR_UNSUPPORTED, "integrator");
  if ((d->integrator == TOG_RK3_IMPLICIT || d->integrator == TOG_MIDPOINT_IMPLICIT) && !ops->implicit)
    return fail(TOG_ERR_UNSUPPORTED, "implicit integrators are built for models with n <= 4 and the quadrotor (no slack controls)");
  int ndev = tog_device_count();
  if (device < 0 || device >= ndev) return fail(TOG_ERR_DEVICE, "no such HIP device");
  tog_handle* h = new tog_handle();
  const int32_t rc = create_single(h, d, opts, ops, device);
  if (rc) {
    tog_destroy(h);
    return rc;
  }
  *out = h;
  return TOG_OK;
}

int32_t tog_create_multi(const tog_problem_desc* d, const tog_options* opts, const int32_t* devices,
                         int32_t ndev, tog_handle** out) {
  if (!d || !opts || !devices || !out) return fail(TOG_ERR_ARG, "null argument");
  *out = nullptr;
  if (ndev < 1) return fail(TOG_ERR_ARG, "ndev must be >= 1");
  if (d->batch < ndev) return fail(TOG_ERR_ARG, "batch must be >= ndev");
  tog_handle* h = new tog_handle();
  const long long B = d->batch, base = B / ndev, rem = B % ndev;
  long long off = 0;
  for (int i = 0; i < ndev; i++) {
    tog_problem_desc di = *d;
    di.batch = base + (i < rem ? 1 : 0);
    tog_handle* p = nullptr;
    int32_t rc = tog_create(&di, opts, devices[i], &p);
    if (rc) {
      const std::string msg = g_err;
      tog_destroy(h);
      return fail(rc, "device " + std::to_string(devices[i]) + ": " + msg);
    }
    h->parts.push_back(p);
    h->part_off.push_back(off);
    off += di.batch;
  }
  h->part_off.push_back(off);
  tog_handle* p0 = h->parts[0];
  h->device = p0->device;
  h->model = p0->model;
  h->integ = p0->integ;
  h->n = p0->n;
  h->m = p0->m;
  h->N = p0->N;
  h->pmax = p0->pmax;
  h->nq = p0->nq;
  h->B = B;
  h->opts = *opts;
  *out = h;
  return TOG_OK;
}

int32_t tog_set_stream(tog_handle* h, void* s) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return fail(TOG_ERR_UNSUPPORTED, "tog_set_stream: a multi-device handle owns one stream per device");
  HIPCHECK(hipSetDevice(h->device));
  HIPCHECK(hipStreamSynchronize(h->stream));
  if (h->own_stream) HIPCHECK(hipStreamDestroy(h->stream));
  if (s) {
    h->stream = (hipStream_t)s;
    h->own_stream = false;
  } else {
    HIPCHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->own_stream = true;
  }
  return TOG_OK;
}

int32_t tog_synchronize(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_synchronize(p); });
  HIPCHECK(hipSetDevice(h->device));
  if (!h->sync_ev) HIPCHECK(hipEventCreateWithFlags(&h->sync_ev, hipEventDisableTiming));
  HIPCHECK(hipEventRecord(h->sync_ev, h->stream));
  return wait_event(h->sync_ev, "tog_synchronize");
}

int32_t tog_dims(tog_handle* h, int64_t* o) {
  if (!h || !o) return fail(TOG_ERR_ARG, "null argument");
  o[0] = h->n;
  o[1] = h->m;
  o[2] = h->N;
  o[3] = h->B;
  o[4] = h->pmax;
  o[5] = h->mode;
  return TOG_OK;
}

int32_t tog_history_enable(tog_handle* h, int32_t capacity) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (capacity < 0) return fail(TOG_ERR_ARG, "capacity must be >= 0");
  const int ocap = h->opts.al_iterations + 1 > 1 ? h->opts.al_iterations + 1 : 1;
  if (is_multi(h)) {
    int32_t rc = each_part(h, [&](tog_handle* p, size_t) { return tog_history_enable(p, capacity); });
    h->buf.hcap = capacity;
    h->buf.ocap = capacity > 0 ? ocap : 0;
    return rc;
  }
  HIPCHECK(hipSetDevice(h->device));
  HIPCHECK(hipStreamSynchronize(h->stream));
  DevBuffers& b = h->buf;
  if (capacity == 0) {  // off (the buffers stay allocated until the handle is destroyed)
    b.hist_in = nullptr;
    b.hist_out = nullptr;
    b.hcap = b.ocap = 0;
    return TOG_OK;
  }
  if (capacity > h->hist_cap_alloc || ocap > h->hist_ocap_alloc || !h->hist_in_alloc) {  // grow (old ones released)
    int rc;
    dfree(h, h->hist_in_alloc);
    dfree(h, h->hist_out_alloc);
    h->hist_in_alloc = h->hist_out_alloc = nullptr;
    h->hist_cap_alloc = h->hist_ocap_alloc = 0;
    if ((rc = dalloc(h, &h->hist_in_alloc, (size_t)h->B * 3 * capacity)) ||
        (rc = dalloc(h, &h->hist_out_alloc, (size_t)h->B * 4 * ocap)))
      return rc;
    h->hist_cap_alloc = capacity;
    h->hist_ocap_alloc = ocap;
  }
  b.hist_in = h->hist_in_alloc;  // a smaller capacity reuses the allocation (records are strided by hcap)
  b.hist_out = h->hist_out_alloc;
  b.hcap = capacity;
  b.ocap = ocap;
  return TOG_OK;
}

static size_t field_count(tog_handle* h, int field, double** dptr) {
  const size_t B = h->B, n = h->n, m = h->m, N = h->N, P1 = h->pmax > 0 ? h->pmax : 1;
  DevBuffers& b = h->buf;
  switch (field) {
    case TOG_FIELD_X: *dptr = b.X; return B * N * n;
    case TOG_FIELD_U: *dptr = b.U; return B * (N - 1) * m;
    case TOG_FIELD_XBAR: *dptr = b.Xb; return B * N * n;
    case TOG_FIELD_UBAR: *dptr = b.Ub; return B * (N - 1) * m;
    case TOG_FIELD_K: *dptr = b.K; return B * (N - 1) * m * n;
    case TOG_FIELD_D: *dptr = b.d; return B * (N - 1) * m;
    case TOG_FIELD_LAMBDA: *dptr = b.lam; return B * N * P1;
    case TOG_FIELD_MU: *dptr = b.mu; return B * N * P1;
    case TOG_FIELD_C: *dptr = b.C; return B * N * P1;
    case TOG_FIELD_X0: *dptr = b.x0; return B * n;
    case TOG_FIELD_S: *dptr = b.Sdbg; return B * N * n * n;
    case TOG_FIELD_SX: *dptr = b.sdbg; return B * N * n;
    case TOG_FIELD_Q: *dptr = b.Qscr; return B * N * (size_t)h->nq;
    case TOG_FIELD_HIST_INNER: *dptr = b.hist_in; return B * 3 * (size_t)b.hcap;
    case TOG_FIELD_HIST_OUTER: *dptr = b.hist_out; return B * 4 * (size_t)b.ocap;
  }
  *dptr = nullptr;
  return 0;
}

int32_t tog_get_device_ptr(tog_handle* h, int32_t field, void** dptr) {
  if (!h || !dptr) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) return fail(TOG_ERR_UNSUPPORTED, "device pointers are per device: use the per-device handles");
  double* p = nullptr;
  field_count(h, field, &p);
  if (field == TOG_FIELD_STATS) {
    *dptr = h->buf.st;
    return TOG_OK;
  }
  if (!p) return fail(TOG_ERR_ARG, "field has no device buffer");
  *dptr = p;
  return TOG_OK;
}

static int get_states(tog_handle* h, std::vector<TrajState>& st) {
  st.resize(h->B);
  HIPCHECK(hipMemcpyAsync(st.data(), h->buf.st, sizeof(TrajState) * h->B, hipMemcpyDeviceToHost, h->stream));
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}
static int put_states(tog_handle* h, const std::vector<TrajState>& st) {
  HIPCHECK(hipMemcpyAsync(h->buf.st, st.data(), sizeof(TrajState) * h->B, hipMemcpyHostToDevice, h->stream));
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}

int32_t tog_get(tog_handle* h, int32_t field, double* out) {
  if (!h || !out) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    const size_t w = per_traj(h, field);
    if (!w) return fail(TOG_ERR_ARG, "unknown field");
    return each_part(h, [&](tog_handle* p, size_t o) { return tog_get(p, field, out + o * w); });
  }
  HIPCHECK(hipSetDevice(h->device));
  const size_t n = h->n, m = h->m, N = h->N, B = h->B;
  DevBuffers& b = h->buf;
  if (field == TOG_FIELD_A || field == TOG_FIELD_B) {
    // strided extraction of ∇F[k].xx / .xu from the [A|B] blocks
    const size_t L = n + m, cols = (field == TOG_FIELD_A) ? n : m, c0 = (field == TOG_FIELD_A) ? 0 : n;
    HIPCHECK(hipMemcpy2DAsync(out, sizeof(double) * n * cols, b.AB + c0 * n, sizeof(double) * n * L,
                              sizeof(double) * n * cols, B * (N - 1), hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    return TOG_OK;
  }
  if (field == TOG_FIELD_HIST_COUNT) {
    std::vector<TrajState> st;
    int rc = get_states(h, st);
    if (rc) return rc;
    for (size_t i = 0; i < B; i++) {
      out[2 * i] = st[i].hn_in;
      out[2 * i + 1] = st[i].hn_out;
    }
    return TOG_OK;
  }
  if ((field == TOG_FIELD_HIST_INNER || field == TOG_FIELD_HIST_OUTER) && !b.hist_in)
    return fail(TOG_ERR_ARG, "iteration histories are off (tog_history_enable)");
  if (field == TOG_FIELD_STATS || field == TOG_FIELD_DV || field == TOG_FIELD_RHO) {
    std::vector<TrajState> st;
    int rc = get_states(h, st);
    if (rc) return rc;
    for (size_t i = 0; i < B; i++) {
      const TrajState& s = st[i];
      if (field == TOG_FIELD_DV) {
        out[2 * i] = s.dV0;
        out[2 * i + 1] = s.dV1;
      } else if (field == TOG_FIELD_RHO) {
        out[2 * i] = s.rho;
        out[2 * i + 1] = s.drho;
      } else {
        double* o = out + i * TOG_NSTATS;
        for (int j = 0; j < TOG_NSTATS; j++) o[j] = 0.0;
        o[TOG_STAT_J] = s.J;
        o[TOG_STAT_DJ] = s.dJ;
        o[TOG_STAT_GRADIENT] = s.grad;
        o[TOG_STAT_ITERATIONS] = s.iters;
        o[TOG_STAT_ZERO_COUNT] = s.zero_cnt;
        o[TOG_STAT_ALPHA] = s.alpha;
        o[TOG_STAT_Z] = s.z;
        o[TOG_STAT_C_MAX] = s.c_max;
        o[TOG_STAT_AL_ITER] = s.al_iter;
        o[TOG_STAT_TOTAL_STEPS] = s.total_steps;
        o[TOG_STAT_LS_TRIALS] = s.ls_trials;
        o[TOG_STAT_BP_RESTARTS] = s.bp_restarts;
        o[TOG_STAT_FLAGS] = s.flags | (s.active ? TOG_TRAJ_ACTIVE : 0);
        o[TOG_STAT_PENALTY_MAX] = s.mu_max;
      }
    }
    return TOG_OK;
  }
  double* p = nullptr;
  size_t count = field_count(h, field, &p);
  if (!p) return fail(TOG_ERR_ARG, "field not available (S/SX need a backward pass with TOG_BP_STORE_S)");
  HIPCHECK(hipMemcpyAsync(out, p, sizeof(double) * count, hipMemcpyDeviceToHost, h->stream));
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}

int32_t tog_set(tog_handle* h, int32_t field, const double* in) {
  if (!h || !in) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    const size_t w = per_traj(h, field);
    if (!w) return fail(TOG_ERR_ARG, "unknown field");
    return each_part(h, [&](tog_handle* p, size_t o) { return tog_set(p, field, in + o * w); });
  }
  HIPCHECK(hipSetDevice(h->device));
  if (field == TOG_FIELD_DV || field == TOG_FIELD_RHO) {
    std::vector<TrajState> st;
    int rc = get_states(h, st);
    if (rc) return rc;
    for (size_t i = 0; i < (size_t)h->B; i++) {
      if (field == TOG_FIELD_DV) {
        st[i].dV0 = in[2 * i];
        st[i].dV1 = in[2 * i + 1];
      } else {
        st[i].rho = in[2 * i];
        st[i].drho = in[2 * i + 1];
      }
    }
    return put_states(h, st);
  }
  if (field == TOG_FIELD_A || field == TOG_FIELD_B || field == TOG_FIELD_STATS || field == TOG_FIELD_HIST_INNER ||
      field == TOG_FIELD_HIST_OUTER || field == TOG_FIELD_HIST_COUNT)
    return fail(TOG_ERR_ARG, "field is read-only");
  double* p = nullptr;
  size_t count = field_count(h, field, &p);
  if (!p) return fail(TOG_ERR_ARG, "field not settable");
  HIPCHECK(hipMemcpyAsync(p, in, sizeof(double) * count, hipMemcpyHostToDevice, h->stream));
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}

int32_t tog_set_state(tog_handle* h, const double* x0, const double* U, const double* X) {
  if (!h || !x0 || !U) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    const size_t n = h->n, m = h->m, N = h->N;
    return each_part(h, [&](tog_handle* p, size_t o) {
      return tog_set_state(p, x0 + o * n, U + o * (N - 1) * m, X ? X + o * N * n : nullptr);
    });
  }
  HIPCHECK(hipSetDevice(h->device));
  h->last_active = -1.0;  // every trajectory is active again
  const size_t n = h->n, m = h->m, N = h->N, B = h->B;
  HIPCHECK(hipMemcpyAsync(h->buf.x0, x0, sizeof(double) * B * n, hipMemcpyHostToDevice, h->stream));
  HIPCHECK(hipMemcpyAsync(h->buf.U, U, sizeof(double) * B * (N - 1) * m, hipMemcpyHostToDevice, h->stream));
  if (X)
    HIPCHECK(hipMemcpyAsync(h->buf.X, X, sizeof(double) * B * N * n, hipMemcpyHostToDevice, h->stream));
  else
    fill(h, h->buf.X, B * N * n, NAN);
  hipLaunchKernelGGL(k_reset_state, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, h->stream, h->buf.st, (long long)B,
                     1.0);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(h->stream));
  return TOG_OK;
}

// ------------------------------------------------------------------------------ step level
int32_t tog_rollout_open_loop(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_rollout_open_loop(p); });
  HIPCHECK(hipSetDevice(h->device));
  h->ops->rollout_open(h->dP, h->buf, h->B, h->integ, h->stream);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_slack_controls(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_slack_controls(p); });
  if (!h->ops->slack) return fail(TOG_ERR_ARG, "slack_controls needs a TOG_PROB_INFEASIBLE handle");
  if (h->ops->min_time)
    return fail(TOG_ERR_ARG, "slack_controls runs on the infeasible problem (infeasible.jl:63-80), before "
                             "minimum_time_problem appends h");
  HIPCHECK(hipSetDevice(h->device));
  h->ops->slack_controls(h->dP, h->buf, h->B, h->integ, h->stream);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_jacobians(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_jacobians(p); });
  HIPCHECK(hipSetDevice(h->device));
  h->ops->jacobian(h->dP, h->buf, h->B, h->N, h->integ, h->stream);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_update_constraints(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_update_constraints(p); });
  HIPCHECK(hipSetDevice(h->device));
  h->ops->update_constraints(h->dP, h->buf, h->B, h->stream);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_cost(tog_handle* h, int32_t al, double* J_out) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h))
    return each_part(h, [&](tog_handle* p, size_t o) { return tog_cost(p, al, J_out ? J_out + o : nullptr); });
  HIPCHECK(hipSetDevice(h->device));
  h->ops->cost(h->dP, h->buf, h->B, al, 0, h->d_scratch, h->stream);
  HIPCHECK(hipGetLastError());
  if (J_out) {
    HIPCHECK(hipMemcpyAsync(J_out, h->d_scratch, sizeof(double) * h->B, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
  }
  return TOG_OK;
}

int32_t tog_cost_expansion(tog_handle* h, int32_t sq, int32_t al) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [&](tog_handle* p, size_t) { return tog_cost_expansion(p, sq, al); });
  HIPCHECK(hipSetDevice(h->device));
  if (h->ops->min_time) return fail(TOG_ERR_UNSUPPORTED, "tog_cost_expansion: minimum-time problems (fused in the backward pass)");
  HIPCHECK(hipMemsetAsync(h->d_iscratch, 0, sizeof(int) * h->B, h->stream));
  h->ops->cost_expansion(h->dP, h->buf, h->B, h->N, sq, al, h->d_iscratch, h->stream);
  HIPCHECK(hipGetLastError());
  std::vector<int> f(h->B);
  HIPCHECK(hipMemcpyAsync(f.data(), h->d_iscratch, sizeof(int) * h->B, hipMemcpyDeviceToHost, h->stream));
  HIPCHECK(hipStreamSynchronize(h->stream));
  for (int v : f)
    if (v) return fail(TOG_ERR_ARG, "PosDefException: cost Hessian not positive definite (objective.jl:70-86)");
  return TOG_OK;
}

int32_t tog_solve_ilqr(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  return tog_solve(h, TOG_MODE_ILQR, 0);
}

int32_t tog_solve_al(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  return tog_solve(h, TOG_MODE_AL, 0);
}

// Batch steps a solve to completion may take: the iteration budget (iterations, x al_iterations for AL,
// + 1 for the final check) times the line-search rounds one iteration can spread over when its trials
// are run LS_FIRST per batch step (pending mode, ceil(nc / LS_FIRST) rounds). A pending step does not
// advance a trajectory's iteration counter, so a budget of one iteration per step would stop hard
// trajectories before the device-side counters flag them MAX_ITERS. Steps beyond need are free:
// tog_solve stops as soon as no trajectory is active.
int32_t tog_solve_budget(tog_handle* h, int32_t mode) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  const tog_options& o = h->opts;
  long long it = (long long)(o.iterations > 0 ? o.iterations : 0);
  if (mode == TOG_MODE_AL) it *= (o.al_iterations > 0 ? o.al_iterations : 0);
  const int nc = std::max(1, std::min(o.iterations_linesearch + 1, 64));
  const long long rounds = getenv("TOG_LS_NOPEND") ? 1 : (nc + LS_FIRST - 1) / LS_FIRST;
  const long long s = (it + 1) * rounds;
  return (int32_t)std::min<long long>(s, INT32_MAX);
}

int32_t tog_backward_pass(tog_handle* h, int32_t sq, int32_t al, int32_t flags, double* dV_out) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h))
    return each_part(h, [&](tog_handle* p, size_t o) {
      return tog_backward_pass(p, sq, al, flags, dV_out ? dV_out + 2 * o : nullptr);
    });
  HIPCHECK(hipSetDevice(h->device));
  if (sq && !h->hostP.sqrt_ok) return fail(TOG_ERR_ARG, "cost Hessians must be PD for the sqrt backward pass");
  if ((flags & TOG_BP_STORE_S) && !h->buf.Sdbg) {
    int rc;
    const size_t B = h->B, n = h->n, N = h->N;
    if ((rc = dalloc(h, &h->buf.Sdbg, B * N * n * n)) || (rc = dalloc(h, &h->buf.sdbg, B * N * n))) return rc;
  }
  if (h->bwd_team) h->ops->expand(h->dP, h->buf, h->B, h->N, h->pmax, sq, al, h->stream);
  h->ops->backward(h->dP, h->buf, h->B, sq, al, flags, h->bwd_team, h->stream);
  HIPCHECK(hipGetLastError());
  if (dV_out) return tog_get(h, TOG_FIELD_DV, dV_out);
  return TOG_OK;
}

int32_t tog_forward_pass(tog_handle* h, int32_t al, const double* J_prev, double* J_out) {
  if (!h || !J_prev) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h))
    return each_part(h, [&](tog_handle* p, size_t o) {
      return tog_forward_pass(p, al, J_prev + o, J_out ? J_out + o : nullptr);
    });
  HIPCHECK(hipSetDevice(h->device));
  HIPCHECK(hipMemcpyAsync(h->d_scratch, J_prev, sizeof(double) * h->B, hipMemcpyHostToDevice, h->stream));
  h->ops->forward(h->dP, h->buf, h->B, h->integ, al ? TOG_MODE_AL : TOG_MODE_ILQR, 0, h->d_scratch, h->d_scratch2,
                  h->stream, nullptr);
  HIPCHECK(hipGetLastError());
  if (J_out) {
    HIPCHECK(hipMemcpyAsync(J_out, h->d_scratch2, sizeof(double) * h->B, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
  }
  return TOG_OK;
}

int32_t tog_rollout(tog_handle* h, double alpha, int32_t* ok_out) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h))
    return each_part(h, [&](tog_handle* p, size_t o) { return tog_rollout(p, alpha, ok_out ? ok_out + o : nullptr); });
  HIPCHECK(hipSetDevice(h->device));
  h->ops->rollout(h->dP, h->buf, h->B, h->integ, alpha, h->d_iscratch, h->stream);
  HIPCHECK(hipGetLastError());
  if (ok_out) {
    HIPCHECK(hipMemcpyAsync(ok_out, h->d_iscratch, sizeof(int) * h->B, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
  }
  return TOG_OK;
}

// ------------------------------------------------------------------------------ solve level
int32_t tog_solve_init(tog_handle* h, int32_t mode) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) {
    h->mode = mode;
    return each_part(h, [&](tog_handle* p, size_t) { return tog_solve_init(p, mode); });
  }
  if (mode != TOG_MODE_ILQR && mode != TOG_MODE_AL) return fail(TOG_ERR_ARG, "mode");
  HIPCHECK(hipSetDevice(h->device));
  h->mode = mode;
  h->last_active = -1.0;
  h->stats_pending = false;  // a check left open by a failed solve is abandoned (its readback is never read)
  h->ops->init(h->dP, h->buf, h->B, h->integ, mode, h->stream);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_solve_step(tog_handle* h, int32_t nsteps) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [&](tog_handle* p, size_t) { return tog_solve_step(p, nsteps); });
  HIPCHECK(hipSetDevice(h->device));
  const int al = (h->mode == TOG_MODE_AL);
  // few trajectories (a small batch, or the convergence tail as of the last host readback of n_active):
  // every trial in one speculative round, so the forward pass is one rollout chain and every step
  // completes an iteration of every active trajectory. Otherwise rounds of LS_FIRST trials, an
  // undecided line search continuing in the next step (pending mode).
  const double few = 65536.0 / h->buf.nc;
  h->buf.ls_first = ((double)h->B <= few || (h->last_active >= 0.0 && h->last_active <= few)) ? h->buf.nc : LS_FIRST;
  // convergence tail (or a small batch): the latency-sized backward kernels (k_bwd_team WPE = 1)
  h->buf.tail = ((double)h->B <= TAIL_ACTIVE || (h->last_active >= 0.0 && h->last_active <= TAIL_ACTIVE)) ? 1 : 0;
  // In the tail the kernels launch over the active trajectories only: k_list_active lists them once per
  // call (trajectories only ever finish during a solve, so the list stays a superset of the active set
  // for the call's steps, and every kernel still checks `active`), and each launch covers
  // ceil(last n_active readback) slots instead of the whole batch (traj_of_slot, tog_kernels.hpp).
  DevBuffers Bt = h->buf;
  long long Bl = h->B;
  if (h->buf.tail && h->last_active >= 0.0 && h->last_active < (double)h->B && !getenv("TOG_NO_COMPACT")) {
    if (h->last_active == 0.0) return TOG_OK;  // nothing left to step
    Bl = (long long)ceil(h->last_active);
    HIPCHECK(hipMemsetAsync(h->d_act_count, 0, sizeof(int), h->stream));
    hipLaunchKernelGGL(k_list_active, dim3((unsigned)((h->B + 255) / 256)), dim3(256), 0, h->stream, h->buf.st,
                       (long long)h->B, h->d_act_list, h->d_act_count);
    Bt.act_list = h->d_act_list;
    Bt.act_count = h->d_act_count;
  }
  for (int i = 0; i < nsteps; i++) {
    timed(h, TOG_KERNEL_JACOBIAN, [&] { h->ops->jacobian(h->dP, Bt, Bl, h->N, h->integ, h->stream); });
    if (h->bwd_team)
      timed(h, TOG_KERNEL_EXPANSION, [&] {
        h->ops->expand(h->dP, Bt, Bl, h->N, h->pmax, h->opts.square_root, al, h->stream);
      });
    timed(h, TOG_KERNEL_BACKWARD,
          [&] { h->ops->backward(h->dP, Bt, Bl, h->opts.square_root, al, 0, h->bwd_team, h->stream); });
    timed(h, TOG_KERNEL_FORWARD,
          [&] {
            h->ops->forward(h->dP, Bt, Bl, h->integ, h->mode, 1, nullptr, nullptr, h->stream,
                            getenv("TOG_NO_OVERLAP") ? nullptr : &h->sp);
          });
  }
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_batch_stats_device(tog_handle* h, void* dptr3) {
  if (!h || !dptr3) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) return fail(TOG_ERR_UNSUPPORTED, "device pointers are per device: use tog_batch_stats");
  HIPCHECK(hipSetDevice(h->device));
  hipLaunchKernelGGL(k_batch_stats, dim3(1), dim3(1024), 0, h->stream, h->buf.st, (long long)h->B, (double*)dptr3);
  HIPCHECK(hipGetLastError());
  return TOG_OK;
}

int32_t tog_batch_stats(tog_handle* h, double* out3) {
  if (!h || !out3) return fail(TOG_ERR_ARG, "null argument");
  // (a multi-device handle queues every device's reduction before it gathers: _begin / _end fan out)
  int32_t rc = tog_batch_stats_begin(h);
  return rc ? rc : tog_batch_stats_end(h, out3);
}

int32_t tog_batch_stats_begin(tog_handle* h) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [](tog_handle* p, size_t) { return tog_batch_stats_begin(p); });
  HIPCHECK(hipSetDevice(h->device));
  if (h->stats_pending) return fail(TOG_ERR_ARG, "tog_batch_stats_begin: the previous check was not ended");
  if (!h->h_stats) HIPCHECK(hipHostMalloc((void**)&h->h_stats, sizeof(double) * 4, hipHostMallocDefault));
  if (!h->stats_ev) HIPCHECK(hipEventCreateWithFlags(&h->stats_ev, hipEventDisableTiming));
  int rc = tog_batch_stats_device(h, h->d_stats);
  if (rc) return rc;
  HIPCHECK(hipMemcpyAsync(h->h_stats, h->d_stats, sizeof(double) * 3, hipMemcpyDeviceToHost, h->stream));
  HIPCHECK(hipEventRecord(h->stats_ev, h->stream));
  h->stats_pending = true;
  return TOG_OK;
}

int32_t tog_batch_stats_end(tog_handle* h, double* out3) {
  if (!h || !out3) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    double acc[3] = {0.0, 0.0, 0.0};
    for (tog_handle* p : h->parts) {
      double v[3];
      int32_t rc = tog_batch_stats_end(p, v);
      if (rc) return rc;
      acc[0] += v[0];
      acc[1] += v[1];
      acc[2] = tog_jlmax(acc[2], v[2]);
    }
    out3[0] = acc[0], out3[1] = acc[1], out3[2] = acc[2];
    return TOG_OK;
  }
  if (!h->stats_pending) return fail(TOG_ERR_ARG, "tog_batch_stats_end without tog_batch_stats_begin");
  HIPCHECK(hipSetDevice(h->device));
  h->stats_pending = false;
  const int rc = wait_event(h->stats_ev, "tog_batch_stats");
  if (rc) return rc;
  out3[0] = h->h_stats[0], out3[1] = h->h_stats[1], out3[2] = h->h_stats[2];
  h->last_active = out3[0];
  return TOG_OK;
}

int32_t tog_total_steps(tog_handle* h, int64_t* out) {
  if (!h || !out) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    int64_t t = 0;
    int32_t rc = each_part(h, [&](tog_handle* p, size_t) {
      int64_t v = 0;
      int32_t r = tog_total_steps(p, &v);
      t += v;
      return r;
    });
    *out = t;
    return rc;
  }
  std::vector<TrajState> st;
  int rc = get_states(h, st);
  if (rc) return rc;
  int64_t t = 0;
  for (const auto& s : st) t += s.total_steps;
  *out = t;
  return TOG_OK;
}

// The stopping check is pipelined: chunk i+1's steps are enqueued before the host waits for chunk i's
// statistics, so the device never idles on the host round trip. The last chunk after the batch finished
// runs on inactive trajectories only (every kernel returns at once for them); the arithmetic of the
// solve does not depend on when the host learns the active count (it only picks launch widths).
// after a failure between tog_batch_stats_begin and _end: no check stays pending on any part, so that the
// handle's next tog_batch_stats / tog_solve does not fail with "the previous check was not ended"
static void abandon_stats(tog_handle* h) {
  h->stats_pending = false;
  for (tog_handle* p : h->parts) abandon_stats(p);
}

int32_t tog_solve(tog_handle* h, int32_t mode, int32_t max_steps) {
  int rc = tog_solve_init(h, mode);
  if (rc) return rc;
  if (max_steps <= 0) max_steps = tog_solve_budget(h, mode);
  const int chunk = 4;
  double stats[3];
  int done = chunk < max_steps ? chunk : max_steps;
  if ((rc = tog_solve_step(h, done)) || (rc = tog_batch_stats_begin(h))) return abandon_stats(h), rc;
  while (true) {
    const int next = chunk < max_steps - done ? chunk : max_steps - done;
    if (next > 0 && (rc = tog_solve_step(h, next))) return abandon_stats(h), rc;
    done += next;
    if ((rc = tog_batch_stats_end(h, stats))) return rc;  // the chunk before `next`
    if (stats[0] == 0.0 || next == 0) break;
    if ((rc = tog_batch_stats_begin(h))) return rc;
  }
  return TOG_OK;
}

int32_t tog_profile(tog_handle* h, int32_t enable) {
  if (!h) return fail(TOG_ERR_ARG, "null handle");
  if (is_multi(h)) return each_part(h, [&](tog_handle* p, size_t) { return tog_profile(p, enable); });
  HIPCHECK(hipSetDevice(h->device));
  if (enable) {
    HIPCHECK(hipStreamSynchronize(h->stream));
    h->ev_used = 0;
    h->ev_kind.clear();
  }
  h->profiling = enable != 0;
  return TOG_OK;
}

int32_t tog_profile_read(tog_handle* h, double* total_ms, int64_t* launches) {
  if (!h || !total_ms || !launches) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {  // summed over devices
    double ms[TOG_NKERNELS] = {0};
    int64_t ln[TOG_NKERNELS] = {0};
    int32_t rc = each_part(h, [&](tog_handle* p, size_t) {
      double a[TOG_NKERNELS];
      int64_t b[TOG_NKERNELS];
      int32_t r = tog_profile_read(p, a, b);
      for (int i = 0; i < TOG_NKERNELS; i++) ms[i] += a[i], ln[i] += b[i];
      return r;
    });
    for (int i = 0; i < TOG_NKERNELS; i++) total_ms[i] = ms[i], launches[i] = ln[i];
    return rc;
  }
  HIPCHECK(hipSetDevice(h->device));
  HIPCHECK(hipStreamSynchronize(h->stream));
  for (int i = 0; i < TOG_NKERNELS; i++) {
    total_ms[i] = 0.0;
    launches[i] = 0;
  }
  for (size_t p = 0; p < h->ev_kind.size(); p++) {
    float ms = 0.f;
    HIPCHECK(hipEventElapsedTime(&ms, h->ev_pool[2 * p], h->ev_pool[2 * p + 1]));
    total_ms[h->ev_kind[p]] += ms;
    launches[h->ev_kind[p]] += 1;
  }
  return TOG_OK;
}

void tog_default_pn_options(tog_pn_options* o) {
  o->n_steps = 1;
  o->solve_type = 0;
  o->active_set_tolerance = 1e-3;
  o->feasibility_tolerance = 1e-6;
}

// solve!(prob, ProjectedNewtonSolver) (projected_newton.jl:6-20): per newton step, k_pn_begin
// (update! + the first viol), then projection_solve!'s loop of at most 10 _projection_solve!s (each
// after k_jacobian at the current X, U), then k_pn_finish (record_iteration!). Trajectories that
// are done return at once from every launch.
int32_t tog_solve_pn(tog_handle* h, const tog_pn_options* opts, double* out) {
  if (!h || !opts) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h))
    return each_part(h, [&](tog_handle* p, size_t o) {
      return tog_solve_pn(p, opts, out ? out + o * TOG_PN_NSTATS : nullptr);
    });
  if (opts->solve_type != 0 && opts->solve_type != 1) return fail(TOG_ERR_ARG, "solve_type must be 0 (:feasible) or 1 (:optimal)");
  const bool optimal = opts->solve_type == 1;
  if (opts->n_steps < 0) return fail(TOG_ERR_ARG, "n_steps must be >= 0");
  if (!h->ops->pn) return fail(TOG_ERR_UNSUPPORTED, "projected Newton needs n + m <= 64 (a lane per variable of a knot)");
  // block stride: n + every row of a knot, capped at a wave's 64 rows; blocks are sized by the *active* rows
  // (k_pn_* flag TOG_TRAJ_PN_BLOCK on a trajectory whose active set outgrows the stride)
  const int SM = std::min(h->n + h->pmax, PN_SM_MAX);
  if (SM < h->n) return fail(TOG_ERR_UNSUPPORTED, "projected Newton needs n <= 64");
  HIPCHECK(hipSetDevice(h->device));
  PNBuffers& W = h->pn;
  const long long B = h->B;
  if (h->pn_alloc && W.SM != SM) return fail(TOG_ERR_ARG, "projected Newton workspace stride changed");
  if (!h->pn_alloc) {
    W.SM = SM;
    W.nb = h->N + 1;
    const size_t blk = (size_t)B * W.nb * SM * SM, vec = (size_t)B * W.nb * SM;
    const size_t pm = (size_t)(h->pmax > 0 ? h->pmax : 1);
    // the whole workspace is sized before any allocation: a batch whose block factors do not fit the
    // device's free memory is refused with TOG_ERR_NOMEM (solve it in slices, tog_create_multi)
    const size_t need = sizeof(double) * (4 * blk + 5 * vec + 2 * (size_t)B * h->N * h->n) +
                        sizeof(int) * ((size_t)B * h->N * pm + (size_t)B * h->N + (size_t)B * W.nb) +
                        sizeof(PNState) * (size_t)B;
    size_t fr = 0, tot = 0;
    HIPCHECK(hipMemGetInfo(&fr, &tot));
    if (need > fr)
      return fail(TOG_ERR_NOMEM, "projected Newton workspace (" + std::to_string(need >> 20) + " MiB) exceeds free device memory (" +
                                     std::to_string(fr >> 20) + " MiB)");
    const size_t mark = h->allocs.size();
    int rc;
    if ((rc = dalloc(h, &W.Sd, blk)) || (rc = dalloc(h, &W.So, blk)) || (rc = dalloc(h, &W.Ld, blk)) ||
        (rc = dalloc(h, &W.Lo, blk)) || (rc = dalloc(h, &W.yv, vec)) || (rc = dalloc(h, &W.xv, vec)) ||
        (rc = dalloc(h, &W.rv, vec)) || (rc = dalloc(h, &W.wv, vec)) || (rc = dalloc(h, &W.dv, vec)) ||
        (rc = dalloc(h, &W.yd, (size_t)B * h->N * h->n)) || (rc = dalloc(h, &W.Xs, (size_t)B * h->N * h->n)) ||
        (rc = dalloc(h, &W.act, (size_t)B * h->N * (h->pmax > 0 ? h->pmax : 1))) ||
        (rc = dalloc(h, &W.na, (size_t)B * h->N)) || (rc = dalloc(h, &W.sz, (size_t)B * W.nb)) ||
        (rc = dalloc(h, &W.st, (size_t)B)) ||
        (h->ops->min_time && (rc = dalloc(h, &W.wt, (size_t)B * ((size_t)h->N * h->n + (size_t)(h->N - 1) * h->m))))) {
      // partial failure: release what this call allocated, so a retry does not leak it
      for (size_t i = mark; i < h->allocs.size(); i++) (void)hipFree(h->allocs[i]);
      h->allocs.resize(mark);
      (void)hipGetLastError();
      return rc;
    }
    h->pn_alloc = true;
  }
  if (optimal && !h->pn_opt_alloc) {  // :optimal's workspace: two more block factors, the duals and the KKT vectors
    const size_t blk = (size_t)B * W.nb * SM * SM, vec = (size_t)B * W.nb * SM;
    const size_t nz = (size_t)B * h->N * (h->n + h->m), nx = (size_t)B * h->N * h->n;
    const size_t nc = (size_t)B * h->N * (h->pmax > 0 ? h->pmax : 1), nu = (size_t)B * (h->N - 1) * h->m;
    const size_t need = sizeof(double) * (2 * blk + 2 * vec + 3 * nz + 4 * nx + 3 * nc + nu) + sizeof(int) * (size_t)B * W.nb;
    size_t fr = 0, tot = 0;
    HIPCHECK(hipMemGetInfo(&fr, &tot));
    if (need > fr)
      return fail(TOG_ERR_NOMEM, "projected Newton :optimal workspace (" + std::to_string(need >> 20) +
                                     " MiB) exceeds free device memory (" + std::to_string(fr >> 20) + " MiB)");
    const size_t mark = h->allocs.size();
    int rc;
    if ((rc = dalloc(h, &W.Ld2, blk)) || (rc = dalloc(h, &W.Lo2, blk)) || (rc = dalloc(h, &W.lb, vec)) ||
        (rc = dalloc(h, &W.tb, vec)) || (rc = dalloc(h, &W.g, nz)) || (rc = dalloc(h, &W.rz, nz)) ||
        (rc = dalloc(h, &W.dz, nz)) || (rc = dalloc(h, &W.nu, nx)) || (rc = dalloc(h, &W.dnu, nx)) ||
        (rc = dalloc(h, &W.nut, nx)) || (rc = dalloc(h, &W.Xv, nx)) || (rc = dalloc(h, &W.lc, nc)) ||
        (rc = dalloc(h, &W.dlc, nc)) || (rc = dalloc(h, &W.lct, nc)) || (rc = dalloc(h, &W.Uv, nu)) ||
        (rc = dalloc(h, &W.szS, (size_t)B * W.nb))) {
      for (size_t i = mark; i < h->allocs.size(); i++) (void)hipFree(h->allocs[i]);
      h->allocs.resize(mark);
      (void)hipGetLastError();
      return rc;
    }
    h->pn_opt_alloc = true;
  }
  W.optimal = optimal ? 1 : 0;
  if (optimal) {  // PrimalDual(prob): zero duals
    HIPCHECK(hipMemsetAsync(W.nu, 0, sizeof(double) * (size_t)B * h->N * h->n, h->stream));
    HIPCHECK(hipMemsetAsync(W.lc, 0, sizeof(double) * (size_t)B * h->N * (h->pmax > 0 ? h->pmax : 1), h->stream));
  }
  W.atol = opts->active_set_tolerance;
  W.eps = opts->feasibility_tolerance;
  HIPCHECK(hipMemsetAsync(W.st, 0, sizeof(PNState) * B, h->stream));
  // solver_pn.stats[:cost] / [:c_max] per newton step (tog_get_pn_history): read after each step's
  // record_iteration! (k_pn_finish); a trajectory records in a step iff its step counter moved
  h->pn_hist.assign((size_t)2 * std::max(opts->n_steps, 0) * B, NAN);
  h->pn_hist_steps = opts->n_steps;
  std::vector<PNState> stp(B);
  for (int step = 0; step < opts->n_steps; step++) {
    h->ops->pn(h->dP, h->buf, W, B, h->integ, 0, h->stream);
    for (int it = 0; it < 10; it++) {
      h->ops->jacobian(h->dP, h->buf, B, h->N, h->integ, h->stream);
      h->ops->pn(h->dP, h->buf, W, B, h->integ, 1, h->stream);
    }
    if (optimal) {  // the KKT step and its line search: 10 trials of at most 12 projection! passes
      h->ops->pn(h->dP, h->buf, W, B, h->integ, 3, h->stream);
      h->ops->jacobian(h->dP, h->buf, B, h->N, h->integ, h->stream);
      h->ops->pn(h->dP, h->buf, W, B, h->integ, 4, h->stream);
      for (int ls = 0; ls < 10; ls++) {
        for (int it = 0; it < 12; it++) {
          h->ops->jacobian(h->dP, h->buf, B, h->N, h->integ, h->stream);
          h->ops->pn(h->dP, h->buf, W, B, h->integ, 5, h->stream);
        }
        h->ops->pn(h->dP, h->buf, W, B, h->integ, 6, h->stream);
      }
    }
    h->ops->pn(h->dP, h->buf, W, B, h->integ, 2, h->stream);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(stp.data(), W.st, sizeof(PNState) * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    for (long long b = 0; b < B; b++)
      if (stp[b].steps == step + 1) {
        h->pn_hist[2 * ((size_t)b * opts->n_steps + step)] = stp[b].J;
        h->pn_hist[2 * ((size_t)b * opts->n_steps + step) + 1] = stp[b].c_max;
      }
  }
  h->pn_hist_rec.assign(B, 0);
  for (long long b = 0; b < B && opts->n_steps > 0; b++) h->pn_hist_rec[b] = stp[b].steps;
  if (out) {
    std::vector<PNState> st(B);
    HIPCHECK(hipMemcpyAsync(st.data(), W.st, sizeof(PNState) * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    for (long long b = 0; b < B; b++) {
      double* o = out + b * TOG_PN_NSTATS;
      o[TOG_PN_VIOL] = st[b].viol;
      o[TOG_PN_C_MAX] = st[b].c_max;
      o[TOG_PN_J] = st[b].J;
      o[TOG_PN_PROJECTIONS] = st[b].projections;
      o[TOG_PN_LINESEARCHES] = st[b].linesearches;
      o[TOG_PN_REFINEMENTS] = st[b].refinements;
      o[TOG_PN_STEPS] = st[b].steps;
    }
  }
  return TOG_OK;
}

int32_t tog_get_pn_history(tog_handle* h, double* out, int32_t* steps_out) {
  if (!h || !out) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) {
    const size_t w = 2 * (size_t)std::max(h->parts[0]->pn_hist_steps, 0);
    return each_part(h, [&](tog_handle* p, size_t o) {
      return tog_get_pn_history(p, out + o * w, steps_out ? steps_out + o : nullptr);
    });
  }
  if (h->pn_hist_steps < 0) return fail(TOG_ERR_ARG, "no projected Newton solve on this handle");
  std::copy(h->pn_hist.begin(), h->pn_hist.end(), out);
  if (steps_out)
    for (long long b = 0; b < h->B; b++) steps_out[b] = h->pn_hist_rec.empty() ? 0 : h->pn_hist_rec[b];
  return TOG_OK;
}

int32_t tog_status(tog_handle* h, int32_t* flags_out) {
  if (!h || !flags_out) return fail(TOG_ERR_ARG, "null argument");
  if (is_multi(h)) return each_part(h, [&](tog_handle* p, size_t o) { return tog_status(p, flags_out + o); });
  std::vector<TrajState> st;
  int rc = get_states(h, st);
  if (rc) return rc;
  for (size_t i = 0; i < st.size(); i++) flags_out[i] = st[i].flags | (st[i].active ? TOG_TRAJ_ACTIVE : 0);
  return TOG_OK;
}

// (internal, diagnostics) the last forward pass's speculative trials: J (nc, B) and rollout status (nc, B)
int32_t tog__debug_ls(tog_handle* h, double* J, int32_t* ok, int32_t* nc) {
  if (!h || is_multi(h)) return fail(TOG_ERR_ARG, "tog__debug_ls: single-device handle");
  *nc = h->buf.nc;
  HIPCHECK(hipStreamSynchronize(h->stream));
  if (J) HIPCHECK(hipMemcpy(J, h->buf.lsJ, sizeof(double) * h->buf.nc * h->B, hipMemcpyDeviceToHost));
  if (ok) HIPCHECK(hipMemcpy(ok, h->buf.lsok, sizeof(int) * h->buf.nc * h->B, hipMemcpyDeviceToHost));
  return TOG_OK;
}

}  // extern "C"
