// tog_plugin.hpp — build a user model (Model(f!, n, m), src/model.jl:103-131) as a libtog plugin.
//
// A plugin is one HIP translation unit, compiled for gfx950 into a shared object:
//
//   #include "tog_plugin.hpp"
//   struct MyModel {
//     static constexpr int n = 2, m = 1, id = TOG_MODEL_USER;
//     template <class T>
//     __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) { ... }
//   };
//   TOG_PLUGIN(MyModel)
//
// f is the continuous dynamics ẋ = f(x, u), written once over the scalar type T: the rollouts call
// it with double, the Jacobian kernel with Dual<W> (ForwardDiff's forward mode, src/model.jl:491-522).
// Use +, -, *, / and the helpers sin_, cos_, sqrt_, inv_ and cst_(value, like) (a constant of T's
// type) from tog_device.hpp. The plugin instantiates every kernel of the path (rollouts, Jacobians,
// backward passes, line search, AL updates, projected Newton) for the model, for its
// infeasible-start variant add_slack_controls(model) (src/model.jl:761-779) and for its minimum-time
// variant add_min_time_controls(model) (src/solvers/altro/minimum_time.jl:83-104); libtog dispatches to
// them through the same ModelOps table its built-in models use. tog_model_load checks the plugin's
// layout fingerprint, so a plugin built against other headers is refused instead of misread.
#pragma once

#include "tog_kernels.hpp"

namespace tog {
// layout fingerprint of the structures shared across the plugin boundary, combined with the hash of
// the text of every libtog header (TOG_HEADER_HASH, tog_device.hpp): a plugin built against other
// kernel code -- same struct sizes, different numerics or protocol -- is refused as well
constexpr long long plugin_fingerprint() {
  return ((long long)TOG_ABI_VERSION * 1000003LL + (long long)sizeof(DevProblem) * 7919LL +
          (long long)sizeof(DevBuffers) * 131LL + (long long)sizeof(ModelOps) * 17LL + (long long)sizeof(TrajState)) ^
         (long long)TOG_HEADER_HASH;
}
}  // namespace tog

#define TOG_PLUGIN(MODEL)                                                                         \
  static_assert(MODEL::n >= 1 && MODEL::n <= tog::NMAX, "plugin model: 1 <= n <= NMAX");          \
  static_assert(MODEL::m >= 1 && MODEL::m + MODEL::n <= tog::MMAX, "plugin model: m + n <= MMAX"); \
  static_assert(MODEL::n + 1 <= tog::NMAX, "plugin model: n + 1 <= NMAX (minimum-time state)");   \
  extern "C" long long tog_plugin_fingerprint() { return tog::plugin_fingerprint(); }             \
  extern "C" const tog::ModelOps* tog_plugin_ops() {                                              \
    static const tog::ModelOps o = tog::ModelLaunch<MODEL>::ops();                                \
    return &o;                                                                                    \
  }                                                                                               \
  extern "C" const tog::ModelOps* tog_plugin_ops_infeasible() {                                   \
    static const tog::ModelOps o = tog::ModelLaunch<tog::Infeasible<MODEL>>::ops();              \
    return &o;                                                                                    \
  }                                                                                               \
  extern "C" const tog::ModelOps* tog_plugin_ops_min_time() {                                     \
    static const tog::ModelOps o = tog::ModelLaunch<tog::MinTime<MODEL>>::ops();                 \
    return &o;                                                                                    \
  }
