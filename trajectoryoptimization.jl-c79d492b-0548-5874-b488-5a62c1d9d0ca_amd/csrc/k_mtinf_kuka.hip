// Kernel instantiation for the infeasible-start minimum-time kuka model, add_min_time_controls(add_slack_controls(
// model)) (altro_methods.jl:98-124): state [x; τ], control [u; s; h] (tog_device.hpp MinTime<Infeasible<M>>).
// m + n + 1 controls > n + 1 states: the LDS backward kernel (k_backward).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mtinf_kuka() {
  static const ModelOps o = ModelLaunch<MinTime<Infeasible<Kuka>>>::ops();
  return &o;
}
}  // namespace tog
