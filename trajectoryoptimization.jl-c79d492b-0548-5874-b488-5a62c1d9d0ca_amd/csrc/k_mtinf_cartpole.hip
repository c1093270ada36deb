// Kernel instantiation for the infeasible-start minimum-time cartpole model, add_min_time_controls(add_slack_controls(
// model)) (altro_methods.jl:98-124): state [x; τ], control [u; s; h] (tog_device.hpp MinTime<Infeasible<M>>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mtinf_cartpole() {
  static const ModelOps o = ModelLaunch<MinTime<Infeasible<Cartpole>>>::ops();
  return &o;
}
}  // namespace tog
