// Kernel instantiation for the infeasible-start minimum-time pendulum model, add_min_time_controls(add_slack_controls(
// model)) (altro_methods.jl:98-124): state [x; τ], control [u; s; h] (tog_device.hpp MinTime<Infeasible<M>>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mtinf_pendulum() {
  static const ModelOps o = ModelLaunch<MinTime<Infeasible<Pendulum>>>::ops();
  return &o;
}
}  // namespace tog
