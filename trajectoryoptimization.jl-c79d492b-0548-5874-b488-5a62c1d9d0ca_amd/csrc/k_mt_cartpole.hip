// Kernel instantiation for the minimum-time cartpole model, add_min_time_controls(model)
// (src/solvers/altro/minimum_time.jl:83-104): state [x; τ], control [u; h], dt = h² (tog_device.hpp MinTime<M>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mt_cartpole() {
  static const ModelOps o = ModelLaunch<MinTime<Cartpole>>::ops();
  return &o;
}
}  // namespace tog
