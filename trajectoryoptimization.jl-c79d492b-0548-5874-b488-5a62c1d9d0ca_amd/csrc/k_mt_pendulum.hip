// Kernel instantiation for the minimum-time pendulum model, add_min_time_controls(model)
// (src/solvers/altro/minimum_time.jl:83-104): state [x; τ], control [u; h], dt = h² (tog_device.hpp MinTime<M>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mt_pendulum() {
  static const ModelOps o = ModelLaunch<MinTime<Pendulum>>::ops();
  return &o;
}
}  // namespace tog
