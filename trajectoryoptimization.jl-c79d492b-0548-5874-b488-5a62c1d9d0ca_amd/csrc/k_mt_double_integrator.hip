// Kernel instantiation for the minimum-time double_integrator model, add_min_time_controls(model)
// (src/solvers/altro/minimum_time.jl:83-104): state [x; τ], control [u; h], dt = h² (tog_device.hpp MinTime<M>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_mt_double_integrator() {
  static const ModelOps o = ModelLaunch<MinTime<DoubleIntegrator>>::ops();
  return &o;
}
}  // namespace tog
