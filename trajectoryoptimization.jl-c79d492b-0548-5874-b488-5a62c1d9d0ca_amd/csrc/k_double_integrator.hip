// Kernel instantiation for the double_integrator model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_double_integrator() {
  static const ModelOps o = ModelLaunch<DoubleIntegrator>::ops();
  return &o;
}
}  // namespace tog
