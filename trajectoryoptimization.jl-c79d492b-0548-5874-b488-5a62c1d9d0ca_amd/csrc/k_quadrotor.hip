// Kernel instantiation for the quadrotor model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_quadrotor() {
  static const ModelOps o = ModelLaunch<Quadrotor>::ops();
  return &o;
}
}  // namespace tog
