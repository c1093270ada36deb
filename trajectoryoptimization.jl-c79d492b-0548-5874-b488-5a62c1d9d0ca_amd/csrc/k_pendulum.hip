// Kernel instantiation for the pendulum model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_pendulum() {
  static const ModelOps o = ModelLaunch<Pendulum>::ops();
  return &o;
}
}  // namespace tog
