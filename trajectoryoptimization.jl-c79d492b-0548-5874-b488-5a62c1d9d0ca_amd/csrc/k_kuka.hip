// Kernel instantiation for the Kuka iiwa model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_kuka() {
  static const ModelOps o = ModelLaunch<Kuka>::ops();
  return &o;
}
}  // namespace tog
