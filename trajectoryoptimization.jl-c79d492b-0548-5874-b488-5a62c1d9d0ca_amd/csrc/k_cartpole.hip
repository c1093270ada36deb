// Kernel instantiation for the cartpole model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_cartpole() {
  static const ModelOps o = ModelLaunch<Cartpole>::ops();
  return &o;
}
}  // namespace tog
