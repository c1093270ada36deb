// Kernel instantiation for the car model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_car() {
  static const ModelOps o = ModelLaunch<Car>::ops();
  return &o;
}
}  // namespace tog
