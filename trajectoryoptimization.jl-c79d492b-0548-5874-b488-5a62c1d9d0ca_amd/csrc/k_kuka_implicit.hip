// Kernel instantiation for the Kuka iiwa model under the implicit integrators (midpoint_implicit,
// rk3_implicit; src/integration.jl:44-73, :171-205): a unit of its own, built in parallel with k_kuka.hip.
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_kuka_implicit() {
  static const ModelOps o = ModelLaunch<KukaImplicit>::ops();
  return &o;
}
}  // namespace tog
