// Kernel instantiation for the quadrotor model (one translation unit per model keeps builds parallel).
#include "tog_kernels.hpp"

namespace tog {
// the Jacobian kernels are instantiated in k_quadrotor_jac.hip, built with another machine scheduler
extern template __global__ void k_jacobian<Quadrotor, TOG_RK3, TOG_JW>(const DevProblem*, DevBuffers, long long);
extern template __global__ void k_jacobian<Quadrotor, TOG_RK4, TOG_JW>(const DevProblem*, DevBuffers, long long);
extern template __global__ void k_jacobian<Quadrotor, TOG_MIDPOINT, TOG_JW>(const DevProblem*, DevBuffers, long long);

const ModelOps* ops_quadrotor() {
  static const ModelOps o = ModelLaunch<Quadrotor>::ops();
  return &o;
}
}  // namespace tog

#ifdef TOG_BWD_PROF
// read (and reset) the backward-kernel section timers of the quadrotor instantiations
extern "C" int tog_bwd_prof_read(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tog::tog_bwd_prof), sizeof(unsigned long long) * tog::BPROF_N) != hipSuccess)
    return -1;
  unsigned long long z[tog::BPROF_N] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(tog::tog_bwd_prof), z, sizeof(z)) == hipSuccess ? tog::BPROF_N : -1;
}
#endif
