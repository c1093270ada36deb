// The quadrotor's dual-number Jacobian kernels (k_jacobian, tog_kernels.hpp) in a translation unit of
// their own, built with LLVM's max-ILP machine scheduler (Makefile): on this kernel it shortens the
// dependent FP64 chains of the RK4 dual evaluation (0.944 -> 0.872 ms at config 3), while the same
// scheduler makes the backward team kernel slower (3.60 -> 3.71 ms), so k_quadrotor.hip keeps the default.
#include "tog_kernels.hpp"

namespace tog {
template __global__ void k_jacobian<Quadrotor, TOG_RK3, TOG_JW>(const DevProblem*, DevBuffers, long long);
template __global__ void k_jacobian<Quadrotor, TOG_RK4, TOG_JW>(const DevProblem*, DevBuffers, long long);
template __global__ void k_jacobian<Quadrotor, TOG_MIDPOINT, TOG_JW>(const DevProblem*, DevBuffers, long long);
}  // namespace tog
