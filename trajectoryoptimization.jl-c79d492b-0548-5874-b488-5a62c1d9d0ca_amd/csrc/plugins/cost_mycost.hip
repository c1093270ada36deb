// GenericCost(mycost, mycost, n, m) of test/cost_tests.jl:98-108 (ForwardDiff expansion):
//   ℓ(x, u) = cos(x1) + u'Ru + Q x2²  (R = 0.1 I, Q = 0.1),  ℓf(xN) = cos(xN1) + xN2²
#include "../tog_cost_plugin.hpp"

struct MyCost {
  static constexpr int n = 2, m = 1;
  template <class T>
  __host__ __device__ __forceinline__ static T stage(const T* x, const T* u) {
    return (tog::cos_(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1]);
  }
  template <class T>
  __host__ __device__ __forceinline__ static T terminal(const T* x) {
    return tog::cos_(x[0]) + x[1] * x[1];
  }
};

TOG_COST_PLUGIN(MyCost)
