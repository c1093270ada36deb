// GenericCost(mycost, mycost, gradient, hess, n, m) of test/cost_tests.jl:112-132 (analytic expansion)
#include "../tog_cost_plugin.hpp"

struct MyCostAnalytic {
  static constexpr int n = 2, m = 1;
  static constexpr bool has_expansion = true;
  __host__ __device__ static double stage(const double* x, const double* u) {
    return (tog::cos_(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1]);
  }
  __host__ __device__ static double terminal(const double* x) { return tog::cos_(x[0]) + x[1] * x[1]; }
  // hess(x, u) = (Diagonal([-cos(x1), 2Q]), 2R, zeros(m, n)); gradient(x, u) = ([-sin(x1), 2Q x2], 2R u)
  __host__ __device__ static void expansion(double* Q, double* R, double* H, double* q, double* r, const double* x,
                                            const double* u) {
    Q[0] = -tog::cos_(x[0]);
    Q[1] = 0.0;
    Q[2] = 0.0;
    Q[3] = 2.0 * 0.1;
    R[0] = 2.0 * 0.1;
    H[0] = 0.0;
    H[1] = 0.0;
    q[0] = -tog::sin_(x[0]);
    q[1] = (2.0 * 0.1) * x[1];
    r[0] = (2.0 * 0.1) * u[0];
  }
  // hess(x) = Diagonal([-cos(x1), 2]); gradient(x) = [-sin(x1), 2 x2]
  __host__ __device__ static void expansion_term(double* Qf, double* qf, const double* x) {
    Qf[0] = -tog::cos_(x[0]);
    Qf[1] = 0.0;
    Qf[2] = 0.0;
    Qf[3] = 2.0;
    qf[0] = -tog::sin_(x[0]);
    qf[1] = 2.0 * x[1];
  }
};

TOG_COST_PLUGIN(MyCostAnalytic)
