// A user model written against the plugin API (tog_plugin.hpp): the reference's pendulum
// (dynamics/pendulum.jl:3-12) as a user would define it with Model(pendulum_dynamics!, 2, 1). The
// operation sequence is the built-in Pendulum's, so tests can hold the plugin path bit for bit against
// the built-in model and the CPU oracle.
#include "../tog_plugin.hpp"

struct UserPendulum {
  static constexpr int n = 2, m = 1, id = TOG_MODEL_USER;
  template <class T>
  __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const double mm = 1.0, b = 0.1, lc = 0.5, I = 0.25, g = 9.81;
    xd[0] = x[1];
    xd[1] = ((u[0] - (mm * g * lc) * tog::sin_(x[0])) - b * x[1]) / I;
  }
  // user constraint functions (Constraint{Inequality}(c!, n, m, p), src/constraints.jl:85-89):
  // fid 0 is circle_constraint(x, 1.2, 2.5, 0.6) (src/utils.jl:140-144), an obstacle in the (θ, ω)
  // plane, written as the built-in circle rows evaluate it.
  static constexpr bool has_con = true;
  template <class T>
  __host__ __device__ __forceinline__ static void con(int fid, T* c, const T* x, const T* u) {
    (void)u;
    if (fid == 0) {
      const double a = 1.2, bb = 2.5, r = 0.6;
      const T dx = x[0] - a, dy = x[1] - bb;
      c[0] = -((dx * dx + dy * dy) - r * r);
    }
  }
};

TOG_PLUGIN(UserPendulum)
