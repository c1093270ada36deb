// A non-quadratic GenericCost over a planar point mass (n = 4: px, py, vx, vy; m = 2): tracking plus a
// smooth obstacle penalty and a speed-dependent control weight, exercising /, sqrt and sin:
//   ℓ(x, u)  = ½(px² + py²) + w / (ε + (px - ox)² + (py - oy)²) + ½ |u|² · sqrt(1 + vx² + vy²) + 0.1 sin(vx) vy
//   ℓf(xN)   = 10 (px² + py²) + 1 / (1 + vx² + vy²)
#include "../tog_cost_plugin.hpp"

struct SoftObstacleCost {
  static constexpr int n = 4, m = 2;
  template <class T>
  __host__ __device__ __forceinline__ static T stage(const T* x, const T* u) {
    const double w = 0.5, eps = 0.1, ox = 1.0, oy = 0.5;
    const T dx = x[0] - ox, dy = x[1] - oy;
    const T track = 0.5 * (x[0] * x[0] + x[1] * x[1]);
    const T obs = w / ((eps + dx * dx) + dy * dy);
    const T speed = tog::sqrt_((1.0 + x[2] * x[2]) + x[3] * x[3]);
    const T effort = (0.5 * (u[0] * u[0] + u[1] * u[1])) * speed;
    return ((track + obs) + effort) + 0.1 * (tog::sin_(x[2]) * x[3]);
  }
  template <class T>
  __host__ __device__ __forceinline__ static T terminal(const T* x) {
    return 10.0 * (x[0] * x[0] + x[1] * x[1]) + 1.0 / ((1.0 + x[2] * x[2]) + x[3] * x[3]);
  }
};

TOG_COST_PLUGIN(SoftObstacleCost)
