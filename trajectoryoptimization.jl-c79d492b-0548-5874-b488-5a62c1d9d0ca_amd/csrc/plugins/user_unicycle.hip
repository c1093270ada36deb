// A user model that is not among the built-in dynamics: a unicycle with first-order speed and turn-rate
// actuators, x = [px, py, θ, v, ω], u = [a, α] (accelerations):
//   ṗx = v cos θ, ṗy = v sin θ, θ̇ = ω, v̇ = a − c_v v, ω̇ = α − c_ω ω.
#include "../tog_plugin.hpp"

struct UserUnicycle {
  static constexpr int n = 5, m = 2, id = TOG_MODEL_USER;
  template <class T>
  __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const double cv = 0.1, cw = 0.2;
    xd[0] = x[3] * tog::cos_(x[2]);
    xd[1] = x[3] * tog::sin_(x[2]);
    xd[2] = x[4];
    xd[3] = u[0] - cv * x[3];
    xd[4] = u[1] - cw * x[4];
  }
  // fid 0: a disc obstacle at (1, 0.5), radius 0.3 (stage); fid 1: traction limit a·v <= 1 (depends on u)
  static constexpr bool has_con = true;
  template <class T>
  __host__ __device__ __forceinline__ static void con(int fid, T* c, const T* x, const T* u) {
    if (fid == 0) {
      const T dx = x[0] - 1.0, dy = x[1] - 0.5;
      c[0] = -((dx * dx + dy * dy) - 0.09);
    } else {
      c[0] = u[0] * x[3] - 1.0;
    }
  }
};

TOG_PLUGIN(UserUnicycle)
