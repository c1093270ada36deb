// Kernel instantiation for the infeasible-start kuka model, add_slack_controls(model)
// (src/model.jl:761-779): n slack controls on top of the model's m (tog_device.hpp Infeasible<M>).
#include "tog_kernels.hpp"

namespace tog {
const ModelOps* ops_inf_kuka() {
  static const ModelOps o = ModelLaunch<Infeasible<Kuka>>::ops();
  return &o;
}
}  // namespace tog
