// plan_rk4_l1.hip — plan-kernel instantiations: RK4, one lane per rollout (throughput regime, work-queue layouts) + its inline-pack host tick
// (one translation unit per variant group; device code in plan_dev.hpp).
#include "plan_dev.hpp"

namespace llampc {

template void launch_plan_group<0, 1>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);
template void launch_plan_inline_group<1>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                              int, int, size_t, hipStream_t, const InlinePack&);

}  // namespace llampc

#ifdef LLAMPC_STAMPS
// diagnostic readers of this TU's stamp buffers (the headline variants live here)
namespace llampc {
extern "C" int llampc_debug_wq_units(unsigned long long* out) {   // [256][8][16][4][2]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wq_unit), sizeof(g_wq_unit)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_wq_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_wq_unit)) != hipSuccess) return -2;
  return hipMemset(p, 0, sizeof(g_wq_unit)) == hipSuccess ? 0 : -2;
}
}  // namespace llampc
#endif
