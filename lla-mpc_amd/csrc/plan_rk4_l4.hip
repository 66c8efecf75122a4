// plan_rk4_l4.hip — plan-kernel instantiations: RK4, four lanes per rollout (the headline C = 1 tick) + its inline-pack host tick
// (one translation unit per variant group; device code in plan_dev.hpp).
#include "plan_dev.hpp"

namespace llampc {

template void launch_plan_group<0, 4>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);
template void launch_plan_inline_group<4>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                              int, int, size_t, hipStream_t, const InlinePack&);

}  // namespace llampc

#ifdef LLAMPC_STAMPS
// diagnostic readers of this TU's stamp buffers (the headline variants live here)
namespace llampc {
extern "C" int llampc_debug_lb_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lb_stamps), sizeof(g_lb_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_rl_ph(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rl_ph), sizeof(g_rl_ph)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_rl(double* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rl_dbg), sizeof(g_rl_dbg)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_la_wave(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_la_wave), sizeof(g_la_wave)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_la_all(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_la_all), sizeof(g_la_all)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_la_step(unsigned long long* out) {   // [1024][25]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_la_step), sizeof(g_la_step)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_la_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_la_stamps), sizeof(g_la_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int llampc_debug_stamps(unsigned long long* out, unsigned* launches) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) != hipSuccess) return -2;
  return hipMemcpyFromSymbol(launches, HIP_SYMBOL(g_stamp_launch), sizeof(unsigned)) == hipSuccess ? 0 : -2;
}
}  // namespace llampc
#endif
