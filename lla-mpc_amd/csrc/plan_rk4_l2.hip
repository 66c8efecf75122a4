// plan_rk4_l2.hip — plan-kernel instantiations: RK4, two lanes per rollout + its inline-pack host tick
// (one translation unit per variant group; device code in plan_dev.hpp).
#include "plan_dev.hpp"

namespace llampc {

template void launch_plan_group<0, 2>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);
template void launch_plan_inline_group<2>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                              int, int, size_t, hipStream_t, const InlinePack&);

}  // namespace llampc
