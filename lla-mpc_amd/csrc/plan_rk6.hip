// plan_rk6.hip — plan-kernel instantiations: the RK6 plant integrator
// (one translation unit per variant group; device code in plan_dev.hpp).
#include "plan_dev.hpp"

namespace llampc {

template void launch_plan_group<2, 1>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);

}  // namespace llampc
