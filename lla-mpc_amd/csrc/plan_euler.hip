// plan_euler.hip — plan-kernel instantiations: the NLP Euler transcription, every lane split
// (one translation unit per variant group; device code in plan_dev.hpp).
#include "plan_dev.hpp"

namespace llampc {

template void launch_plan_group<1, 4>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);
template void launch_plan_group<1, 2>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);
template void launch_plan_group<1, 1>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&, int,
                                            int, bool, size_t, hipStream_t, int);

}  // namespace llampc
