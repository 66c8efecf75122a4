#!/bin/bash
# C = 1 headline-shape timeline and the controller phases (stamps build); controller tests.
set -o pipefail
T=${1:-r04tl}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > $OUT/tl.txt 2>&1 || { echo "timeline failed"; tail -20 $OUT/tl.txt; exit 1; }
grep -v amdgpu.ids $OUT/tl.txt | grep "lb_final\|final_select\|all 157"
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_phases.log 2>&1 || { echo "ctl_phases failed"; tail -30 $OUT/ctl_phases.log; exit 1; }
grep -v amdgpu.ids $OUT/ctl_phases.log
timeout -k 10 420 python -u -m pytest tests/test_ctl_gpu.py -x -q --timeout 150 --timeout-method thread > $OUT/ctl.log 2>&1 || { echo "ctl tests failed"; tail -30 $OUT/ctl.log; exit 1; }
tail -n 1 $OUT/ctl.log
