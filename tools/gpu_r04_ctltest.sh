#!/bin/bash
set -o pipefail
T=${1:-r04ct}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 420 python -u -m pytest tests/test_ctl_gpu.py -x -v --timeout 150 --timeout-method thread > $OUT/ctl.log 2>&1 || { echo "ctl tests failed"; tail -40 $OUT/ctl.log; exit 1; }
grep -E "PASS|FAIL" $OUT/ctl.log | tail -12
