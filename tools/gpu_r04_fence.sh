#!/bin/bash
# The controller tick's record phase: ctl_phases with the system fence (stamps build) and
# with a plain vmcnt wait in its place (diagnostic ctlwc.so).  usage: tools/gpu_r04_fence.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_fence.txt 2>&1 || { tail -5 $OUT/ctl_fence.txt; exit 1; }
LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/ctlwc.so timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_waitcnt.txt 2>&1 || { tail -5 $OUT/ctl_waitcnt.txt; exit 1; }
cut -c1-260 $OUT/ctl_fence.txt $OUT/ctl_waitcnt.txt
