#!/bin/bash
# Controller stamps with the look-ahead prologue split.  usage: tools/gpu_r04_pro.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_phases.txt 2>&1 || { tail -5 $OUT/ctl_phases.txt; exit 1; }
cut -c150-420 $OUT/ctl_phases.txt | grep -v amdgpu
