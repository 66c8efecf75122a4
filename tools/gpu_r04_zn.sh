#!/bin/bash
# Controller variates drawn one tick ahead (CtlLaunch.znoise): the controller GPU tests, an
# alternating A/B of the paced two-track step against prev.so, the controller stamps.
# usage: tools/gpu_r04_zn.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py tests/test_gpu_parity.py -k "ctl or controller" -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2 3; do
  echo "new  $rep: $(timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 500 plant 2>/dev/null | grep two-track)" | tee -a $OUT/ab.log || exit 1
  echo "prev $rep: $(LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/prev.so timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 500 plant 2>/dev/null | grep two-track)" | tee -a $OUT/ab.log || exit 1
done
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_phases.txt 2>&1 || { tail -5 $OUT/ctl_phases.txt; exit 1; }
cut -c1-300 $OUT/ctl_phases.txt | grep tick
cut -c150-420 $OUT/ctl_phases.txt | grep -v amdgpu
