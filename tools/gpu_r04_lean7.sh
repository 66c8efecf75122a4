#!/bin/bash
# A/B of the 8-term (v8.so) and 7-term (v7.so) lean look-ahead cores, then the GPU parity and
# controller tests on the 7-term library.  usage: tools/gpu_r04_lean7.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
bash $R/tools/gpu_ab_r04.sh $T v8.so v7.so || exit 1
export HIP_FORCE_DEV_KERNARG=1
LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/v7.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ctl_gpu.py -x -v --timeout 150 --timeout-method thread > $OUT/tests_v7.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests_v7.log; exit 1; }
tail -3 $OUT/tests_v7.log
