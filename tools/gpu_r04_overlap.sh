#!/bin/bash
# Config 5 with the concurrency hint; its test.
set -o pipefail
T=${1:-r04o}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "concurrency or polled_completion" -x -q --timeout 150 --timeout-method thread > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -n 1 $OUT/t.log
timeout -k 10 300 python3 -u tools/diag/bench_extra.py config5,config5 > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail -20 $OUT/c5.log; exit 1; }
grep -v "amdgpu.ids" $OUT/c5.log
