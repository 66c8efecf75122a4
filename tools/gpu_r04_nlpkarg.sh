#!/bin/bash
# setupNLP inputs as kernel arguments (no H2D before the launch): the NLP GPU tests, then an
# alternating A/B of the solve latency against prev.so, and the kernel trace of the solves.
# usage: tools/gpu_r04_nlpkarg.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nlp or solve" -x -v --timeout 150 --timeout-method thread > $OUT/nlp_tests.log 2>&1 || { echo "nlp tests failed"; tail -30 $OUT/nlp_tests.log; exit 1; }
tail -1 $OUT/nlp_tests.log
for rep in 1 2 3; do
  echo "new  $rep: $(timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 2>/dev/null | tail -1)" | tee -a $OUT/ab.log || exit 1
  echo "prev $rep: $(LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/prev.so timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 2>/dev/null | tail -1)" | tee -a $OUT/ab.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/tools/diag/nlp_solve.py 60 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
