#!/bin/bash
# Persistent NLP rounds: the setupNLP GPU tests, solve latency with every round in one launch
# vs one launch per round (LLAMPC_NLP_ROUND_LAUNCHES=1, alternating), the NLP stamps, and the
# controller record phase with the system fence vs a vmcnt wait (ctlwc.so).
# usage: tools/gpu_r04_nlpp.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nlp or solve" -x -v --timeout 150 --timeout-method thread > $OUT/nlp_tests.log 2>&1 || { echo "nlp tests failed"; tail -30 $OUT/nlp_tests.log; exit 1; }
tail -2 $OUT/nlp_tests.log
for rep in 1 2 3; do
  echo "persistent $rep: $(timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 2>/dev/null | tail -1)" | tee -a $OUT/solve_ab.log || exit 1
  echo "per-round  $rep: $(LLAMPC_NLP_ROUND_LAUNCHES=1 timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 2>/dev/null | tail -1)" | tee -a $OUT/solve_ab.log || exit 1
done
timeout -k 10 120 python -u tools/diag/nlp_phases.py > $OUT/nlp_phases.txt 2>&1 || { tail -5 $OUT/nlp_phases.txt; exit 1; }
cut -c1-250 $OUT/nlp_phases.txt | tail -3
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_fence.txt 2>&1 || { tail -5 $OUT/ctl_fence.txt; exit 1; }
LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/ctlwc.so timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_waitcnt.txt 2>&1 || { tail -5 $OUT/ctl_waitcnt.txt; exit 1; }
cut -c1-300 $OUT/ctl_fence.txt $OUT/ctl_waitcnt.txt | grep tick
