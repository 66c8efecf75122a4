#!/bin/bash
# NLP tests, phases and latency.
set -o pipefail
T=${1:-r04n}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "setupnlp or nlp" -x -q --timeout 150 --timeout-method thread > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -n 1 $OUT/t.log
timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 > $OUT/nlp.log 2>&1 || { echo "nlp failed"; tail -20 $OUT/nlp.log; exit 1; }
grep solve $OUT/nlp.log
timeout -k 10 120 python -u tools/diag/nlp_phases.py > $OUT/nlp_phases.log 2>&1 || { echo "phases failed"; tail -20 $OUT/nlp_phases.log; exit 1; }
grep solve $OUT/nlp_phases.log | tail -2
