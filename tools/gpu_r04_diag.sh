#!/bin/bash
# Round-4 diagnostics on one GPU: controller phase stamps, the controller tests, a kernel
# trace of setupNLP.solve.  usage: tools/gpu_r04_diag.sh <tag>
set -o pipefail
T=${1:-r04d}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 6 > $OUT/ctl_phases.log 2>&1 || { echo "ctl_phases failed"; tail -30 $OUT/ctl_phases.log; exit 1; }
cat $OUT/ctl_phases.log
timeout -k 10 420 python -u -m pytest tests/test_ctl_gpu.py -x -v --timeout 150 --timeout-method thread > $OUT/ctl.log 2>&1 || { echo "ctl tests failed"; tail -30 $OUT/ctl.log; exit 1; }
tail -n 2 $OUT/ctl.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k setupnlp -x -v --timeout 150 --timeout-method thread > $OUT/nlp_tests.log 2>&1 || { echo "nlp tests failed"; tail -30 $OUT/nlp_tests.log; exit 1; }
tail -n 2 $OUT/nlp_tests.log
timeout -k 10 120 python -u tools/diag/nlp_phases.py > $OUT/nlp_phases.log 2>&1 || { echo "nlp_phases failed"; tail -30 $OUT/nlp_phases.log; exit 1; }
cat $OUT/nlp_phases.log
timeout -k 10 120 python -u tools/diag/nlp_solve.py 100 > $OUT/nlp.log 2>&1 || { echo "nlp failed"; tail -30 $OUT/nlp.log; exit 1; }
cat $OUT/nlp.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_nlp" -o run -- \
  python3 $R/tools/diag/nlp_solve.py 100 > $OUT/nlp_prof.log 2>&1 || { echo "nlp prof failed"; tail -30 $OUT/nlp_prof.log; exit 1; }
find $OUT/prof_nlp -name "*stats*" | head
