#!/bin/bash
# Round-3 (session 2) A/B: full GPU tests on the new library, alternating C=1 and C=64 runs of
# libold.so vs libllampc_hip.so, then the work-queue unit stamps (stamps build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
OUT=${1:?out dir}; mkdir -p $OUT gpurun_out/ab
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
BENCH_ARGS="--steps 1000" timeout -k 10 300 bash tools/ab_lib.sh "${LIBS:-libold.so libllampc_hip.so libold.so libllampc_hip.so}" "4" > $OUT/ab_c1.log 2>&1 || { cat $OUT/ab_c1.log; exit 1; }
cat $OUT/ab_c1.log
BENCH_ARGS="--C 64 --steps 100" timeout -k 10 300 bash tools/ab_lib.sh "${LIBS64:-libold.so libllampc_hip.so libold.so libllampc_hip.so}" "1" > $OUT/ab_c64.log 2>&1 || { cat $OUT/ab_c64.log; exit 1; }
cat $OUT/ab_c64.log
if [ -n "$WQ_DIAG" ]; then
  timeout -k 10 120 python -u tools/diag/wq_units.py 10000 64 > $OUT/wq_units.txt 2>&1 || { tail -5 $OUT/wq_units.txt; exit 1; }
  cat $OUT/wq_units.txt
fi
