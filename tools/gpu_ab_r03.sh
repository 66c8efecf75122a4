#!/bin/bash
# Round-3 A/B: GPU tests on the new library, then alternating headline (C=1) and C=64 runs of
# libold.so (previous build) vs libllampc_hip.so (new build) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
OUT=${1:-gpurun_out/ab_r03}; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
BENCH_ARGS="--steps 1000" bash tools/ab_lib.sh "${LIBS:-libold.so libllampc_hip.so libold.so libllampc_hip.so libold.so libllampc_hip.so}" "4" > $OUT/ab_c1.log 2>&1 || { cat $OUT/ab_c1.log; exit 1; }
cat $OUT/ab_c1.log
BENCH_ARGS="--C 64 --steps 100" bash tools/ab_lib.sh "${LIBS64:-libold.so libllampc_hip.so libold.so libllampc_hip.so}" "1" > $OUT/ab_c64.log 2>&1 || { cat $OUT/ab_c64.log; exit 1; }
cat $OUT/ab_c64.log
