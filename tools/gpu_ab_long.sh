#!/bin/bash
# Longer alternating A/B of library variants on the headline shape (libs under _lib/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
BENCH_ARGS="--steps 1000" bash tools/ab_lib.sh "${LIBS:-libold.so libllampc_hip.so libold.so libllampc_hip.so libold.so libllampc_hip.so}" "4"
