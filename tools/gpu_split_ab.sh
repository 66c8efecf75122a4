#!/bin/bash
# GPU tests, then an alternating A/B of the previous library (libold.so) against the current
# one on the headline shape, then the multi-rank rehearsal's timing path (sampled events).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log && \
bash tools/ab_lib.sh "libold.so libllampc_hip.so libold.so libllampc_hip.so libold.so libllampc_hip.so" "4"
