#!/bin/bash
# Full GPU test suite on the current library, then the long alternating A/B against libold.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  && bash tools/gpu_ab_long.sh > gpurun_out/ab.txt 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/ab.txt
exit $rc
