#!/bin/bash
# Sharded/exchange tests (ExternalStream on the bank's own stream), NLP tests + latency +
# phases, then the K = 20 per-dispatch trace.
set -o pipefail
T=${1:-r04c}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/${T}
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_exchange_gpu.py -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/${T}/sharded.log 2>&1 || { echo "sharded tests failed"; tail -30 $R/gpurun_out/${T}/sharded.log; exit 1; }
tail -n 1 $R/gpurun_out/${T}/sharded.log
bash tools/gpu_r04_nlp.sh ${T}_nlp || exit $?
bash tools/gpu_r04_k20.sh ${T}_k20 || exit $?
