#!/bin/bash
# rocprofv3 kernel trace of the forced 1-rank exchange (peer transport): plan kernel, the
# exchange kernel and the gaps between them.  The rank environment is exported here (no
# launcher under the profiler).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/peerprof
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LLAMPC_FORCE_EXCHANGE=1
export LLAMPC_EXCHANGE=${1:-peer}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peerprof -o $LLAMPC_EXCHANGE -- \
  python3 bench.py --gpus 1 --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-timing \
  > gpurun_out/peerprof/$LLAMPC_EXCHANGE.json 2> gpurun_out/peerprof/$LLAMPC_EXCHANGE.err
