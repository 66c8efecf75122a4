#!/bin/bash
# Multi-rank rehearsal on one GPU: 2 ranks, records gathered over gloo, merged on the device
# (the N > 1 bench flow; RCCL refuses two ranks on one device).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 200 --warmup 10 \
  --no-cpu-baseline > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -20 gpurun_out/rehearse2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/rehearse2.json').read().strip().splitlines()[-1]);print('2-rank gloo rehearsal', round(d['ms_per_step']*1e3,1), 'us/tick', d['result_check'], d['exchange'], 'C64', d.get('C64',{}).get('ms_per_step'))"
