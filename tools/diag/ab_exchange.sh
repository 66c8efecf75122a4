#!/bin/bash
# A/B of the N>1 tick's exchange transport on ONE GPU (forced exchange on a 1-rank RCCL
# group): native llampc_exchange_device vs the c10d all_gather_into_tensor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/abx
port=29551
for rep in 1 2; do
  for mode in native c10d; do
    port=$((port+1))
    if [ $mode = c10d ]; then export LLAMPC_C10D_EXCHANGE=1; else unset LLAMPC_C10D_EXCHANGE; fi
    LLAMPC_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra \
      > gpurun_out/abx/$mode.$rep.json 2> gpurun_out/abx/$mode.$rep.err || { echo "FAIL $mode"; tail -5 gpurun_out/abx/$mode.$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abx/$mode.$rep.json').read().strip().splitlines()[-1]);print('$mode', round(d['ms_per_step']*1e3,2), 'us/tick; plan', round(d['kernel_us']['plan'],2), 'host issue', round(d['host_issue_us_per_step'],2), d['result_check'])"
  done
done
