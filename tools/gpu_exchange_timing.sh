#!/bin/bash
# The N > 1 tick (forced exchange on a 1-rank RCCL group, native all-gather + merge) with
# the sampled plan-kernel events vs no events at all: what the timing costs the timed loop.
# Then the 2-rank gloo rehearsal of the bench flow.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/xt
port=29561
for rep in 1 2; do
  for mode in sampled none; do
    port=$((port+1))
    extra=""; [ $mode = none ] && extra="--no-timing"
    LLAMPC_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --steps 800 --warmup 40 --no-cpu-baseline --no-extra $extra \
      > gpurun_out/xt/$mode.$rep.json 2> gpurun_out/xt/$mode.$rep.err || { echo "FAIL $mode"; tail -5 gpurun_out/xt/$mode.$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/xt/$mode.$rep.json').read().strip().splitlines()[-1]);print('$mode', round(d['ms_per_step']*1e3,2), 'us/tick; plan', round(d['kernel_us']['plan'],2), d['kernel_us']['bracket'], d['result_check'])"
  done
done
bash tools/gpu_rehearse.sh
