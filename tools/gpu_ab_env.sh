#!/bin/bash
# Alternating A/B of one environment switch on the headline shape (one library).
# usage: tools/gpu_ab_env.sh VAR=value [reps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/abenv
for i in $(seq ${2:-3}); do
  for mode in base env; do
    if [ $mode = env ]; then E="$1"; else E="LLAMPC_AB_NONE=1"; fi
    env $E timeout -k 10 120 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/abenv/$mode.$i.json 2>gpurun_out/abenv/$mode.$i.err || { echo "FAIL $mode"; tail -3 gpurun_out/abenv/$mode.$i.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abenv/$mode.$i.json').read().strip().splitlines()[-1]);print('$mode ($E)', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2), d['result_check'])"
  done
done
