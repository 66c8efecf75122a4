#!/bin/bash
# A/B on the headline: look-back models per lane R = 1 (default) vs LLAMPC_LB_R=2, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ablbr
for i in 1 2 3; do
  for r in 1 2; do
    LLAMPC_LB_R=$r timeout -k 10 120 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra \
      > gpurun_out/ablbr/r$r.$i.json 2> gpurun_out/ablbr/r$r.$i.err || { tail -3 gpurun_out/ablbr/r$r.$i.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ablbr/r$r.$i.json').read().strip().splitlines()[-1]);print('R=$r', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2), d['result_check'])"
  done
done
