#!/bin/bash
# A/B of a runtime environment variable on the headline bench (same library), alternating.
# usage: VAR=HIP_FORCE_DEV_KERNARG VALS="0 1 0 1" bash tools/gpu_ab_env_r03.sh gpurun_out/<tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_env}; mkdir -p $OUT
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra --no-call-latency ${BENCH_ARGS} > $OUT/$VAR.$v.json 2>$OUT/$VAR.$v.err || { echo "FAIL $v"; tail -3 $OUT/$VAR.$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$VAR.$v.json').read().strip().splitlines()[-1]);print('$VAR=$v', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2))"
done
