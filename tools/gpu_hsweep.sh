#!/bin/bash
# Tick time vs horizon H and bank size N (fixed overhead = the intercept), one GPU call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/hsweep
for N in ${NS:-10 10000}; do
  for H in ${HS:-1 2 5 10 20}; do
    timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra --n-per-gpu $N --H $H > gpurun_out/hsweep/$N.$H.json 2>gpurun_out/hsweep/$N.$H.err || { echo "FAIL $N $H"; tail -3 gpurun_out/hsweep/$N.$H.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/hsweep/$N.$H.json').read().strip().splitlines()[-1]);print('N=$N H=$H', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2))"
  done
done
