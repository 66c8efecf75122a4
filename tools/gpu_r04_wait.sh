#!/bin/bash
# The driver's command (K = 20, W = 5) with HIP's default host wait and with a longer active
# (spinning) wait before the interrupt-based one (ROC_ACTIVE_WAIT_TIMEOUT), alternating.
set -o pipefail
T=${1:-r04w}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
for rep in 1 2 3; do
  for v in default 100000; do
    if [ $v = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$v; fi
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err || { echo "FAIL $v"; tail -5 $OUT/$v.$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/$v.$rep.json').read().strip().splitlines()[-1]);print('$rep $v', round(d['ms_per_step']*1e3,2), 'kernel', round(d['kernel_us']['plan'],2), 'call p50', round(d['plan_call_us']['p50'],2))" | tee -a $OUT/ab.log
  done
done
