#!/bin/bash
# A/B of the bench procedure (bench_ab_old.py: events created between the warmup and the timed
# loop; bench.py: before the warmup) at the driver's K = 20, W = 5 and at the defaults,
# alternating on one box.  usage (gpurun): bash tools/gpu_ab_bench_gap.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for rep in 1 2 3 4; do
  for b in bench_ab_old.py bench.py; do
    for cfg in "5 20" "20 200"; do
      set -- $cfg
      timeout -k 10 120 python -u $b --warmup $1 --steps $2 --no-extra --no-cpu-baseline --no-call-latency \
        > "$OUT/$b.$1.$rep.json" 2> "$OUT/$b.$1.$rep.err" || exit $?
      python -c "import json;d=json.loads(open('$OUT/$b.$1.$rep.json').read().strip().splitlines()[-1]);print('$b W=$1 K=$2 rep $rep', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['kernel_us']['plan'],2), d['kernel_us']['events'])"
    done
  done
done
