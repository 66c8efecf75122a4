#!/bin/bash
# Round 5 A/B: HIP's host wait mode (hipSetDeviceFlags before torch's context) on the driver's
# command's plan leg, alternating, K = 20 and 200.
# usage (gpurun): bash tools/gpu_r05_sched.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
B="--no-cpu-baseline --no-extra --no-call-latency"
for rep in 1 2 3; do
  for sch in none spin; do
    for k in 20 200; do
      tag="${sch}_k${k}_$rep"
      if [ "$sch" = none ]; then E=""; else E="LLAMPC_BENCH_SCHED=$sch"; fi
      env $E timeout -k 10 120 python -u bench.py --steps $k --warmup 5 $B > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "failed $tag"; tail -5 "$OUT/$tag.err"; exit 1; }
      python3 -c "
import json
d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1])
print('$tag', 'tick', round(d['ms_per_step']*1e3,3), 'kernel', round(d['kernel_us']['plan'],3))"
    done
  done
done
grep -h hipSetDeviceFlags "$OUT"/*.err | sort | uniq -c
echo "[$(date +%T)] done"
