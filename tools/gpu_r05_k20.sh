#!/bin/bash
# Round 5: where the driver's K = 20 tick loses to K = 200 — the headline command with and
# without the timing events, at K = 20 / 200 / 2000, alternating (bench.py's plan leg only).
# usage (gpurun): bash tools/gpu_r05_k20.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
B="--no-cpu-baseline --no-extra --no-call-latency"
for rep in 1 2; do
  for k in 20 200 2000; do
    for t in "" "--no-timing"; do
      tag="k${k}${t:+_nt}_$rep"
      timeout -k 10 120 python -u bench.py --steps $k --warmup 5 $B $t > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "failed $tag"; tail -5 "$OUT/$tag.err"; exit 1; }
      python3 -c "
import json
d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1])
k=d.get('kernel_us',{}).get('plan')
print('$tag', 'tick', round(d['ms_per_step']*1e3,3), 'kernel', k and round(k,3), 'issue', round(d.get('host_issue_us_per_step',0),2))"
    done
  done
done
echo "[$(date +%T)] done"
