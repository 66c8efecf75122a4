#!/bin/bash
# LPM / C / H sweep of the fused tick (no CPU baseline); one JSON line per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sweep.jsonl
: > $out
for C in 1 64; do
  for L in 0 1 2 4; do
    LLAMPC_LPM=$L timeout -k 10 120 python bench.py --C $C --steps 100 --warmup 10 --no-cpu-baseline --no-extra >> $out 2>> gpurun_out/sweep.err || exit 1
  done
done
for H in 40; do
  for L in 0 2 4; do
    LLAMPC_LPM=$L timeout -k 10 120 python bench.py --track ETHZMobil --H $H --steps 100 --warmup 10 --no-cpu-baseline --no-extra >> $out 2>> gpurun_out/sweep.err || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d = json.loads(l)
    c = d["config"]
    print(f'C={c["C"]:3d} H={c["H"]} lpm={d["lpm"]} ms/tick={d["ms_per_step"]:.4f} value={d["value"]:.3e} plan_us={d["kernel_us"]["plan"]:.1f}')
PY
