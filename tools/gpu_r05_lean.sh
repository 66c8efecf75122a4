#!/bin/bash
# Round 5: the look-ahead's lean-core length against the accuracy on the configs' own inputs
# (config 3's Mobil scenario states are ill-conditioned: a 1-ulp change of x0 moves some costs
# by ~1e-8 relative) and the headline tick: per library (7 / 8 / 9 terms) the accuracy
# diagnostic, then alternating bench runs of the headline tick.
# usage (gpurun): bash tools/gpu_r05_lean.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
for lib in libllampc_hip lean8 lean9; do
  echo "[$(date +%T)] accuracy $lib"
  LLAMPC_HIP_LIB=$L/$lib.so timeout -k 10 400 python -u tools/diag/accuracy_headroom.py "$OUT/acc_$lib.json" \
    c3_scenario,c2_scenario,c1_h40,c1_h20,c64_h20,wide > "$OUT/acc_$lib.log" 2>&1 || { echo "accuracy $lib failed"; tail -5 "$OUT/acc_$lib.log"; exit 1; }
  cat "$OUT/acc_$lib.log" | grep shape | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  $lib', d['shape'], 'max', d['cost']['max'], 'p99.9', d['cost']['p99_9'], 'cond', d.get('worst_conditioning',{}).get('ulp_x0_rel_change'))"
done
for rep in 1 2; do
  for lib in libllampc_hip lean8 lean9; do
    LLAMPC_HIP_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-call-latency \
      > "$OUT/bench_$lib.$rep.json" 2> "$OUT/bench_$lib.$rep.err" || { echo "bench $lib failed"; tail -3 "$OUT/bench_$lib.$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_$lib.$rep.json').read().strip().splitlines()[-1]);print('$lib rep $rep', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['kernel_us']['plan'],2))"
  done
done
for lib in libllampc_hip lean8 lean9; do
  LLAMPC_HIP_LIB=$L/$lib.so timeout -k 10 120 python bench.py --C 64 --steps 60 --warmup 5 --no-cpu-baseline --no-extra --no-call-latency \
    > "$OUT/bench64_$lib.json" 2> "$OUT/bench64_$lib.err" || { echo "bench64 $lib failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench64_$lib.json').read().strip().splitlines()[-1]);print('$lib C=64', round(d['ms_per_step']*1e3,2), 'us/tick')"
done
echo "[$(date +%T)] done"
