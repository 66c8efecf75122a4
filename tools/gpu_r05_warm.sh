#!/bin/bash
# Round 5: final_poll's dry pass through the record code (a warm instruction cache for the
# C = 1 tail) against the previous build: the GPU parity tests on the new library, the stamps
# timeline of one C = 1 tick per build, then alternating headline bench runs (the repo's
# default 400-step run and the driver's 20-step run) per build.
# usage (gpurun): bash tools/gpu_r05_warm.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
echo "[$(date +%T)] gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
tail -2 "$OUT/gputest.log"
for s in base_r05_stamps libllampc_hip_stamps; do
  LLAMPC_HIP_LIB=$L/$s.so timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_$s.txt" 2>&1 || { echo "timeline $s failed"; tail -5 "$OUT/timeline_$s.txt"; exit 1; }
done
for rep in 1 2 3; do
  for lib in base_r05 libllampc_hip; do
    LLAMPC_HIP_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-call-latency \
      > "$OUT/bench_$lib.$rep.json" 2> "$OUT/bench_$lib.$rep.err" || { echo "bench $lib failed"; tail -3 "$OUT/bench_$lib.$rep.err"; exit 1; }
    LLAMPC_HIP_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-call-latency \
      > "$OUT/bench20_$lib.$rep.json" 2> "$OUT/bench20_$lib.$rep.err" || { echo "bench20 $lib failed"; tail -3 "$OUT/bench20_$lib.$rep.err"; exit 1; }
    python3 -c "
import json
a=json.loads(open('$OUT/bench_$lib.$rep.json').read().strip().splitlines()[-1])
b=json.loads(open('$OUT/bench20_$lib.$rep.json').read().strip().splitlines()[-1])
print('$lib rep $rep', 'K400', round(a['ms_per_step']*1e3,2), 'us/tick kernel', round(a['kernel_us']['plan'],2), '| K20', round(b['ms_per_step']*1e3,2), 'kernel', round(b['kernel_us']['plan'],2), a['result_check'])"
  done
done
echo "[$(date +%T)] done"
