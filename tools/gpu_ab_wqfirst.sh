#!/bin/bash
# A/B of the work queue's static first units (default build) against every wave taking its
# first unit from the counter (ab_dynfirst.so, -DLLAMPC_WQ_DYN_FIRST) at C = 64, alternating on
# one box; then the work-queue GPU tests on the default build.
# usage (gpurun): bash tools/gpu_ab_wqfirst.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
echo "[$(date +%T)] work-queue tests"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "work_queue or sharded" \
  > "$OUT/wq_tests.log" 2>&1 || { tail -5 "$OUT/wq_tests.log"; exit 1; }
tail -1 "$OUT/wq_tests.log"
for rep in 1 2 3; do
  for lib in libllampc_hip.so ab_dynfirst.so; do
    for N in 10000 3000; do
      LLAMPC_HIP_LIB=$L/$lib timeout -k 10 120 python -u bench.py --C 64 --n-per-gpu $N --steps 100 --warmup 20 \
        --no-cpu-baseline --no-extra --no-call-latency > "$OUT/$lib.$N.$rep.json" 2> "$OUT/$lib.$N.$rep.err" || exit $?
      python -c "import json;d=json.loads(open('$OUT/$lib.$N.$rep.json').read().strip().splitlines()[-1]);print('$lib N=$N rep $rep', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['kernel_us']['plan'],2), d['result_check'])"
    done
  done
done
echo "[$(date +%T)] done"
