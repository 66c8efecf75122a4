#!/bin/bash
# The plan kernel's completion tail: GPU tests, the C = 1 stamps timeline, an alternating A/B
# (headline K = 200 and the driver's K = 20) against prev.so.  usage: tools/gpu_r04_tail.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > $OUT/timeline_c1.txt 2>&1 || { tail -5 $OUT/timeline_c1.txt; exit 1; }
grep -E "lb_final|final_select|all 157" $OUT/timeline_c1.txt
for rep in 1 2 3; do
  for lib in prev.so libllampc_hip.so; do
    for cfg in "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
      LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/$lib timeout -k 10 120 python -u bench.py $cfg --no-extra --no-cpu-baseline --no-call-latency > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('$rep $lib $cfg', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['kernel_us']['plan'],2))" | tee -a $OUT/ab.log
    done
  done
done
