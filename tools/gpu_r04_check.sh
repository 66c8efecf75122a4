#!/bin/bash
# Round-4 GPU check: controller-tick tests, the full GPU suite, then the default bench.
# usage: tools/gpu_r04_check.sh <tag> [pytest -k expr]
set -o pipefail
T=${1:-r04}
OUT=gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 420 python -u -m pytest tests/test_ctl_gpu.py -x -v --timeout 150 --timeout-method thread > $OUT/ctl.log 2>&1 || { echo "ctl tests failed"; tail -30 $OUT/ctl.log; exit 1; }
tail -3 $OUT/ctl.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --deselect tests/test_ctl_gpu.py > $OUT/gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu.log; exit 1; }
tail -3 $OUT/gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value',d['value'],'ms',d['ms_per_step'],'kernel_us',d['kernel_us'])
for k in ('controller_tick_us','config5','config3','C64','paced_plan_latency_us'):
    print(k, json.dumps(d.get(k))[:600])
"
