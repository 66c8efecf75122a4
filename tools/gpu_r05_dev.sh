#!/bin/bash
# Round 5: the controller's device time (llampc_ctl_device_us): the prelaunch tests, then the
# default bench line (controller_tick_us.device_us).
# usage (gpurun): bash tools/gpu_r05_dev.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
echo "[$(date +%T)] ctl tests"
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ctltest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/ctltest.log"; exit 1; }
tail -2 "$OUT/ctltest.log"
echo "[$(date +%T)] bench"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -10 "$OUT/bench.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
c=d['controller_tick_us']
print('tick', round(d['ms_per_step']*1e3,2), 'ctl p50/p99', round(c['p50'],1), round(c['p99'],1), 'kernel', c['kernel_us_avg'])
print('device_us', json.dumps(c['device_us']))"
echo "[$(date +%T)] done"
