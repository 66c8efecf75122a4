#!/bin/bash
# Round 5: controller tail changes — the ctl GPU tests, the armed phases (stamps build), the
# paced two-track step (three alternating runs: prelaunch with spec) and the default bench line.
# usage (gpurun): bash tools/gpu_r05_ctlx.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
echo "[$(date +%T)] ctl tests"
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ctltest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/ctltest.log"; exit 1; }
tail -1 "$OUT/ctltest.log"
echo "[$(date +%T)] phases"
timeout -k 10 200 python -u tools/diag/ctl_phases.py 10000 6 prelaunch > "$OUT/phases.txt" 2>&1 || { echo "phases failed"; tail -5 "$OUT/phases.txt"; exit 1; }
grep "paced" "$OUT/phases.txt" | head -3 | cut -c1-420
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/diag/ctl_two_tracks.py 10000 1000 plant prelaunch > "$OUT/two.$i.txt" 2>&1 || { echo "two-track failed"; tail -5 "$OUT/two.$i.txt"; exit 1; }
  tail -1 "$OUT/two.$i.txt"
done
echo "[$(date +%T)] bench"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -10 "$OUT/bench.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
c=d['controller_tick_us']
print('tick', round(d['ms_per_step']*1e3,2), 'ctl p50/p99', round(c['p50'],1), round(c['p99'],1), 'device', json.dumps(c['device_us']['armed']))"
echo "[$(date +%T)] done"
