#!/bin/bash
# Round 5 check after armed controller ticks: the GPU tests, smoke(), the default bench line
# (its controller_tick_us extra runs armed ticks) and the driver's command.
# usage (gpurun): bash tools/gpu_r05e.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
echo "[$(date +%T)] gpu tests"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
tail -2 "$OUT/gputest.log"
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -10 "$OUT/smoke.log"; exit 1; }
echo "[$(date +%T)] bench (default)"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -10 "$OUT/bench_default.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1])
print('tick', round(d['ms_per_step']*1e3,2), 'us; kernel', round(d['kernel_us']['plan'],2))
c=d.get('controller_tick_us') or {}
print('controller p50/p99/max', c.get('p50'), c.get('p99'), c.get('max'), 'kernel', c.get('kernel_us_avg'), 'device', (c.get('device_us') or {}).get('armed'))
s=d.get('solve_us') or {}
print('solve p50', s.get('p50'))
"
echo "[$(date +%T)] bench (driver)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || { echo "bench k20 failed"; tail -10 "$OUT/bench_k20.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench_k20.json').read().strip().splitlines()[-1])
print('K20 tick', round(d['ms_per_step']*1e3,2), 'us; kernel', round(d['kernel_us']['plan'],2), 'ctl', (d.get('controller_tick_us') or {}).get('p50'))"
echo "[$(date +%T)] done"
