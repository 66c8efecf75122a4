#!/bin/bash
# Round 5: the NLP solve with a completion block and tagged hand-offs — its GPU tests, the
# round phases (stamps build) and the default bench line (solve_us).
# usage (gpurun): bash tools/gpu_r05_nlp.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
echo "[$(date +%T)] nlp tests"
timeout -k 10 400 python -u -m pytest tests -m gpu -k "nlp or setupnlp" -x -q --timeout 120 --timeout-method thread > "$OUT/nlptest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/nlptest.log"; exit 1; }
tail -2 "$OUT/nlptest.log"
echo "[$(date +%T)] phases"
timeout -k 10 200 python -u tools/diag/nlp_phases.py > "$OUT/phases.txt" 2>&1 || { echo "phases failed"; tail -10 "$OUT/phases.txt"; exit 1; }
cat "$OUT/phases.txt"
echo "[$(date +%T)] bench"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -10 "$OUT/bench.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
s=d['solve_us']
print('tick', round(d['ms_per_step']*1e3,2), 'solve p50/p99', round(s['p50'],1), round(s['p99'],1), 'kernel', round(s['kernel_us_avg'],1))"
echo "[$(date +%T)] done"
