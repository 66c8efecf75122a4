#!/bin/bash
# Controller record words + persistent NLP rounds: the controller and setupNLP GPU tests, the
# solve latency, the NLP and controller stamps, and the default bench line.
# usage: tools/gpu_r04_rec.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2; do
  echo "persistent $rep: $(timeout -k 10 120 python -u tools/diag/nlp_solve.py 300 2>/dev/null | tail -1)" | tee -a $OUT/solve.log || exit 1
done
timeout -k 10 120 python -u tools/diag/nlp_phases.py > $OUT/nlp_phases.txt 2>&1 || { tail -5 $OUT/nlp_phases.txt; exit 1; }
cut -c1-250 $OUT/nlp_phases.txt | tail -3
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_phases.txt 2>&1 || { tail -5 $OUT/ctl_phases.txt; exit 1; }
cut -c1-300 $OUT/ctl_phases.txt | grep tick
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > $OUT/timeline_c1.txt 2>&1 || { tail -5 $OUT/timeline_c1.txt; exit 1; }
grep -E "lb_final|final_select|all 157" $OUT/timeline_c1.txt
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('tick', d['ms_per_step']*1e3, 'ctl', d['controller_tick_us'], 'solve', d['solve_us'])"
bash $R/tools/gpu_ab_r04.sh $T prev.so libllampc_hip.so || exit 1
