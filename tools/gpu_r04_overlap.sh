#!/bin/bash
# The controller step after k other banks; ctl tests; headline bench without extras.
set -o pipefail
T=${1:-r04o}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
for v in bank,bank,controller controller bank,controller; do
  timeout -k 10 300 python3 -u tools/diag/bench_extra.py $v >> $OUT/extras.log 2>&1 || { echo "variant $v failed"; tail -20 $OUT/extras.log; exit 1; }
  echo "-- $v" >> $OUT/extras.log
done
grep -v "amdgpu.ids\|^bank\|^headline" $OUT/extras.log
timeout -k 10 300 python -u -m pytest tests/test_ctl_gpu.py -x -q --timeout 150 --timeout-method thread > $OUT/ctl.log 2>&1 || { echo "ctl tests failed"; tail -30 $OUT/ctl.log; exit 1; }
tail -n 1 $OUT/ctl.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/b20.json 2>$OUT/b20.err || { echo "bench failed"; tail -20 $OUT/b20.err; exit 1; }
timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline > $OUT/b200.json 2>$OUT/b200.err || { echo "bench failed"; tail -20 $OUT/b200.err; exit 1; }
python3 -c "
import json
for f in ('b20','b200'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['ms_per_step']*1e3, d['kernel_us']['plan'], d['host_issue_us_per_step'])"
