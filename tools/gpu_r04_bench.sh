#!/bin/bash
# The default bench line (N=1) and its extras.  usage: tools/gpu_r04_bench.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('tick', round(d['ms_per_step']*1e3,2), 'ctl', {k:v for k,v in d['controller_tick_us'].items() if k in ('p50','p99','max','kernel_us_avg','host_split_us_p50')}, 'solve', d['solve_us']['p50'])"
