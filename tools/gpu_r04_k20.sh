#!/bin/bash
# Per-dispatch durations of the driver's command (K = 20, W = 5) under a kernel trace.
set -o pipefail
T=${1:-r04k20}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-call-latency > $OUT/b.json 2> $OUT/b.err || { echo "failed"; tail -20 $OUT/b.err; exit 1; }
python3 $R/tools/diag/trace_list.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) plan_kernel 30
python3 -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('ms_per_step', d['ms_per_step']*1e3, 'kernel', d['kernel_us']['plan'])"
