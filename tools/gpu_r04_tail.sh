#!/bin/bash
# The paced tick's tail: 2,000 host-pointer ticks at 1 ms under a kernel trace, then the split.
set -o pipefail
T=${1:-r04t}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
  python3 $R/tools/diag/paced_tail.py run $OUT/lat 2000 > $OUT/run.log 2>&1 || { echo "run failed"; tail -20 $OUT/run.log; exit 1; }
grep paced $OUT/run.log
python3 $R/tools/diag/paced_tail.py split $OUT/lat $(find $OUT/prof -name "*kernel_trace.csv" | head -1) | tee $OUT/split.txt
