#!/bin/bash
# Kernel trace of short and long headline runs: per-dispatch durations and gaps show how the
# first ticks after the warmup differ from the steady state.  usage: bash tools/gpu_ramp_trace.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/$OUT"
export TMPDIR=/tmp
cd /tmp
for cfg in "5 20" "5 2000"; do
  set -- $cfg
  echo "[$(date +%T)] trace warmup $1 steps $2"
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/w$1_s$2" -o run -- \
    python3 "$R/bench.py" --warmup $1 --steps $2 --no-extra --no-cpu-baseline --no-call-latency \
    > "$R/$OUT/w$1_s$2.json" 2> "$R/$OUT/w$1_s$2.err" || exit $?
done
echo "[$(date +%T)] done"
