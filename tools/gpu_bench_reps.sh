#!/bin/bash
# Headline bench repeated at the driver's K/W and at the defaults, plus a rocprofv3 kernel-trace
# summary of the default run.  usage (gpurun): bash tools/gpu_bench_reps.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/$OUT"
cd "$R"
for cfg in "5 20" "20 200" "5 20" "20 200" "5 20" "2000 2000"; do
  set -- $cfg
  echo "[$(date +%T)] warmup $1 steps $2"
  timeout -k 10 120 python -u bench.py --warmup $1 --steps $2 --no-extra --no-cpu-baseline --no-call-latency \
    >> "$OUT/reps.jsonl" 2>> "$OUT/reps.err" || exit $?
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- \
  python3 "$R/bench.py" --no-extra --no-cpu-baseline > "$R/$OUT/prof_bench.json" 2>&1 || exit $?
echo "[$(date +%T)] done"
