#!/bin/bash
# One GPU-box check of the committed tree: GPU tests, smoke, the default bench line, the
# self-spawned 2-rank rehearsal bench, and a rocprofv3 kernel-trace summary of the bench.
# Usage (from gpurun): bash tools/gpu_check.sh gpurun_out/<tag> [pytest -k expr]
set -o pipefail
OUT=${1:?out dir}
K=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "gpu tests"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/gputest.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1
fi
rc=$?
tail -3 "$OUT/gputest.log"
case $rc in 0|1) ;; *) step "pytest rc=$rc: stopping"; exit $rc ;; esac
step "smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
step "bench"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
step "bench 2 ranks, self-spawned, one device"
LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline \
  > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err" || exit $?
step "rocprof kernel trace of the bench"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-extra --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
step "done (pytest rc=$rc)"
exit $rc
