#!/bin/bash
# Round 6 quick check: the given GPU tests, then (optional) the 2-rank one-device rehearsal bench
# and the default bench line.
# usage (gpurun): [K="<pytest -k expr>"] bash tools/gpu_r06_quick.sh gpurun_out/<tag> "<pytest args>" [g2] [bench]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
if [ -n "$2" ]; then
  step "gpu tests: $2"
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $2 ${K:+-k "$K"} \
    > "$OUT/tests.log" 2>&1
  rc=$?
  tail -4 "$OUT/tests.log"
  [ $rc -eq 0 ] || { step "tests rc=$rc: stopping"; exit $rc; }
fi
shift 2
for what in "$@"; do
  case $what in
    g2) step "bench 2 ranks, self-spawned, one device"
        LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline \
          > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err" || exit $? ;;
    g2host) step "bench 2 ranks, host exchange"
        LLAMPC_EXCHANGE=host LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 \
          --no-cpu-baseline > "$OUT/bench_g2host.json" 2> "$OUT/bench_g2host.err" || exit $? ;;
    bench) step "bench"
        timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $? ;;
    cotenant) step "co-tenant cost of armed launches"
        timeout -k 10 300 python -u tools/diag/cotenant.py 10000 300 "$OUT/cotenant.json" > "$OUT/cotenant.log" 2>&1 || exit $? ;;
    nlp) step "NLP solve latency (bench extra alone)"
        timeout -k 10 300 python -u -c "
import sys, json, argparse; sys.argv=['bench.py']; import bench
print(json.dumps(bench.solve_latency(argparse.Namespace())))" > "$OUT/nlp_solve.json" 2> "$OUT/nlp_solve.err" || exit $? ;;
    k20) step "driver's command"
        timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || exit $? ;;
  esac
done
step "done"
