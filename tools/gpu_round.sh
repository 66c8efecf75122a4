#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; steps chained with && (stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGE=${1:-all}
run_tests() { timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; }
run_bench() { timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; }
run_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-timing > gpurun_out/prof.log 2>&1
}
case "$STAGE" in
  tests) run_tests ;;
  all) run_tests && run_smoke && run_bench && run_prof ;;
  bench) run_bench && run_prof ;;
  *) echo "unknown stage $STAGE"; exit 2 ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc"
tail -5 gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
