#!/bin/bash
# Round 6: the tests of the changed paths first (sharded controller over every transport, the
# exchange transports, the self-spawned bench), then the whole GPU suite + smoke + bench.
# usage (gpurun): bash tools/gpu_r06_focus.sh gpurun_out/<tag> [pytest -k expr]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
step "focused gpu tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_sharded_ctl_gpu.py tests/test_exchange_gpu.py "tests/test_sharded_gpu.py::test_bench_spawns_its_own_ranks" \
  ${2:+-k "$2"} > "$OUT/focus.log" 2>&1
rc=$?
tail -5 "$OUT/focus.log"
[ $rc -eq 0 ] || { step "focused rc=$rc: stopping"; exit $rc; }
bash tools/gpu_check.sh "$OUT" || exit $?
step "driver's command"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || exit $?
step "all done"
