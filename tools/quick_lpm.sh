#!/bin/bash
# Quick A/B of look-ahead work splits on the headline shape + VALU instruction counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
for L in ${LPMS:-0 4}; do
  LLAMPC_LPM=$L timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/q/b$L.json 2>gpurun_out/q/b$L.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q/b$L.json').read().strip().splitlines()[-1]);print('lpm=$L', round(d['ms_per_step'],4), 'plan_us', round(d['kernel_us']['plan'],1))"
  LLAMPC_LPM=$L timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d gpurun_out/q/p$L -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extra --no-timing ${BENCH_ARGS} > gpurun_out/q/p$L.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/q/p$L 2>&1 | grep -v "^void" | sed "s/^/   lpm=$L /"
done
