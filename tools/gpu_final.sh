#!/bin/bash
# Round-end check on one GPU: the full GPU suite, smoke, bench (headline) + its rocprofv3
# kernel trace, and BASELINE config 3 (ETHZMobil, H=40, sudden drop).  && stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_round.sh all && \
timeout -k 10 300 python bench.py --track ETHZMobil --H 40 --scenario sudden --no-extra > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err
rc=$?
python -c "import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]);print('headline', round(d['ms_per_step']*1e3,2),'us/tick', d['value'], 'kernel', d['kernel_us']['plan'], 'sync p50', d['sync_plan_latency_us']['p50'], 'cfg5 p99', d['config5']['p99_us'])"
python -c "import json;d=json.loads(open('gpurun_out/bench_config3.json').read().strip().splitlines()[-1]);print('config3', round(d['ms_per_step']*1e3,2),'us/tick', d['value'], d['result_check'])"
exit $rc
