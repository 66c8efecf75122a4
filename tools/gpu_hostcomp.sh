#!/bin/bash
# GPU tests + host-latency probe with and without host completion + default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log && \
timeout -k 10 120 ./tools/micro/host_latency > gpurun_out/hl_host.jsonl 2>&1 && cat gpurun_out/hl_host.jsonl && \
LLAMPC_SYNC_COMPLETION=1 timeout -k 10 120 ./tools/micro/host_latency > gpurun_out/hl_sync.jsonl 2>&1 && grep "\"plan\"" gpurun_out/hl_sync.jsonl && LLAMPC_NO_INLINE=1 timeout -k 10 120 ./tools/micro/host_latency > gpurun_out/hl_noinl.jsonl 2>&1 && grep "\"plan\"" gpurun_out/hl_noinl.jsonl && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && python -c "
import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('tick us', round(d['ms_per_step']*1e3,2), 'plan us', round(d['kernel_us']['plan'],2), 'sync', d.get('sync_plan_latency_us'), 'cfg5', d.get('config5'))"
