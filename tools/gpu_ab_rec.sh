#!/bin/bash
# A/B of libold.so vs libllampc_hip.so: exchange/sharded GPU tests on the new library, the
# headline tick, and the forced 1-rank fused peer exchange (torch.distributed.run, nccl group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=${1:?out}; mkdir -p $O gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_exchange_gpu.py \
  tests/test_sharded_gpu.py tests/test_gpu_parity.py -k "exchange or sharded or polled or ticket or host_completion or closed_loop" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in libold.so libllampc_hip.so libold.so libllampc_hip.so libold.so libllampc_hip.so; do
  LLAMPC_HIP_LIB=$PWD/lla-mpc_amd/llampc/_lib/$lib timeout -k 10 120 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra > $O/c1_$lib.json 2>$O/c1.err || exit 1
  LLAMPC_HIP_LIB=$PWD/lla-mpc_amd/llampc/_lib/$lib LLAMPC_FORCE_EXCHANGE=1 LLAMPC_EXCHANGE=peer timeout -k 10 180 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 1 --steps 2000 --warmup 50 \
    --no-cpu-baseline --no-extra > $O/px_$lib.json 2> $O/px.err || { tail -5 $O/px.err; exit 1; }
  python3 -c "
import json
a=json.loads(open('$O/c1_$lib.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/px_$lib.json').read().strip().splitlines()[-1])
print('$lib', 'plain', round(a['ms_per_step']*1e3,2), 'us/tick; forced peer exchange', round(b['ms_per_step']*1e3,2), 'us/tick', b['config'].get('transport'), b['result_check'])"
done
