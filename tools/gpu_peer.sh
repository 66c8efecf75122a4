#!/bin/bash
# Peer (xGMI mailbox) exchange on a one-GPU box: its GPU tests, the forced 1-rank exchange
# bench per transport (nccl group; peer = fused into the plan launch, peer_split = second
# kernel), the 2-rank same-device rehearsal, and an A/B of the headline (N=1, no exchange)
# against libold.so.  Every GPU step has its own limit; && stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/peer
O=gpurun_out/peer
tr1() {  # $1 transport [$2 tag]  (env LLAMPC_PEER_SPLIT passes through)
  LLAMPC_FORCE_EXCHANGE=1 LLAMPC_EXCHANGE=$1 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 1 --steps 2000 --warmup 50 \
    --no-cpu-baseline --no-extra > $O/force1_${2:-$1}.json 2> $O/force1_${2:-$1}.err
}
rh2() {  # $1 transport
  LLAMPC_EXCHANGE=$1 LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 240 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 2 --steps 1000 \
    --warmup 20 --no-cpu-baseline --no-extra > $O/rehearse2_$1.json 2> $O/rehearse2_$1.err
}
split() { LLAMPC_PEER_SPLIT=1 tr1 peer peer_split; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_exchange_gpu.py \
  tests/test_sharded_gpu.py > $O/pytest.log 2>&1 && \
tr1 peer && split && tr1 rccl && tr1 peer peer_b && LLAMPC_PEER_SPLIT=1 tr1 peer peer_split_b && tr1 rccl rccl_b && \
rh2 peer && \
LIBS="libold.so libllampc_hip.so libold.so libllampc_hip.so libold.so libllampc_hip.so" bash tools/gpu_ab_long.sh > $O/ab.txt 2>&1
rc=$?
tail -3 $O/pytest.log
cat $O/ab.txt
for f in $O/*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step']*1e3,2),'us/tick', d['kernel_us']['plan'], d['result_check'])" 2>/dev/null; done
exit $rc
