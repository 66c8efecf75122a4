set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06z
for rep in 1 2 3; do
  for k in 1 0; do
    HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python -u -c "
import sys, json, argparse; sys.argv=['bench.py']; import bench
r = bench.solve_latency(argparse.Namespace()); print(json.dumps({'k': $k, 'p50': r['p50'], 'p99': r['p99'], 'kernel': r['kernel_us_avg']}))" >> gpurun_out/r06z/kernarg.txt 2>/dev/null || exit $?
  done
done
cat gpurun_out/r06z/kernarg.txt
