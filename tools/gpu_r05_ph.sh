set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05ph
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 4 prelaunch > gpurun_out/r05ph/phases_armed.txt 2>&1 || { tail -5 gpurun_out/r05ph/phases_armed.txt; exit 1; }
cat gpurun_out/r05ph/phases_armed.txt
