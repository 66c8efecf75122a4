#!/bin/bash
# Builds tools/micro/step_bench in ablation variants (diagnostic only).
set -e
D=$(cd "$(dirname "$0")" && pwd)
for v in full NODIV NOPSI NODPP NOPOLY; do
  def=""; [ "$v" != full ] && def="-DLLAMPC_ABL_$v"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm $def -DVARIANT="\"$v\"" \
     -I$D/../../lla-mpc_amd/csrc -I$D/../../include -o $D/step_$v $D/step_bench.hip
done
