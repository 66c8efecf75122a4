#!/bin/bash
# Builds tools/micro/quad_bench in variants (diagnostic only): ROLL=1/2.
set -e
D=$(cd "$(dirname "$0")" && pwd)
build() {  # name, flags
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm $2 -DVARIANT="\"$1\"" \
     -I$D/../../lla-mpc_amd/csrc -I$D/../../include -o $D/qb_$1 $D/quad_bench.hip
}
build full ""
build roll2 "-DROLL=2"
