#!/bin/bash
set -e
D=$(cd "$(dirname "$0")" && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm -I$D/../../lla-mpc_amd/csrc -I$D/../../include -o $D/chain_bench $D/chain_bench.hip && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm -I$D/../../lla-mpc_amd/csrc -o $D/lat_bench $D/lat_bench.hip
