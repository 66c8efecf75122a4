#!/bin/bash
# Build an A/B variant of the library (every translation unit of the Makefile, in parallel)
# into lla-mpc_amd/llampc/_lib/<name>.so with extra hipcc flags.
# usage: tools/build_variant.sh <name> [flags...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=lla-mpc_amd/csrc
OBJ=lla-mpc_amd/build/variant_$NAME
mkdir -p $OBJ
pids=()
for f in capi kernels ctl plan_rk4_l4 plan_rk4_l2 plan_rk4_l1 plan_euler plan_rk6 nlp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -disable-machine-licm \
    -Iinclude -Wall -Wno-unused-result "$@" -c -o $OBJ/$f.o $SRC/$f.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lla-mpc_amd/llampc/_lib/$NAME.so $OBJ/*.o
