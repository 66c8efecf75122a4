#!/bin/bash
# Build an A/B variant of the library from a source directory (default: the tree's csrc)
# into lla-mpc_amd/llampc/_lib/<name>.so with extra hipcc flags.
# usage: tools/build_variant.sh <name> <srcdir> [flags...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=${2:-lla-mpc_amd/csrc}; shift 2 || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -disable-machine-licm \
  -Iinclude -I"$SRC" -Wall -Wno-unused-result "$@" -o lla-mpc_amd/llampc/_lib/$NAME.so \
  "$SRC/capi.hip" "$SRC/kernels.hip"
