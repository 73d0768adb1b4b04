#!/bin/bash
# Fast lab variant: reuse the main build's objects and recompile only the
# named kernel files with extra flags (same namespace; one variant per
# process, as tools/gpu_ab.sh runs them).
# usage: tools/lab/quick_variant.sh <name> "<kernel files, e.g. ntt_inv>" [extra -D flags]
set -eu
NAME=$1; FILES=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG=$ROOT/node-fhe-accelerate_amd
OBJ=$PKG/build/obj_$NAME
mkdir -p $OBJ
cp $PKG/build/obj/*.o $OBJ/
pids=""
for f in $FILES; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
    -c $PKG/csrc/$f.hip -o $OBJ/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/build/libfhe_gpu_$NAME.so $OBJ/*.o -Wl,-soname,libfhe_gpu_$NAME.so
echo "built build/libfhe_gpu_$NAME.so ($FILES $*)"
