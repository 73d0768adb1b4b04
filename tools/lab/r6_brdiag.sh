#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/r6g; mkdir -p $O
for lib in main base; do
  L=node-fhe-accelerate_amd/build/libfhe_gpu.so; [ $lib != main ] && L=node-fhe-accelerate_amd/build/libfhe_gpu_$lib.so
  echo "== $lib"
  FHE_GPU_LIB=$L timeout -k 10 240 python tools/lab/br_diag.py 2048 40961 5 2 1 10 2>&1 | tail -12 || exit 1
  FHE_GPU_LIB=$L timeout -k 10 240 python tools/lab/br_diag.py 4096 40961 5 2 1 5 2>&1 | tail -6 || exit 1
done
