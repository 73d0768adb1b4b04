#!/bin/bash
# Interleaved blind-rotation timings of library variants (tools/lab/br_stamps.py).
# usage: bash tools/lab/br_ab.sh "main,lb1,..." [rounds]
set -u
V=${1:-main}; R=${2:-2}
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in ${V//,/ }; do
    lib=node-fhe-accelerate_amd/build/libfhe_gpu.so; [ $v != main ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
    echo "== $v"; FHE_GPU_LIB=$lib timeout -k 10 200 python -u tools/lab/br_stamps.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
