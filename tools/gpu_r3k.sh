#!/bin/bash
# Round 3k: k = 2 single-launch blind rotation, twiddle prefetch depth A/B
# (main: FHE_BRK_PF=4, _pf2: 2), interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=node-fhe-accelerate_amd/build
: > gpurun_out/br_r3k.log
for r in 1 2; do
  for v in main pf2; do
    lib=$B/libfhe_gpu.so; [ "$v" != "main" ] && lib=$B/libfhe_gpu_$v.so
    echo "== $v" >> gpurun_out/br_r3k.log
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/br_composed.py --batches 1,64 >> gpurun_out/br_r3k.log 2>&1 || { tail gpurun_out/br_r3k.log; exit 1; }
  done
done
grep -E "==|\"n\": 1024" gpurun_out/br_r3k.log
