#!/bin/bash
# Round 3b: flag-free 64-bit arithmetic A/B (FHE_U64_NOVCC; mulhi carry vs
# carry-free) on the q62 C3 and polymul kernels, parity of the variants on
# the transform tests.  Every GPU step has its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_keygen.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_r3b_keygen.log 2>&1; tail -15 gpurun_out/pytest_r3b_keygen.log
for v in novcc novcc4; do
  FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_r3b_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r3b_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_r3b_$v.log
done
: > gpurun_out/ab_r3b.log
for r in 1 2 3; do
  for v in main novcc novcc4; do
    lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
    [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops fwd_mul,polymul \
      --qs 4611686018326724609 >> gpurun_out/ab_r3b.log 2>&1 || exit 1
  done
done
python tools/lab/ab_summary.py gpurun_out/ab_r3b.log
