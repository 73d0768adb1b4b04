#!/bin/bash
# Round 3f: full -m gpu suite on the main build (u64 paired polymul at
# prefetch depth 0, depth-1 twiddle stream in the E32 forward, decrypt with
# one inverse, paired u64 ct multiply, u64 VGPR-slot ct multiply re-enabled),
# then interleaved A/B of the forward stream depth and the pre-round-3 u64
# geometry.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=node-fhe-accelerate_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3f_main.log 2>&1 || { tail -40 gpurun_out/pytest_r3f_main.log; exit 1; }
echo "main: $(tail -1 gpurun_out/pytest_r3f_main.log)"
FHE_GPU_LIB=$B/libfhe_gpu_d4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3f_d4.log 2>&1 \
  || { tail -30 gpurun_out/pytest_r3f_d4.log; exit 1; }
echo "d4: $(tail -1 gpurun_out/pytest_r3f_d4.log)"
: > gpurun_out/ab_r3f.log
for r in 1 2 3; do
  for v in main old d4; do
    lib=$B/libfhe_gpu.so; [ "$v" != "main" ] && lib=$B/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops fwd_mul,polymul,fwd,inv,ct_mul \
      --qs 4611686018326724609 >> gpurun_out/ab_r3f.log 2>&1 || { tail gpurun_out/ab_r3f.log; exit 1; }
  done
done
python tools/lab/ab_summary.py gpurun_out/ab_r3f.log
