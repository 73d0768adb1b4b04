#!/bin/bash
# Round 3e: q62 at N = 16384 -- 32 coefficients per thread with streamed
# twiddles and the split exchange (forward, inverse), paired-transform
# polymul vs the E32 HBM-stash polymul, streamed twiddles in the u32 paired
# kernels, single-inverse decrypt, paired u64 ct multiply.  Full -m gpu suite
# on the main build, parity of each variant, interleaved A/B timing.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=node-fhe-accelerate_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3e_main.log 2>&1 || { tail -40 gpurun_out/pytest_r3e_main.log; exit 1; }
echo "main: $(tail -1 gpurun_out/pytest_r3e_main.log)"
for v in p2 ns2; do
  FHE_GPU_LIB=$B/libfhe_gpu_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cipher.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3e_$v.log 2>&1 \
    || { tail -30 gpurun_out/pytest_r3e_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_r3e_$v.log)"
done
: > gpurun_out/ab_r3e.log
for r in 1 2 3; do
  for v in main old p2 ns2; do
    lib=$B/libfhe_gpu.so; [ "$v" != "main" ] && lib=$B/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops fwd_mul,polymul,fwd,inv \
      --qs 4611686018326724609 >> gpurun_out/ab_r3e.log 2>&1 || { tail gpurun_out/ab_r3e.log; exit 1; }
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops polymul,ct_mul \
      --qs 132120577 >> gpurun_out/ab_r3e.log 2>&1 || { tail gpurun_out/ab_r3e.log; exit 1; }
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops polymul,fwd_mul --mode negacyclic \
      --qs 132120577 >> gpurun_out/ab_r3e.log 2>&1 || { tail gpurun_out/ab_r3e.log; exit 1; }
  done
done
python tools/lab/ab_summary.py gpurun_out/ab_r3e.log
