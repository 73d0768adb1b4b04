#!/bin/bash
# Round 3m: q62 forward (+ modmul) A/B: old (lane index held across the
# transform, stream depth 1) vs t1d1 (TidSource after the transform) vs
# t1d2 (TidSource, stream depth 2); parity of the transforms on each first.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=node-fhe-accelerate_amd/build
for v in t1d1 t1d2; do
  FHE_GPU_LIB=$B/libfhe_gpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    -k "transforms or non_canonical or golden" --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_r3m_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r3m_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_r3m_$v.log)"
done
: > gpurun_out/ab_r3m.log
for r in 1 2 3; do
  for v in main t1d1 t1d2; do
    lib=$B/libfhe_gpu.so; [ "$v" != "main" ] && lib=$B/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops fwd_mul,fwd \
      --qs 4611686018326724609 >> gpurun_out/ab_r3m.log 2>&1 || { tail gpurun_out/ab_r3m.log; exit 1; }
  done
done
python tools/lab/ab_summary.py gpurun_out/ab_r3m.log
