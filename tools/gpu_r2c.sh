#!/bin/bash
# Round 2c: the whole -m gpu suite and smoke() on the 64-bit mad-chain build,
# an interleaved A/B of the q62 kernels against the previous 64-bit
# arithmetic (variant "u64base"), the default bench line, and rocprofv3
# passes of the q62 C3 kernel.  Every GPU step has its own time limit; the
# script stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r2c.log 2>&1 || { tail -30 gpurun_out/pytest_r2c.log; exit 1; }
tail -2 gpurun_out/pytest_r2c.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2c.log 2>&1 || exit 1
: > gpurun_out/ab_r2c.log
for r in 1 2 3; do
  for v in u64base main; do
    lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
    [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --ops fwd_mul,polymul \
      --qs 4611686018326724609 >> gpurun_out/ab_r2c.log 2>&1 || exit 1
  done
done
python tools/lab/ab_summary.py gpurun_out/ab_r2c.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r2c.json 2> gpurun_out/bench_r2c.err || exit 1
tail -1 gpurun_out/bench_r2c.json
KERNEL=fwd_mul bash tools/gpu_profile.sh r2c_q62 --q 4611686018326724609
