#!/bin/bash
# GPU parity tests of the main build, then an interleaved A/B of library
# variants, one process per (round, variant).
# usage: bash tools/gpu_ab.sh "base,main,x" [rounds] [ab_bench args]   ("main" = libfhe_gpu.so)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1; R=${2:-3}; shift; shift || true
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -2 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
: > gpurun_out/ab.log
for r in $(seq 1 $R); do
  for v in ${V//,/ }; do
    lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
    [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v "$@" >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
python tools/lab/ab_summary.py gpurun_out/ab.log
