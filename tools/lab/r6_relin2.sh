#!/bin/bash
# Relinearisation at two workgroups per CU (k_relin2, ntt_ext.hip): parity of
# each variant library against the oracle (the relinearisation GPU tests),
# then an interleaved A/B against the main build (equal output checksums).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; shift
VARS="$*"
mkdir -p $O
L=node-fhe-accelerate_amd/build
for v in $VARS; do
  FHE_GPU_LIB=$L/libfhe_gpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cipher.py -k "relin" -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "parity $v failed rc=$?"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
: > $O/ab.log
for r in 1 2 3; do
  for v in main $VARS; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 132120577 --ops relin >> $O/ab.log 2>&1 || exit 1
  done
done
python tools/lab/ab_summary.py $O/ab.log
