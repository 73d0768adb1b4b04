#!/bin/bash
# -m gpu suite, then main vs base on ciphertext multiply only (the unit that
# took the opaque twiddle pointers, FHE_OPAQUE_TW=2), equal checksums.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; R=${2:-4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=node-fhe-accelerate_amd/build
: > $O/ab.log
for r in $(seq 1 $R); do
  for v in base main; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 132120577,4611686018326724609 --ops ct_mul >> $O/ab.log 2>&1 || exit 1
    echo "round $r $v done $(date +%T)"
  done
done
python tools/lab/ab_summary.py $O/ab.log
