#!/bin/bash
# -m gpu suite of this tree, then an interleaved A/B of libfhe_gpu.so against
# libfhe_gpu_base.so (tools/lab/build_variant.sh base <ref>), equal output
# checksums required (ab_summary.py).
# usage: bash tools/lab/r6_ab.sh <tag> [rounds]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; R=${2:-3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=node-fhe-accelerate_amd/build
: > $O/ab.log
for r in $(seq 1 $R); do
  for v in base main; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 132120577 --ops fwd_mul,polymul,relin,ct_mul >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 4611686018326724609 --ops fwd_mul,polymul,inv,ext1,ext2 >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --n 4096 --batch 4096 --qs 1152921504606584833 --ops br256 --steps 2 >> $O/ab.log 2>&1 || exit 1
    echo "round $r $v done $(date +%T)"
  done
done
python tools/lab/ab_summary.py $O/ab.log
