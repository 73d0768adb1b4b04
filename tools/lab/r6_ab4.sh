#!/bin/bash
# Generic A/B: main vs the listed variant libraries on the listed ab_bench
# ops, R rounds interleaved, optionally after a pytest -k selection.
# usage: r6_ab4.sh OUT R "variants" "ab_bench args" ["pytest -k expr"]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; R=$2; VS=$3; AB=$4; K=${5:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 \
    || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
L=node-fhe-accelerate_amd/build
: > $O/ab.log
for r in $(seq 1 $R); do
  for v in $VS main; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v $AB >> $O/ab.log 2>&1 || exit 1
  done
  echo "round $r done $(date +%T)"
done
python tools/lab/ab_summary.py $O/ab.log
