#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
for c in "1024 4611686018326724609 15 2 1 1 compat" "1024 132120577 9 2 1 1 compat"; do
  echo "== $2 $c" >> $O/diag3.log
  FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_$2.so timeout -k 10 120 python tools/lab/br_diag.py $c >> $O/diag3.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $O/diag3.log; exit 1; }
done
cat $O/diag3.log
