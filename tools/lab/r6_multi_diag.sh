#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
for c in "1024 4611686018326724609 15 2 1 2 negacyclic" "1024 4611686018326724609 15 2 1 2 compat" "2048 40961 5 2 1 2 compat" "2048 1125899906826241 15 2 1 2 compat" "4096 1152921504606584833 10 3 1 2 compat" "1024 132120577 9 3 1 2 negacyclic" "1024 132120577 9 2 1 2 negacyclic"; do
  echo "== $c" >> $O/diag.log
  timeout -k 10 120 python tools/lab/br_diag.py $c >> $O/diag.log 2>&1 || { echo "diag failed rc=$? ($c)"; tail -20 $O/diag.log; exit 1; }
done
cat $O/diag.log
