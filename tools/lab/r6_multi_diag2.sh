#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
for c in "1024 4611686018326724609 15 2" "1024 132120577 9 2"; do
  echo "== $c" >> $O/diag2.log
  timeout -k 10 300 python tools/lab/br_multi_diag.py $c >> $O/diag2.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $O/diag2.log; exit 1; }
done
cat $O/diag2.log
