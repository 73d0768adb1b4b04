#!/bin/bash
# After the store pad: the two diagnostics on the shipped build, the
# previously intermittent pair case repeated, then the blind-rotation tests.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
for c in "1024 4611686018326724609 15 2 1 3 compat" "2048 1125899906826241 15 2 1 3 compat" "4096 1152921504606584833 10 3 1 3 compat" "1024 4611686018326724609 15 2 1 3 negacyclic" "2048 40961 5 2 1 30 compat"; do
  echo "== $c" >> $O/diag.log
  timeout -k 10 300 python tools/lab/br_diag.py $c >> $O/diag.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $O/diag.log; exit 1; }
done
grep -v amdgpu.ids $O/diag.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "blind_rotate or br_ or bootstrap" > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
