#!/bin/bash
# The -m gpu suite twice more on the closing build (the intermittent
# blind-rotation mismatch of this round: any recurrence shows here).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$i.log 2>&1 \
    || { echo "pytest $i failed rc=$?"; tail -30 $O/pytest_$i.log; exit 1; }
  tail -1 $O/pytest_$i.log
done
