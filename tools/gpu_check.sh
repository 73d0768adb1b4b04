#!/bin/bash
# GPU parity tests then one bench line.  Usage: bash tools/gpu_check.sh [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.log
K=${1:-}
timeout -k 10 1000 python -m pytest tests -m gpu -x -q --timeout 400 -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> gpurun_out/progress.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2 $(date)" >> gpurun_out/progress.log
exit $rc2
