#!/bin/bash
# Round 3j: single-launch blind rotation at GLWE dimension 2 (k_br_persist_k):
# the cipher GPU tests, then the k = 2 / N = 32768 blind-rotation timing.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_cipher.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_r3j.log 2>&1 || { tail -40 gpurun_out/pytest_r3j.log; exit 1; }
echo "cipher: $(tail -1 gpurun_out/pytest_r3j.log)"
timeout -k 10 300 python tools/lab/br_composed.py > gpurun_out/br_r3j.json 2>&1 || { tail gpurun_out/br_r3j.json; exit 1; }
cat gpurun_out/br_r3j.json
