#!/bin/bash
# engine ops (encrypt / decrypt / add_plain / bootstrap) on the GPU
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $T tests/test_gpu_engine.py > gpurun_out/pytest_r2b.log 2>&1
