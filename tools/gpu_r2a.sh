#!/bin/bash
# round-2 check: the previously faulting ct_mul case alone first, then the
# new GPU tests, then a 2-rank bench rehearsal on one GPU (gloo)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 200 $T "tests/test_gpu_cipher.py::test_decryption_identity_negacyclic" > gpurun_out/pytest_r2a0.log 2>&1 || exit $?
timeout -k 10 600 $T tests/test_gpu_multi.py tests/test_distributed.py tests/test_gpu_cipher.py > gpurun_out/pytest_r2a.log 2>&1 || exit $?
FHE_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu --no-q62 --no-cipher > gpurun_out/bench_g2.log 2>&1
