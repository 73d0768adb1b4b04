set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_rl2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher.py tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "relin or multiply_relin or identity" > gpurun_out/pytest_rl2.log 2>&1 || exit $?
SKIP_TESTS=1 bash tools/gpu_ab.sh main,rl2 3 --ops relin --qs 132120577
