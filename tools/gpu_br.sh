set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/br
timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher.py tests/test_gpu_engine.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "blind or bootstrap" > gpurun_out/br/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --only blind_rotate --steps 8 > gpurun_out/br/bench_default.json 2>&1 || exit $?
FHE_BR_PERSIST_MAX=100000 timeout -k 10 300 python -u bench.py --only blind_rotate --steps 8 > gpurun_out/br/bench_persist.json 2>&1 || exit $?
FHE_BR_PERSIST_MAX=0 timeout -k 10 300 python -u bench.py --only blind_rotate --steps 8 > gpurun_out/br/bench_steps.json 2>&1 || exit $?
