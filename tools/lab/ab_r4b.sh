set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,e16p1,e16c4,alu,e16alu" 3 --ops polymul --qs 132120577 --steps 10 && cp gpurun_out/ab.log gpurun_out/ab_poly27.log
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,m4,nv4,nv0" 3 --ops polymul,inv --qs 4611686018326724609 --steps 4 && cp gpurun_out/ab.log gpurun_out/ab_poly62.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_wide.py tests/test_gpu_keygen.py tests/test_gpu_parity.py tests/test_napi.py tests/test_gpu_cipher.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
echo "pytest rc=$? $(tail -1 gpurun_out/pytest_new.log)"
