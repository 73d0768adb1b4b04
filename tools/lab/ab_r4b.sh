# round-4 lab batch: correctness of the new paths first, then A/Bs
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cipher.py tests/test_gpu_engine.py tests/test_gpu_wide.py tests/test_gpu_keygen.py tests/test_gpu_parity.py tests/test_napi.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/pytest_new.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_new.log | head -20; exit 1; }
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,rl_old,xa_h1,xa_p2,xa_old" 3 --ops relin,ext2 --qs 132120577,4611686018326724609 --steps 5 && cp gpurun_out/ab.log gpurun_out/ab_relin_ext.log || exit 1
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,e16p1,e16c4,alu,e16alu" 3 --ops polymul --qs 132120577 --steps 10 && cp gpurun_out/ab.log gpurun_out/ab_poly27.log || exit 1
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,m4,nv4,nv0" 3 --ops polymul,inv --qs 4611686018326724609 --steps 4 && cp gpurun_out/ab.log gpurun_out/ab_poly62.log || exit 1
timeout -k 10 300 python -u bench.py --only br_presets --steps 3 > gpurun_out/br_presets.json 2> gpurun_out/br_presets.err || { tail gpurun_out/br_presets.err; exit 1; }
tail -c 800 gpurun_out/br_presets.json
