# round-4 lab batch c: blind rotation geometry (E = 8 per thread at N = 2048 / 4096), polymul loads in flight
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_dbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cipher.py -m gpu -k "ct_multiply" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dbg.log 2>&1
rc=$?
echo "pytest dbg-slots rc=$rc $(tail -1 gpurun_out/pytest_dbg.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error|slot" gpurun_out/pytest_dbg.log | head -20; exit 1; }
for v in main bre3; do
  lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
  [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
  FHE_GPU_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher.py -m gpu -k "blind" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_br_$v.log 2>&1
  rc=$?
  echo "pytest blind $v rc=$rc $(tail -1 gpurun_out/pytest_br_$v.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_br_$v.log | head -20; exit 1; }
done
for v in main bre3; do
  lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
  [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
  FHE_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --only br_presets --steps 3 > gpurun_out/br_$v.json 2> gpurun_out/br_$v.err || { tail gpurun_out/br_$v.err; exit 1; }
done
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,in2,in4,ch16,in2c16" 3 --ops polymul --qs 132120577 --steps 10 && cp gpurun_out/ab.log gpurun_out/ab_poly27c.log || exit 1
