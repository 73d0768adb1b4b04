# round-4 lab batch i: two-launch relinearisation -- parity per variant, then timing vs MODE 1 (rlold)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in main rls rlp1; do
  lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
  [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
  FHE_GPU_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cipher.py -m gpu -k "relinearize" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1
  echo "pytest $v rc=$? $(tail -1 gpurun_out/pytest_$v.log)"
done
SKIP_TESTS=1 bash tools/gpu_ab.sh "main,rls,rlp1,rlold" 2 --ops relin --qs 132120577 --steps 5 && cp gpurun_out/ab.log gpurun_out/ab_relin_split.log
