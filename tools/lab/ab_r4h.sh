# round-4 lab batch h: one-workgroup blind rotation at 4 coefficients per thread (bl2) for large batches
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
FHE_GPU_LIB=node-fhe-accelerate_amd/build/libfhe_gpu_bl2.so FHE_BR_PAIR=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher.py -m gpu -k "blind" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bl2.log 2>&1
rc=$?
echo "pytest bl2 rc=$rc $(tail -1 gpurun_out/pytest_bl2.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_bl2.log | head -20; exit 1; }
for r in 1 2; do
for v in main bl2; do
  lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
  [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
  FHE_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --only br_presets --steps 3 > gpurun_out/br_${v}_$r.json 2> gpurun_out/br_${v}_$r.err || { tail gpurun_out/br_${v}_$r.err; exit 1; }
  FHE_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --only blind_rotate --steps 3 > gpurun_out/brc1_${v}_$r.json 2> gpurun_out/brc1_${v}_$r.err || { tail gpurun_out/brc1_${v}_$r.err; exit 1; }
done
done
echo done
