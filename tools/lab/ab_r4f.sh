# round-4 lab batch f: blind rotation on two CUs per ciphertext (k_br_pair) vs one (FHE_BR_PAIR=0)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher.py tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -k "blind or bootstrap" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pair.log 2>&1
rc=$?
echo "pytest pair rc=$rc $(tail -1 gpurun_out/pytest_pair.log)"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_pair.log | head -20; exit 1; }
for r in 1 2; do
for v in 1 0; do
  FHE_BR_PAIR=$v timeout -k 10 300 python -u bench.py --only br_presets --steps 3 > gpurun_out/br_p${v}_$r.json 2> gpurun_out/br_p${v}_$r.err || { tail gpurun_out/br_p${v}_$r.err; exit 1; }
  FHE_BR_PAIR=$v timeout -k 10 300 python -u bench.py --only blind_rotate --steps 3 > gpurun_out/brc1_p${v}_$r.json 2> gpurun_out/brc1_p${v}_$r.err || { tail gpurun_out/brc1_p${v}_$r.err; exit 1; }
done
done
echo done
