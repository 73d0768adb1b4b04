#!/bin/bash
# Unit-twiddle kernels (ntt_core.hpp gk_compat): the -m gpu suite, then
# interleaved timings with FHE_UNIT_TW=1 / 0 (same library) of the kernels
# that take them, and the blind-rotation presets.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/unit_pytest.log 2>&1 || { tail -30 gpurun_out/unit_pytest.log; exit 1; }
tail -1 gpurun_out/unit_pytest.log
: > gpurun_out/unit_ab.log
for r in 1 2 3; do for u in 1 0; do
  FHE_UNIT_TW=$u timeout -k 10 300 python tools/lab/ab_bench.py unit$u --ops fwd_mul,polymul,relin,ext1,ext2 >> gpurun_out/unit_ab.log 2>&1 || exit 1
done; done
python tools/lab/ab_summary.py gpurun_out/unit_ab.log
for r in 1 2; do for u in 1 0; do
  echo "== FHE_UNIT_TW=$u"; FHE_UNIT_TW=$u timeout -k 10 200 python -u tools/lab/br_stamps.py --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
