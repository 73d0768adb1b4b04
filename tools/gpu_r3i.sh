#!/bin/bash
# Round 3i: moduli >= 2^62 (ntt_wide.hip) first, then the full -m gpu suite,
# the bench line, profiles of C5, negacyclic C3/C4 and the q62 paired
# polymul, and the composed blind rotation timing.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_r3i_wide.log 2>&1 || { tail -40 gpurun_out/pytest_r3i_wide.log; exit 1; }
echo "wide: $(tail -1 gpurun_out/pytest_r3i_wide.log)"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3i.log 2>&1 || { tail -40 gpurun_out/pytest_r3i.log; exit 1; }
echo "pytest: $(tail -1 gpurun_out/pytest_r3i.log)"
timeout -k 10 600 python bench.py > gpurun_out/bench_r3i.json 2> gpurun_out/bench_r3i.err || { tail -20 gpurun_out/bench_r3i.err; exit 1; }
bash tools/gpu_prof_side.sh r3i_c5 c5 || exit 1
KERNEL=polymul bash tools/gpu_profile.sh r3i_nega_polymul --mode negacyclic || exit 1
KERNEL=fwd_mul bash tools/gpu_profile.sh r3i_nega_fwd_mul --mode negacyclic || exit 1
KERNEL=polymul bash tools/gpu_profile.sh r3i_q62_polymul --q 4611686018326724609 || exit 1
timeout -k 10 300 python tools/lab/br_composed.py > gpurun_out/br_composed_r3i.json 2>&1 || { tail gpurun_out/br_composed_r3i.json; exit 1; }
cat gpurun_out/br_composed_r3i.json
