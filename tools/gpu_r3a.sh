#!/bin/bash
# Round 3a: baseline on a fresh box -- the -m gpu suite, the default bench
# line, and the first rocprofv3 summary of the q62 polymul kernel (none was
# kept in round 2).  Each GPU step has its own time limit; stop at the first
# failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3a.log 2>&1 || { tail -30 gpurun_out/pytest_r3a.log; exit 1; }
tail -2 gpurun_out/pytest_r3a.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r3a.json 2> gpurun_out/bench_r3a.err || exit 1
tail -c 600 gpurun_out/bench_r3a.json
KERNEL=polymul bash tools/gpu_profile.sh r3_q62_polymul --q 4611686018326724609
