#!/bin/bash
# Round 3g: fresh-container rebuild check: full -m gpu suite, default bench
# line, and the 2-rank gloo rehearsal on one GPU.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3g.log 2>&1 || { tail -40 gpurun_out/pytest_r3g.log; exit 1; }
echo "pytest: $(tail -1 gpurun_out/pytest_r3g.log)"
timeout -k 10 600 python bench.py > gpurun_out/bench_r3g.json 2> gpurun_out/bench_r3g.err || { tail -20 gpurun_out/bench_r3g.err; exit 1; }
tail -c 300 gpurun_out/bench_r3g.json
FHE_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 > gpurun_out/bench_r3g_dist2.json 2> gpurun_out/bench_r3g_dist2.err || { tail -20 gpurun_out/bench_r3g_dist2.err; exit 1; }
tail -c 600 gpurun_out/bench_r3g_dist2.json
