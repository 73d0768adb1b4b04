#!/bin/bash
# Round 3l (final): full -m gpu suite, smoke, the default bench line, and the
# k = 2 blind-rotation prefetch A/B (main PF=4 vs _pf2).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3l.log 2>&1 || { tail -40 gpurun_out/pytest_r3l.log; exit 1; }
echo "pytest: $(tail -1 gpurun_out/pytest_r3l.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3l.log 2>&1 || { tail gpurun_out/smoke_r3l.log; exit 1; }
tail -1 gpurun_out/smoke_r3l.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r3l.json 2> gpurun_out/bench_r3l.err || { tail -20 gpurun_out/bench_r3l.err; exit 1; }
tail -c 200 gpurun_out/bench_r3l.json
bash tools/gpu_r3k.sh
