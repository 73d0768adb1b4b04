#!/bin/bash
# One GPU lease: the whole -m gpu suite, smoke(), the default bench line, and
# the rocprofv3 evidence (trace + PMC) of every kernel the bench times, all
# from the library in this tree (tools/gpu_evidence.sh).
# Usage: bash tools/gpu_round.sh <tag> [evidence workloads ...]
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
echo "pytest: $(tail -1 $OUT/pytest.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json
bash tools/gpu_evidence.sh $TAG "$@"
