#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke(), the default bench line, and
# the rocprofv3 kernel-trace summary of that same bench command.
# Usage: bash tools/gpu_round.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
