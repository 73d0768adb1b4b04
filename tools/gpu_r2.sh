#!/bin/bash
# Round-2 record: -m gpu suite, smoke(), the default bench line, and the
# rocprofv3 summaries (kernel trace + PMC passes) of C4 polymul and C3.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
KERNEL=polymul timeout -k 10 900 bash tools/gpu_profile.sh ${TAG}_polymul || exit $?
KERNEL=fwd_mul timeout -k 10 900 bash tools/gpu_profile.sh ${TAG}_fwd_mul || exit $?
