#!/bin/bash
# Round-6 closing lease: the rest of the evidence (tools/gpu_evidence.sh),
# summaries into profiles/, then the -m gpu suite, smoke() and the bench line
# against those profiles.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_evidence.sh $TAG "$@" || exit 1
bash tools/collect_evidence.sh $TAG > /dev/null || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_line.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_line.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'))"
