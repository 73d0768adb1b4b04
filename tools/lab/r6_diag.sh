#!/bin/bash
# Round-6 first lease: the -m gpu suite on this tree, the VALU issue-rate
# table (valu_rates), the gfx950 counter list, and one diagnostic run of the
# cooperative-launch exit crash under rocprofv3 (last: a crash ends the call).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/r6a
mkdir -p $O
echo "pytest $(date +%T)" > $O/progress.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo "valu_rates $(date +%T)" >> $O/progress.log
timeout -k 10 120 tools/lab/valu_rates > $O/valu_rates.txt 2>&1 || { echo "valu_rates rc=$?"; exit 1; }
cat $O/valu_rates.txt
echo "counters $(date +%T)" >> $O/progress.log
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list rc=$?"
echo "coop diag $(date +%T)" >> $O/progress.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/coop -o run --output-format csv -- \
  python3 tools/lab/exit_maps.py $O/maps_coop.txt -- --steps 2 --warmup 1 --only br_presets > $O/coop.log 2>&1
echo "coop diag rc=$?"
tail -30 $O/coop.log
