#!/bin/bash
# Copy tools/gpu_evidence.sh summaries into profiles/<tag>_<workload>/
# (summary.json + the kernel-trace stats), which bench.py matches by build id.
# usage: bash tools/collect_evidence.sh <tag>   (here, or on the GPU box)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
for s in gpurun_out/evidence_$TAG/*/summary.json; do
  d=$(dirname $s); w=$(basename $d)
  mkdir -p profiles/${TAG}_$w
  cp $s profiles/${TAG}_$w/
  st=$d/trace/run_kernel_stats.csv
  [ -f $st ] && cp $st profiles/${TAG}_$w/kernel_stats.csv
  echo "profiles/${TAG}_$w"
done
cp gpurun_out/evidence_$TAG/build_id.txt profiles/ 2>/dev/null && mv profiles/build_id.txt profiles/${TAG}_build_id.txt || true
