#!/bin/bash
# Dry run of the evidence pipeline on one workload: rocprofv3 trace + PMC
# passes (tools/gpu_evidence.sh), the summary copied into profiles/, then the
# bench's side metric for that workload, which must attach the VALU roofline.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
timeout -k 10 600 bash tools/gpu_evidence.sh r6e relin || exit 1
mkdir -p profiles/r6e_relin && cp gpurun_out/evidence_r6e/relin/summary.json gpurun_out/evidence_r6e/relin/*.csv profiles/r6e_relin/ 2>/dev/null
cp gpurun_out/evidence_r6e/relin/trace/*kernel_stats.csv profiles/r6e_relin/kernel_stats.csv 2>/dev/null
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --only relin > gpurun_out/evidence_r6e/bench_relin.json 2> gpurun_out/evidence_r6e/bench_relin.err || exit 1
python3 -c "
import json; d = json.load(open('gpurun_out/evidence_r6e/bench_relin.json'))['cipher']['relinearize']
print(json.dumps({k: d.get(k) for k in ('kernel_ms', 'traffic_over_algorithmic', 'frac_profile')}))
print(json.dumps(d.get('valu_roofline'))[:600])"
