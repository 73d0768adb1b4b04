#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then PMC
# counters in separate passes (FETCH_SIZE and WRITE_SIZE cannot share one).
# Usage: [KERNEL=fwd_mul|polymul] bash tools/gpu_profile.sh <tag> [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
K=${KERNEL:-fwd_mul}
B="bench.py --steps 5 --warmup 1 --no-cpu --no-q62 --no-check --only $K $*"
echo "trace $(date)" >> $OUT/progress.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $B > $OUT/trace.log 2>&1 || exit $?
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  name=$(echo $ctr | tr ' ' '_' | cut -c1-40)
  echo "pmc $ctr $(date)" >> $OUT/progress.log
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$name -o run --output-format csv -- python3 $B > $OUT/pmc_$name.log 2>&1 || { echo "pmc $ctr failed rc=$?" >> $OUT/progress.log; }
done
echo "done $(date)" >> $OUT/progress.log
