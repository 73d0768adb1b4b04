#!/bin/bash
# rocprofv3 kernel trace + PMC passes of one bench side workload
# (c5 | ct_mul | relin | blind_rotate), one summary per kernel afterwards.
# usage: bash tools/gpu_prof_side.sh <tag> <only>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; ONLY=$2
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --steps 4 --warmup 1 --only $ONLY"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $B > $OUT/trace.log 2>&1 || exit $?
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  name=$(echo $ctr | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$name -o run --output-format csv -- python3 $B > $OUT/pmc_$name.log 2>&1 || exit $?
done
