#!/bin/bash
# PMC passes of ab_bench.py for several library variants (lab A/B).
# usage: bash tools/lab/prof_ab.sh "main,x" <op> <q> [n] [batch]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=$1; OP=$2; Q=$3; N=${4:-16384}; B=${5:-65536}
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"
      "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64")
for v in ${V//,/ }; do
  lib=node-fhe-accelerate_amd/build/libfhe_gpu.so
  [ "$v" != "main" ] && lib=node-fhe-accelerate_amd/build/libfhe_gpu_$v.so
  OUT=gpurun_out/pab_$v
  mkdir -p $OUT
  A="tools/lab/ab_bench.py $v --ops $OP --qs $Q --n $N --batch $B --steps 3"
  FHE_GPU_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $A > $OUT/trace.log 2>&1 || exit $?
  i=0
  for s in "${SETS[@]}"; do
    FHE_GPU_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $s -d $OUT/pmc_$i -o run --output-format csv -- python3 $A > $OUT/pmc_$i.log 2>&1 || exit $?
    i=$((i+1))
  done
done
