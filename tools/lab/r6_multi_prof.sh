#!/bin/bash
# rocprofv3 evidence of the multi-CU blind rotation (k_br_multi, six CUs per
# ciphertext) inside bench.py's preset lines: kernel trace + stats, then the
# two SQ counter passes, summarised for tfhe-256-secure at batch 1.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
BID=$(python3 -c "import sys; sys.path.insert(0, 'node-fhe-accelerate_amd'); import fhe_gpu; print(fhe_gpu.build_id())") || exit 1
B="bench.py --only br_presets"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.log 2>&1 \
  || { echo "trace failed rc=$?"; tail -5 $O/trace.log; exit 1; }
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 400 rocprofv3 --pmc $ctr -d $O/pmc_$i -o run --output-format csv -- python3 $B > $O/pmc_$i.log 2>&1 \
    || { echo "pmc $i failed rc=$?"; tail -5 $O/pmc_$i.log; exit 1; }
done
python3 tools/summarize_profile.py $O $O/summary --kernel-substr "k_br_multi<16396" --workload "br_multi,4096,1,1152921504606584833" --build-id $BID > /dev/null \
  || { echo "summarize failed"; exit 1; }
python3 -c "
import json; s = json.load(open('$O/summary/summary.json'))
print(s.get('kernel_name'), s.get('kernel_trace_full_batch'), s.get('valu_insts_per_wave'), s.get('effective_clock_ghz'))"
