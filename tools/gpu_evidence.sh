#!/bin/bash
# Roofline evidence for the kernels bench.py times, from the library in this
# tree: per workload one rocprofv3 kernel-trace + stats pass and separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, one SQ set), summarised with the exact
# demangled kernel name and fhe_build_id() (tools/summarize_profile.py).
# bench.py attaches a traffic figure only from a summary whose kernel and
# build id match what it runs.  Run it in the same lease as the bench line.
#
# usage: bash tools/gpu_evidence.sh <tag> [workload ...]
#   workloads: fwd_mul polymul q62_fwd_mul q62_polymul nega_fwd_mul
#              nega_polymul ct_mul relin c5 br   (default: all)
# output: gpurun_out/evidence_<tag>/<workload>/summary.json (copy to profiles/)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
WLS=${*:-"fwd_mul polymul q62_fwd_mul q62_polymul nega_fwd_mul nega_polymul ct_mul relin c5 br"}
P27=132120577; P62=4611686018326724609
BID=$(python3 -c "import sys; sys.path.insert(0, 'node-fhe-accelerate_amd'); import fhe_gpu; print(fhe_gpu.build_id())") || exit 1
OUT=gpurun_out/evidence_$TAG
mkdir -p $OUT
echo "build_id $BID" > $OUT/build_id.txt
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"
# VALU-issue roofline (tools/valu_roofline.py): busy cycles + the clock
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"

# name -> bench args | summaries (kernel-substr=workload ...)
spec() {
  case $1 in
    fwd_mul)      echo "--only fwd_mul --no-check --no-q62|k_ntt_fwd_mul=fwd_mul,16384,65536,$P27";;
    polymul)      echo "--only polymul --no-check --no-q62|k_polymul=polymul,16384,65536,$P27";;
    q62_fwd_mul)  echo "--only fwd_mul --no-check --q $P62|k_ntt_fwd_mul=fwd_mul,16384,65536,$P62";;
    q62_polymul)  echo "--only polymul --no-check --q $P62|k_polymul=polymul,16384,65536,$P62";;
    nega_fwd_mul) echo "--only fwd_mul --no-check --no-q62 --mode negacyclic|k_ntt_fwd_mul=fwd_mul,16384,65536,$P27,negacyclic";;
    nega_polymul) echo "--only polymul --no-check --no-q62 --mode negacyclic|k_polymul=polymul,16384,65536,$P27,negacyclic";;
    ct_mul)       echo "--only ct_mul|k_ct_mul=ct_mul,16384,8192,$P27";;
    relin)        echo "--only relin|k_dmac=relin,16384,8192,$P27";;
    br)           echo "--only br_presets|k_br_pair=br_pair,4096,64,1152921504606584833";;
    c5)           echo "--only c5|k_extprod2=extprod_B23_L1,16384,4096,$P62 k_extprod_acc=extprod_B15_L2,16384,4096,$P62";;
    *) return 1;;
  esac
}

for wl in $WLS; do
  sp=$(spec $wl) || { echo "unknown workload $wl"; exit 2; }
  args=${sp%%|*}; sums=${sp#*|}
  d=$OUT/$wl; mkdir -p $d
  B="bench.py --steps 10 --warmup 3 $args"
  echo "$wl: trace $(date +%T)" | tee -a $OUT/progress.log
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python3 $B \
    > $d/trace.log 2>&1 || { echo "$wl trace failed rc=$?"; tail -5 $d/trace.log; exit 1; }
  i=0
  # relinearisation: L2 -> CU read requests and L2 hit/miss (the prepared
  # key is re-read from L2 by every workgroup)
  EXTRA=""; [ $wl = relin ] && EXTRA="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
  for ctr in FETCH_SIZE WRITE_SIZE "$SQ" "$SQ2" ${EXTRA:+"$EXTRA"}; do
    i=$((i + 1))
    echo "$wl: pmc$i $(date +%T)" >> $OUT/progress.log
    timeout -s KILL 240 rocprofv3 --pmc $ctr -d $d/pmc_$i -o run --output-format csv -- python3 $B \
      > $d/pmc_$i.log 2>&1 || { echo "$wl pmc $ctr failed rc=$?"; tail -5 $d/pmc_$i.log; exit 1; }
  done
  for s in $sums; do
    ks=${s%%=*}; w=${s#*=}
    sub=$d; [ "$(echo $sums | wc -w)" -gt 1 ] && sub=$OUT/${w%%,*}
    mkdir -p $sub
    python3 tools/summarize_profile.py $d $sub --kernel-substr "$ks" --workload "$w" --build-id $BID > /dev/null \
      || { echo "summarize $wl failed"; exit 1; }
    python3 - "$sub/summary.json" <<'EOF'
import json, sys
s = json.load(open(sys.argv[1]))
kt = s.get("kernel_trace_full_batch", {})
alg = None
print(f"{s['workload']['kernel']}: {s.get('kernel_name', s.get('kernel_names'))[:90]} "
      f"avg {kt.get('avg_ns', 0) / 1e6:.3f} ms, traffic {s.get('hbm_traffic_bytes_per_launch', 0) / 1e9:.3f} GB, "
      f"VALU/wave {s.get('valu_insts_per_wave', 0):.0f}")
EOF
  done
done
echo "done $(date +%T)" >> $OUT/progress.log
