#!/bin/bash
# Round 6: the -m gpu suite, the extended VALU issue-rate table and its PMC
# calibration (SQ_ACTIVE_INST_VALU on kernels of known issue rate), then the
# barrier-free exchange bound: main vs the FHE_LAB_NOBAR=1 variant (wrong
# results, timing only) on the kernels with internal spectra.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 tools/lab/valu_rates > $O/valu_rates.txt 2>&1 || { echo "valu_rates rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  -d $O/vr_pmc -o run --output-format csv -- tools/lab/valu_rates > $O/vr_pmc.log 2>&1 || { echo "vr pmc rc=$?"; exit 1; }
L=node-fhe-accelerate_amd/build
: > $O/ab.log
for r in 1 2; do
  for v in main nobar; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 132120577 --ops polymul,relin,ct_mul >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 4611686018326724609 --ops fwd_mul,polymul,ext1,ext2 >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --n 4096 --batch 4096 --qs 1152921504606584833 --ops br256 --steps 2 >> $O/ab.log 2>&1 || exit 1
    echo "round $r $v done $(date +%T)"
  done
done
python tools/lab/ab_summary.py $O/ab.log
