#!/bin/bash
# -m gpu suite, then main vs base on the units that took the flag-free
# 64-bit arithmetic (ntt_ext / ntt_cipher / ntt_engine_enc), equal checksums.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; R=${2:-3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=node-fhe-accelerate_amd/build
: > $O/ab.log
for r in $(seq 1 $R); do
  for v in base main; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 4611686018326724609 --ops ext1,ext2,ct_mul,relin,polymul >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --qs 132120577 --ops ct_mul,relin >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python tools/lab/ab_bench.py $v --n 8192 --batch 4096 --qs 4611686018326724609 --ops br8192 --steps 3 >> $O/ab.log 2>&1 || exit 1
    FHE_GPU_LIB=$lib timeout -k 10 300 python bench.py --only engine > $O/engine_${v}_${r}.json 2>/dev/null && \
      python3 -c "import json,sys; d=json.load(open('$O/engine_${v}_${r}.json'))['engine_chain']; print('ENGINE $v', d['device_resident']['ms'], d['host_resident']['ms'])" >> $O/ab.log
    echo "round $r $v done $(date +%T)"
  done
done
python tools/lab/ab_summary.py $O/ab.log
grep ENGINE $O/ab.log
