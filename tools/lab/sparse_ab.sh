#!/bin/bash
# Interleaved A/B of the sparse-modulus kernels (runtime FHE_SPARSE=0/1, same
# library): q62 C3 / polymul / C5 (ab_bench.py) and the blind rotation
# presets (br_stamps.py).  usage: bash tools/lab/sparse_ab.sh [rounds]
set -u
R=${1:-2}
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for sp in 0 1; do
    FHE_SPARSE=$sp timeout -k 10 300 python -u tools/lab/ab_bench.py sparse$sp --ops fwd_mul,polymul,ext1,ext2 \
      --qs 4611686018326724609 || exit 1
    echo "== sparse$sp"; FHE_SPARSE=$sp timeout -k 10 200 python -u tools/lab/br_stamps.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
