#!/bin/bash
# Multi-CU blind rotation at 8 coefficients per thread (512 threads) vs 4
# (1024 threads, shipped): preset lines, main vs the e8 variant, twice.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
L=node-fhe-accelerate_amd/build
for r in 1 2; do
  for v in main e8; do
    lib=$L/libfhe_gpu.so; [ $v != main ] && lib=$L/libfhe_gpu_$v.so
    FHE_GPU_LIB=$lib timeout -k 10 300 python bench.py --only br_presets > $O/br_$v$r.json 2> $O/br_$v$r.err \
      || { echo "bench failed rc=$?"; tail -20 $O/br_$v$r.err; exit 1; }
    python3 - $O/br_$v$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for name, v in d["cipher"]["blind_rotate_presets"].items():
    if isinstance(v, dict):
        print(sys.argv[2], name, {b: round(v[b]["ms"], 2) for b in ("batch1", "batch64")})
PY
  done
done
