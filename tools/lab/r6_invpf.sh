#!/bin/bash
# k_br_multi with the inverse's first-pass twiddles prefetched across the
# hand-off (main) vs loaded after it (nopf): blind-rotation tests, presets x2.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "blind_rotate or br_ or bootstrap" > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=node-fhe-accelerate_amd/build
for r in 1 2; do
  for v in nopf main; do
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
