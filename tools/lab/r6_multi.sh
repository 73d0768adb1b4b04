#!/bin/bash
# Multi-CU blind rotation (k_br_multi): the blind-rotation GPU tests, then the
# preset lines with and without it (FHE_BR_MULTI=0: the pair), same build.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ulimit -c 0
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "blind_rotate or br_ or bootstrap" > $O/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1; do
  FHE_BR_MULTI=$v timeout -k 10 300 python bench.py --only br_presets > $O/br_multi$v.json 2> $O/br_multi$v.err \
    || { echo "bench failed rc=$?"; tail -20 $O/br_multi$v.err; exit 1; }
  python3 - $O/br_multi$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d["cipher"]["blind_rotate_presets"]
for name, v in p.items():
    if isinstance(v, dict):
        br = {b: round(v[b]["ms"], 2) for b in ("batch1", "batch64", "batch8192") if b in v}
        bs = {b: round(v["bootstrap"][b]["ms"], 2) for b in ("batch1", "batch64") if b in v.get("bootstrap", {})}
        print("MULTI", sys.argv[2], name, "br", br, "bootstrap", bs)
PY
done
