#!/bin/bash
# Round 3c: the whole -m gpu suite (FHEEngine JS surface, keygen parity,
# flag-free forward kernels) and smoke().  Stop at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_r3c.log 2>&1 || { grep -E "FAILED|Error|error|assert" gpurun_out/pytest_r3c.log | head -40; tail -60 gpurun_out/pytest_r3c.log; exit 1; }
tail -2 gpurun_out/pytest_r3c.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3c.log 2>&1 || { cat gpurun_out/smoke_r3c.log; exit 1; }
tail -1 gpurun_out/smoke_r3c.log
