#!/bin/bash
# host-resident (FHE_HOST) path: tests touching host arrays, then the bench's
# host_resident measurement at two staging chunk sizes
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/host
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/host/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --only-host > gpurun_out/host/h32.json 2>&1 || exit $?
FHE_STAGE_MB=8 timeout -k 10 300 python -u bench.py --only-host > gpurun_out/host/h8.json 2>&1 || exit $?
FHE_STAGE_MB=128 timeout -k 10 300 python -u bench.py --only-host > gpurun_out/host/h128.json 2>&1 || exit $?
