#!/bin/bash
# Round 3d: the default bench line (negacyclic block, engine chain, C2 CPU
# baseline, q62 roofline) and rocprofv3 summaries of the negacyclic C3/C4
# kernels and the flag-free q62 C3 kernel.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r3d.json 2> gpurun_out/bench_r3d.err || { tail -20 gpurun_out/bench_r3d.err; exit 1; }
tail -c 400 gpurun_out/bench_r3d.json
KERNEL=fwd_mul bash tools/gpu_profile.sh r3_nega_fwd_mul --mode negacyclic || exit 1
KERNEL=polymul bash tools/gpu_profile.sh r3_nega_polymul --mode negacyclic || exit 1
KERNEL=fwd_mul bash tools/gpu_profile.sh r3_q62_fwd_mul --q 4611686018326724609 || exit 1
