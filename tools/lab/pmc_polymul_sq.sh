set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c_polymul_sq2
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/r4c_polymul_sq2/pmc -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --only polymul --no-check --no-q62 > gpurun_out/r4c_polymul_sq2/pmc.log 2>&1 || { tail -5 gpurun_out/r4c_polymul_sq2/pmc.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r4c_polymul_sq2/grbm -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --only polymul --no-check --no-q62 > gpurun_out/r4c_polymul_sq2/grbm.log 2>&1 || { tail -5 gpurun_out/r4c_polymul_sq2/grbm.log; exit 1; }
ls gpurun_out/r4c_polymul_sq2/pmc
