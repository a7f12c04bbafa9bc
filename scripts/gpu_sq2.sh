#!/bin/bash
# SQ instruction-mix / stall counters per kernel (per dispatch) of a short depth-1 bench.
# usage: scripts/gpu_sq2.sh TAG
set -o pipefail
TAG=${1:-sq}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
BENCH="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --images 2048 --unique 64 --procs 0 --depth 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/${TAG}_a -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/${TAG}_b -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_b.log 2>&1 || exit $?
python scripts/pmc_counters.py gpurun_out/${TAG}_a gpurun_out/${TAG}_b > gpurun_out/${TAG}_table.txt 2>&1
cat gpurun_out/${TAG}_table.txt
