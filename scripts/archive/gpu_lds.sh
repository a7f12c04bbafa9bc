#!/bin/bash
# LDS counters per kernel (bank / address conflicts, unaligned stalls) of the bench at depth 1.
# usage: scripts/gpu_lds.sh TAG [c2|c3]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-lds}; W=${2:-c2}
if [ $W = c3 ]; then EXTRA="--mixed --unique 1024 --images 2048"; else EXTRA="--images 4096 --procs 0"; fi
CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $CTRS -d gpurun_out/${TAG}_${W}_lds -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --depth 1 $EXTRA \
  > gpurun_out/${TAG}_${W}_lds.log 2>&1 || exit $?
python scripts/pmc_counters.py gpurun_out/${TAG}_${W}_lds > gpurun_out/${TAG}_${W}_lds.txt || exit $?
cat gpurun_out/${TAG}_${W}_lds.txt
