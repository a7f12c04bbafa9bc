#!/bin/bash
# SQ counters (instruction mix / waits / LDS conflicts) of every kernel: C2 and C3, two passes each.
set -o pipefail
TAG=${1:-sq4}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for W in c2 c3; do
  if [ $W = c3 ]; then EXTRA="--mixed --unique 64"; else EXTRA="--unique 256"; fi
  BENCH="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --images 2048 --procs 0 --depth 1 $EXTRA"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/${TAG}_${W}_a -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${W}_a.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/${TAG}_${W}_b -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${W}_b.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/${TAG}_${W}_c -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${W}_c.log 2>&1 || exit $?
  python scripts/pmc_counters.py gpurun_out/${TAG}_${W}_a gpurun_out/${TAG}_${W}_b gpurun_out/${TAG}_${W}_c > gpurun_out/${TAG}_${W}_table.txt 2>&1
done
