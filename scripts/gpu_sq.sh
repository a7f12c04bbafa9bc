#!/bin/bash
# Per-kernel instruction / cycle counters of the bench at depth 1 (serialised batches), C2 and
# C3: pass "i" = instruction mix, pass "w" = where the wave cycles go (WAIT_ANY = parked on
# s_waitcnt / barrier, WAIT_INST_ANY = issue stall, ACTIVE_INST_* = issuing; quad-cycles).
# usage: scripts/gpu_sq.sh TAG [c2,c3]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-sq}
WL=${2:-c2,c3}
CTRS_i="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
CTRS_w="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
for W in ${WL//,/ }; do
  if [ $W = c3 ]; then EXTRA="--mixed --unique 1024 --images 2048"; else EXTRA="--images 4096 --procs 0"; fi
  for P in i w; do
    eval CTRS=\$CTRS_$P
    timeout -s KILL 240 rocprofv3 --pmc $CTRS -d gpurun_out/${TAG}_${W}_sq$P -o run --output-format csv -- \
      python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --depth 1 $EXTRA \
      > gpurun_out/${TAG}_${W}_sq$P.log 2>&1 || exit $?
  done
  python scripts/pmc_counters.py gpurun_out/${TAG}_${W}_sqi gpurun_out/${TAG}_${W}_sqw > gpurun_out/${TAG}_${W}_sq.txt || exit $?
  cat gpurun_out/${TAG}_${W}_sq.txt
done
exit 0
