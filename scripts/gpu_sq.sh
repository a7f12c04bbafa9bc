#!/bin/bash
# Per-kernel instruction / cycle counters (one rocprofv3 --pmc pass per workload, 8 SQ counters)
# of the bench at depth 1 (serialised batches), C2 and C3.
# usage: scripts/gpu_sq.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-sq}
CTRS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for W in c2 c3; do
  if [ $W = c3 ]; then EXTRA="--mixed --unique 1024 --images 2048"; else EXTRA="--images 4096 --procs 0"; fi
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d gpurun_out/${TAG}_${W}_sq -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --depth 1 $EXTRA \
    > gpurun_out/${TAG}_${W}_sq.log 2>&1 || exit $?
  python scripts/pmc_counters.py gpurun_out/${TAG}_${W}_sq > gpurun_out/${TAG}_${W}_sq.txt || exit $?
done
exit 0
