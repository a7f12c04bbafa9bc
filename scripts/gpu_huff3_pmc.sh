#!/bin/bash
# Memory-side traffic of the decode kernels on C3 (k_huff3 read amplification):
# FETCH / WRITE and the L2 / L1 request counters, per build/lib_<name>.so given.
# usage: scripts/gpu_huff3_pmc.sh TAG name1 name2 ...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
BENCH="python bench.py --mixed --steps 3 --warmup 1 --no-cpu-baseline --no-extras --images 2048 --unique 512 --procs 0 --depth 1"
for n in "$@"; do
  export DINO_INGEST_LIB=build/lib_$n.so
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_${n}_a -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${n}_a.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/${TAG}_${n}_b -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${n}_b.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/${TAG}_${n}_c -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${n}_c.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_READ_sum TCC_WRITE_sum -d gpurun_out/${TAG}_${n}_d -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${n}_d.log 2>&1 || exit $?
  python scripts/pmc_counters.py gpurun_out/${TAG}_${n}_a gpurun_out/${TAG}_${n}_b gpurun_out/${TAG}_${n}_c gpurun_out/${TAG}_${n}_d > gpurun_out/${TAG}_${n}_table.txt 2>&1
  grep -E "kernel|huff|idct|color|destuff|hresize" gpurun_out/${TAG}_${n}_table.txt
done
