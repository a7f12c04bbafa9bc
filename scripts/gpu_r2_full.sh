#!/bin/bash
# One GPU session: PMC traffic passes (-> profiles/r02_pmc_traffic.json, which the bench
# line reads), GPU tests, the default bench (driver contract), the C3 bench and a
# rocprofv3 kernel-trace summary of the default bench.  usage: scripts/gpu_r2_full.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2c}
BENCH="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --images 8192 --procs 0 --depth 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_write.log 2>&1 || exit $?
python scripts/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_traffic.json || exit $?
cp gpurun_out/${TAG}_traffic.json profiles/r02_pmc_traffic.json
echo "pmc done"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
timeout -k 10 300 python bench.py --mixed --no-cpu-baseline --images 8192 --unique 2048 --steps 16 \
  > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --depth 1 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python scripts/show_bench.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_c3_bench.json
exit $rc
