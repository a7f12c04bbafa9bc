#!/bin/bash
# GPU tests, then the default bench (driver contract) and the C3 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2b}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
timeout -k 10 300 python bench.py --mixed --no-cpu-baseline --images 8192 --unique 2048 --steps 16 \
  > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err || exit $?
python scripts/show_bench.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_c3_bench.json
exit $rc
