#!/bin/bash
# Round-4 GPU session: parity tests, smoke, the driver's default bench line (with the c3 /
# fp8 / c2_dri / e2e legs), and a depth-1 rocprofv3 kernel summary of the C2 leg.
# usage: scripts/gpu_r3.sh TAG [tests|bench|prof|all]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4a}
WHAT=${2:-all}
rc=0
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 840 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gputests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${TAG}_gputests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures (keep going), else stop
  timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
  head -c 400 gpurun_out/${TAG}_bench.json; echo
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --depth 1 --procs 0 --images 8192 \
    > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
fi
exit $rc
