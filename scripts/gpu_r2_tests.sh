#!/bin/bash
# Round-2 GPU check: parity tests, smoke, short bench (each step under its own limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r2_gputests.log 2>&1
rc=$?
tail -5 gpurun_out/r2_gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures (keep going), else stop
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r2_smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err || exit $?
cat gpurun_out/r2_bench.json | head -c 600
exit $rc
