#!/bin/bash
# GPU session: parity tests + smoke, the driver's default bench line, depth-1 rocprofv3
# kernel summaries (C2, C3) and the FETCH / WRITE PMC passes (C2, C3).
# usage: scripts/gpu_session.sh TAG [tests|bench|prof|pmc|all]  (comma list)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5}
WHAT=${2:-all}
has() { [ "$WHAT" = all ] || [[ ",$WHAT," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 840 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_gputests.log
  timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
fi
if has bench; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
  head -c 300 gpurun_out/${TAG}_bench.json; echo
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --depth 1 --procs 0 --images 8192 \
    > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c3 -o run --output-format csv -- \
    python bench.py --mixed --steps 10 --warmup 2 --no-cpu-baseline --no-extras --depth 1 --images 4096 --unique 1024 \
    > gpurun_out/${TAG}_prof_c3.log 2>&1 || exit $?
fi
if has pmc; then
  for W in c2 c3; do
    if [ $W = c3 ]; then EXTRA="--mixed --unique 1024 --images 4096"; else EXTRA="--images 8192 --procs 0"; fi
    BENCH="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --depth 1 $EXTRA"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_${W}_fetch -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${W}_fetch.log 2>&1 || exit $?
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_${W}_write -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_${W}_write.log 2>&1 || exit $?
    python scripts/pmc_traffic.py gpurun_out/${TAG}_${W}_fetch gpurun_out/${TAG}_${W}_write gpurun_out/${TAG}_pmc_${W}.json || exit $?
  done
fi
exit 0
