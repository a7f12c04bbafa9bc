#!/bin/bash
# rocprofv3 kernel trace of the default bench (pipelined, depth 3): scripts/gpu_trace.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --images 16384 "$@" > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
tail -c 400 gpurun_out/${TAG}_prof.log
