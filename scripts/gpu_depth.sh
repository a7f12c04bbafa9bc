#!/bin/bash
# C2 bench line at several pipeline depths (batches in flight) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for dp in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --depth $dp > gpurun_out/dp_$dp.json 2> gpurun_out/dp_$dp.err || exit $?
done
for dp in 1 2 3 4; do python scripts/show_bench.py gpurun_out/dp_$dp.json; done
