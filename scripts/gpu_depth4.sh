#!/bin/bash
# C2 and C3 bench lines at pipeline depths 2-4 (batches in flight), one box.
set -o pipefail
TAG=${1:-dp4}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for dp in 3 2 4; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras --depth $dp > gpurun_out/${TAG}_c2_$dp.json 2> gpurun_out/${TAG}_c2_$dp.err || exit $?
  timeout -k 10 300 python bench.py --mixed --steps 20 --warmup 3 --no-cpu-baseline --no-extras --images 8192 --unique 1024 --depth $dp > gpurun_out/${TAG}_c3_$dp.json 2> gpurun_out/${TAG}_c3_$dp.err || exit $?
  echo "depth $dp c2 $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().splitlines()[-1])['value'])" gpurun_out/${TAG}_c2_$dp.json) c3 $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().splitlines()[-1])['value'])" gpurun_out/${TAG}_c3_$dp.json)"
done
