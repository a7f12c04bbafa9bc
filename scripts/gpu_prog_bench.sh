#!/bin/bash
# The bench's c2_prog and e2e legs after its C2 leg (one process), and the route study's
# side route, on the in-tree library.
set -o pipefail
TAG=${1:-pb}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --legs c2_prog,e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('c2', d['value'], 'c2_prog', d['c2_prog']['value'], 'e2e', d['e2e']['e2e_images_per_s'])" gpurun_out/${TAG}_bench.json
