#!/bin/bash
# e2e feed A/B: native shard feed vs the Python prefetch thread, copier threads.
# usage: scripts/gpu_e2e_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-e2e}
for v in "native 8" "python 8" "native 4" "native 12"; do
  set -- $v
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extras --e2e \
    --e2e-feed $1 --gather-threads $2 > gpurun_out/${TAG}_$1_t$2.json 2> gpurun_out/${TAG}_$1_t$2.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['e2e']; print(sys.argv[1], d['value'], e['e2e_images_per_s'], e['e2e_host_ms_per_batch'], e.get('e2e_feed_stats'))" gpurun_out/${TAG}_$1_t$2.json
done
