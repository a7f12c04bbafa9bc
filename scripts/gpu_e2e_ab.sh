#!/bin/bash
# e2e feed A/B: batches in flight / copier threads / feed kind / copy stream.
# usage: scripts/gpu_e2e_ab.sh TAG "feed threads inflight copystream" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-e2e}
shift
for v in "$@"; do
  set -- $v
  f=gpurun_out/${TAG}_$1_t$2_d$3_cs$4
  DINO_COPY_STREAM=$4 timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extras --e2e \
    --e2e-feed $1 --gather-threads $2 --e2e-in-flight $3 > $f.json 2> $f.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['e2e']; print(sys.argv[1], d['value'], e['e2e_images_per_s'], e['e2e_host_ms_per_batch'], e.get('e2e_feed_stats'))" $f.json
done
