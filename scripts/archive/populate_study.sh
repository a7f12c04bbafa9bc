#!/bin/bash
# e2e leg with the native feed's shard pre-fault on / off (DINO_FEED_POPULATE), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2 3; do for pp in 1 0; do
  DINO_FEED_POPULATE=$pp DINO_FEED_TRACE=gpurun_out/pp${pp}_ft_$i.txt timeout -k 10 300 python bench.py --only-leg e2e --procs 16 \
    > gpurun_out/pp${pp}_$i.json 2> gpurun_out/pp${pp}_$i.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['e2e_images_per_s'], d['e2e_feed_stats'])" gpurun_out/pp${pp}_$i.json
  python scripts/feed_trace.py gpurun_out/pp${pp}_ft_$i.txt
done; done
