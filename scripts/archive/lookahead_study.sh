#!/bin/bash
# e2e leg with the native feed's look-ahead (= opener threads, at most 4) at 2 and 4, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do for la in 2 4; do
  DINO_FEED_LOOKAHEAD=$la DINO_FEED_TRACE=gpurun_out/la${la}_ft_$i.txt timeout -k 10 300 python bench.py --only-leg e2e --procs 16 \
    > gpurun_out/la${la}_$i.json 2> gpurun_out/la${la}_$i.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['e2e_images_per_s'], d['e2e_feed_stats'])" gpurun_out/la${la}_$i.json
  python scripts/feed_trace.py gpurun_out/la${la}_ft_$i.txt
done; done
