#!/bin/bash
# Side route (B = 512, 32 progressive, look-ahead 48) with the side decode confined to N CUs.
set -o pipefail
TAG=${1:-cus}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in 0 128 192 0; do
  DINO_SIDE_CUS=$c timeout -k 10 240 python scripts/route_study.py --batch 512 --batches 160 --ks 32 \
    --routes side --side-ahead 48 --warm 70 > gpurun_out/${TAG}_$c.jsonl 2> gpurun_out/${TAG}_$c.err || exit $?
  echo "cus=$c $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read())['images_per_s'])" gpurun_out/${TAG}_$c.jsonl)"
done
