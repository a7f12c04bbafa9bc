#!/bin/bash
# The side route run twice in one process (a second pipeline in a process measured slower:
# c2_prog leg, route studies), with HIP's default hardware queues and with more.
set -o pipefail
TAG=${1:-srep}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for q in default 8 16; do
  if [ $q = default ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
  timeout -k 10 400 python scripts/route_study.py --batch 512 --batches 160 --ks 32 --routes side --side-ahead 48 \
    --warm 70 --repeat 3 > gpurun_out/${TAG}_q$q.jsonl 2> gpurun_out/${TAG}_q$q.err || exit $?
  echo "queues $q: $(python -c "import json,sys; print([json.loads(l)['images_per_s'] for l in open(sys.argv[1])])" gpurun_out/${TAG}_q$q.jsonl)"
done
