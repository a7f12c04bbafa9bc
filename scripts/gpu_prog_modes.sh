#!/bin/bash
# The side route (B = 512, 32 progressive) built directly and through MI355XBackend, each in
# a fresh process.
set -o pipefail
TAG=${1:-pm}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for mode in direct backend direct backend; do
  if [ $mode = backend ]; then B=--backend; else B=; fi
  timeout -k 10 300 python scripts/route_study.py --batch 512 --batches 160 --ks 32 --routes side --side-ahead 48 \
    --warm 70 $B >> gpurun_out/${TAG}_$mode.jsonl 2>> gpurun_out/${TAG}_$mode.err || exit $?
  echo "$mode $(tail -1 gpurun_out/${TAG}_$mode.jsonl | python -c "import json,sys; print(json.loads(sys.stdin.read())['images_per_s'])")"
done
