#!/bin/bash
# The side route (backend default) with a quarter of each batch progressive (VERDICT r3 #2:
# 64 per 256; round 3: 8.6k img/s), and 1/16 for reference, on the in-tree library.
# usage: scripts/gpu_prog64.sh TAG
set -o pipefail
TAG=${1:-p64}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python scripts/route_study.py --batch 256 --batches 160 --ks 64,16 --routes side --side-ahead 48 \
  --warm 70 > gpurun_out/${TAG}_side256.jsonl 2> gpurun_out/${TAG}_side256.err || exit $?
cat gpurun_out/${TAG}_side256.jsonl
