#!/bin/bash
# Side route (B = 512, 32 progressive) after another pipeline in the same process:
# (a) after an all-baseline pipeline (k = 0), (b) after the in-batch device route.
set -o pipefail
TAG=${1:-po}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python scripts/route_study.py --batch 512 --batches 160 --ks 0,32 --routes side --side-ahead 48 \
  --warm 70 > gpurun_out/${TAG}_a.jsonl 2> gpurun_out/${TAG}_a.err || exit $?
python -c "import json,sys; print('a', [(json.loads(l)['k_progressive'], json.loads(l)['images_per_s']) for l in open(sys.argv[1])])" gpurun_out/${TAG}_a.jsonl
timeout -k 10 400 python scripts/route_study.py --batch 512 --batches 100 --ks 32 --routes device,side --side-ahead 48 \
  --warm 40 > gpurun_out/${TAG}_b.jsonl 2> gpurun_out/${TAG}_b.err || exit $?
python -c "import json,sys; print('b', [(json.loads(l)['route'], json.loads(l)['images_per_s']) for l in open(sys.argv[1])])" gpurun_out/${TAG}_b.jsonl
