#!/bin/bash
# Lane-mode AC refinement (k_prefine): GPU tests on the in-tree library, then progressive capacity
# and the side route for the variants given (build/lib_<name>.so).
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputests.log
for n in "$@"; do
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 240 python scripts/prog_scale.py --ns 64,512,2048 --reps 3 --streams 4 \
    > gpurun_out/${TAG}_scale_$n.jsonl 2> gpurun_out/${TAG}_scale_$n.err || exit $?
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 240 python scripts/route_study.py --batch 512 --batches 160 --ks 32 \
    --routes side --side-ahead 48 --warm 70 > gpurun_out/${TAG}_side_$n.jsonl 2> gpurun_out/${TAG}_side_$n.err || exit $?
  echo "$n side $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read())['images_per_s'])" gpurun_out/${TAG}_side_$n.jsonl)"
  cat gpurun_out/${TAG}_scale_$n.jsonl
done
