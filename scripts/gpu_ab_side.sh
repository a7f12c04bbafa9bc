#!/bin/bash
# A/B of library variants on the side route (B = 512, 32 progressive, look-ahead 48) and on C2.
# usage: scripts/gpu_ab_side.sh TAG name1 name2 ...   (build/lib_<name>.so)
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in "$@"; do
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 240 python scripts/route_study.py --batch 512 --batches 160 --ks 32 \
    --routes side --side-ahead 48 --warm 70 > gpurun_out/${TAG}_side_$n.jsonl 2> gpurun_out/${TAG}_side_$n.err || exit $?
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
    > gpurun_out/${TAG}_c2_$n.json 2> gpurun_out/${TAG}_c2_$n.err || exit $?
  echo "$n side $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read())['images_per_s'])" gpurun_out/${TAG}_side_$n.jsonl) c2 $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().splitlines()[-1])['value'])" gpurun_out/${TAG}_c2_$n.json)"
done
