#!/bin/bash
# Side route at B = 512, 32 progressive per batch, look-ahead 48: scan waves per CU x side pool size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-p4b}
for cfg in 1:512 2:512 3:512 2:1024 3:1024; do
  pc=${cfg%%:*}; mx=${cfg##*:}
  DINO_PSCAN_PER_CU=$pc DINO_SIDE_MAX=$mx timeout -k 10 240 python scripts/route_study.py --batch 512 --batches 160 --ks 32 \
    --routes side --side-ahead 48 --warm 70 > gpurun_out/${TAG}_pc${pc}_mx${mx}.jsonl 2> gpurun_out/${TAG}_pc${pc}_mx${mx}.err || exit $?
  echo "pc=$pc max=$mx $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d['images_per_s'], d['side_launches'], d['host_ms_per_batch'])" gpurun_out/${TAG}_pc${pc}_mx${mx}.jsonl)"
done
for pc in 3 4; do
  DINO_PSCAN_PER_CU=$pc timeout -k 10 240 python scripts/prog_scale.py --ns 512,1024,2048 --reps 3 --streams 4 \
    > gpurun_out/${TAG}_scale_pc$pc.jsonl 2> gpurun_out/${TAG}_scale_pc$pc.err || exit $?
  cat gpurun_out/${TAG}_scale_pc$pc.jsonl
done
