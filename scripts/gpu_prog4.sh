#!/bin/bash
# Round-4 progressive study: side route at B = 512 with 32 progressive per batch (the c2_prog leg's
# mix) at look-ahead 16 / 48, and the progressive-only launch capacity at 1 / 2 scan waves per CU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-p4}
for sa in 16 48; do
  timeout -k 10 240 python scripts/route_study.py --batch 512 --batches 140 --ks 32 --routes side --side-ahead $sa --warm 60 \
    > gpurun_out/${TAG}_route_sa$sa.jsonl 2> gpurun_out/${TAG}_route_sa$sa.err || exit $?
  cat gpurun_out/${TAG}_route_sa$sa.jsonl
done
for pc in 1 2; do
  DINO_PSCAN_PER_CU=$pc timeout -k 10 240 python scripts/prog_scale.py --ns 512,2048 --reps 3 --streams 4 \
    > gpurun_out/${TAG}_scale_pc$pc.jsonl 2> gpurun_out/${TAG}_scale_pc$pc.err || exit $?
  cat gpurun_out/${TAG}_scale_pc$pc.jsonl
done
