#!/bin/bash
# Side-path knob sweep (16 progressive per 256-image batch): pool size, contexts, dedicated
# queues.  usage: scripts/gpu_side_sweep.sh TAG "MIN:ENGINES:DEDICATED ..." [side_ahead]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=$1; CONFS=$2; AHEAD=${3:-48}
for c in $CONFS; do
  IFS=: read MIN ENG DED <<< "$c"
  DINO_SIDE_MIN=$MIN DINO_SIDE_ENGINES=$ENG DINO_SIDE_DEDICATED=$DED timeout -k 10 200 python scripts/route_study.py \
    --batches ${BATCHES:-120} --warm ${WARM:-60} --side-ahead $AHEAD --ks 16 --routes side > gpurun_out/${TAG}_$c.jsonl 2> gpurun_out/${TAG}_$c.err || exit $?
  echo "$c $(tail -1 gpurun_out/${TAG}_$c.jsonl)"
done
