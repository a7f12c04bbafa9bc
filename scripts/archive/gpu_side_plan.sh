# Side plan (round 6): GPU tests on the new defaults, then the c2_prog leg with the default plan
# (look-ahead 256, lane decoder, pools of 4096) against the wave decoder at the same look-ahead
# and the round-5 plan (look-ahead 48, wave, pools of 512), one box
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6sp}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
export R6TAG=${TAG:-r6sp}
bash scripts/gpu_prog_ab.sh plan1:X=1 wave256:DINO_SIDE_DECODER=wave,DINO_SIDE_MAX=2048 r5plan:DINO_SIDE_AHEAD=48,DINO_SIDE_DECODER=wave \
  plan2:X=1 r5plan2:DINO_SIDE_AHEAD=48,DINO_SIDE_DECODER=wave plan3:X=1 || exit 1
