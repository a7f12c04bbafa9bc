# c2_prog at look-ahead 256: lane decoder waves per launch, half-size rings, priority; wave decoder (one box)
set -o pipefail
export TMPDIR=/tmp
export R6TAG=r6lc STEPS=400
L=DINO_PROG_LANE=1,DINO_SIDE_AHEAD=256,DINO_SIDE_MAX=4096
bash scripts/gpu_prog_ab.sh lane:$L lane_w128:$L,DINO_PLSCAN_WAVES=128 lane_w256:$L,DINO_PLSCAN_WAVES=256 \
  lsmall:$L,DINO_INGEST_LIB=build/lib_lsmall.so lane_prio:$L,DINO_SCAN_PRIO=1 \
  wave_a256_m2048:DINO_SIDE_AHEAD=256,DINO_SIDE_MAX=2048 lane_again:$L
