# c2_prog: side look-ahead x pool size for the wave and lane decoders (one box)
set -o pipefail
export TMPDIR=/tmp
export R6TAG=r6la STEPS=160
bash scripts/gpu_prog_ab.sh wave_a48:X=1 wave_a96_m1024:DINO_SIDE_AHEAD=96,DINO_SIDE_MAX=1024 \
  lane_a48_m1024:DINO_PROG_LANE=1,DINO_SIDE_MAX=1024 lane_a96_m1024:DINO_PROG_LANE=1,DINO_SIDE_AHEAD=96,DINO_SIDE_MAX=1024 \
  lane_a96_m2048:DINO_PROG_LANE=1,DINO_SIDE_AHEAD=96,DINO_SIDE_MAX=2048 lane_a128_m2048:DINO_PROG_LANE=1,DINO_SIDE_AHEAD=128,DINO_SIDE_MAX=2048
