# Side plan sweep: longer look-aheads / larger pools / a third side context (one box)
set -o pipefail
export TMPDIR=/tmp
export R6TAG=r6sq STEPS=400
bash scripts/gpu_prog_ab.sh a256_m4096:X=1 a384_m6144:DINO_SIDE_AHEAD=384,DINO_SIDE_MAX=6144 \
  a512_m8192:DINO_SIDE_AHEAD=512,DINO_SIDE_MAX=8192 a384_m4096_e3:DINO_SIDE_AHEAD=384,DINO_SIDE_ENGINES=3 \
  a256_m3072:DINO_SIDE_MAX=3072 a256_m4096_again:X=1 || exit 1
