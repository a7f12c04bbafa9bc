# c2_prog under the round-6 side plan: copier threads of the host pack (one box, interleaved)
set -o pipefail
export TMPDIR=/tmp
R6TAG=r6p bash scripts/gpu_prog_ab.sh g8a:DINO_GATHER_THREADS=8 g16a:DINO_GATHER_THREADS=16 g4a:DINO_GATHER_THREADS=4 \
  g8b:DINO_GATHER_THREADS=8 g16b:DINO_GATHER_THREADS=16 g4b:DINO_GATHER_THREADS=4 || exit 1
