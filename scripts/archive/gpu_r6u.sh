# c2_prog: staging ring +0 / +16 buffers (interleaved)
set -o pipefail
export TMPDIR=/tmp
R6TAG=r6u bash scripts/gpu_prog_ab.sh s0a:DINO_STAGING_EXTRA=0 s16a:DINO_STAGING_EXTRA=16 s0b:DINO_STAGING_EXTRA=0 \
  s16b:DINO_STAGING_EXTRA=16 s0c:DINO_STAGING_EXTRA=0 s16c:DINO_STAGING_EXTRA=16 || exit 1
