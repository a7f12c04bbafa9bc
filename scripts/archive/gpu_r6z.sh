# c2_prog: the copy stream from the least-priority queue pool (default) or on a queue of its own
set -o pipefail
export TMPDIR=/tmp
R6TAG=r6z bash scripts/gpu_prog_ab.sh poolA:X=1 ownA:DINO_COPY_QUEUE=own poolB:X=1 ownB:DINO_COPY_QUEUE=own \
  poolC:X=1 ownC:DINO_COPY_QUEUE=own || exit 1
