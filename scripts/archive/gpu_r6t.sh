# c2_prog: hardware queues per process (GPU_MAX_HW_QUEUES 4 = the box default, 8, 16), interleaved
set -o pipefail
export TMPDIR=/tmp
R6TAG=r6t bash scripts/gpu_prog_ab.sh q4a:GPU_MAX_HW_QUEUES=4 q8a:GPU_MAX_HW_QUEUES=8 q16a:GPU_MAX_HW_QUEUES=16 \
  q4b:GPU_MAX_HW_QUEUES=4 q8b:GPU_MAX_HW_QUEUES=8 q16b:GPU_MAX_HW_QUEUES=16 || exit 1
