#!/bin/bash
# Development GPU session: a sync-checked batch, the GPU tests, a C2 and a C3 bench
# line (no CPU baseline).  usage: scripts/gpu_r2_dev.sh TAG
set -o pipefail
TAG=${1:-dev}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_e4.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_tests.log -- python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider && \
scripts/gpu_step.sh 300 gpurun_out/${TAG}_c2.json -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline && \
scripts/gpu_step.sh 300 gpurun_out/${TAG}_c3.json -- python bench.py --mixed --no-cpu-baseline --images 8192 --unique 2048 --steps 16 && \
tail -3 gpurun_out/${TAG}_tests.log && python scripts/show_bench.py gpurun_out/${TAG}_c2.json gpurun_out/${TAG}_c3.json
