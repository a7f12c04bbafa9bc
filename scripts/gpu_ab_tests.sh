#!/bin/bash
# GPU tests (fail-fast), then the A/B bench lines: scripts/gpu_ab_tests.sh TAG name1 name2 ...
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_e4.log -- python scripts/exp_batches.py 512 full 0,0,512 || exit $?
scripts/gpu_step.sh 600 gpurun_out/${TAG}_tests.log -- python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 gpurun_out/${TAG}_tests.log
bash scripts/gpu_ab.sh "$@"
