#!/bin/bash
# Session-3 batch: split-stream priority study, 2-rank rehearsal of the N-GPU bench path on
# one card, adaptive k_hresize A/B on C2 and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python scripts/pipe_study.py 30 2,3 > gpurun_out/ps3.log 2>&1 || exit $?
tail -3 gpurun_out/ps3.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --images 8192 --unique 512 \
  > gpurun_out/r2rank.json 2> gpurun_out/r2rank.err || exit $?
head -c 300 gpurun_out/r2rank.json; echo
bash scripts/gpu_ab.sh ab15 vt tpw25 tpw50 || exit $?
AB_ARGS="--mixed --images 8192 --unique 512 --steps 16" bash scripts/gpu_ab.sh ab15c3 vt tpw25 tpw50
