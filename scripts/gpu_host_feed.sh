#!/bin/bash
# Host half at 8 ranks on the GPU box's host cores: per-feed scaling with copier
# threads, 8 concurrent feeds at 2 threads (16 cores), and 8 feeds with rank 0 on the GPU pipeline.
set -o pipefail
TAG=${1:-hf}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { timeout -k 10 300 python scripts/host_feed_study.py "$@" >> gpurun_out/${TAG}.jsonl 2>> gpurun_out/${TAG}.err || exit $?; tail -c 400 gpurun_out/${TAG}.jsonl; echo; }
run --ranks 1 --threads 2 --seconds 6
run --ranks 1 --threads 8 --seconds 6
run --ranks 8 --threads 2 --seconds 8
run --ranks 8 --threads 2 --seconds 8 --gpu-rank
