#!/bin/bash
# MFMA horizontal pass: GPU tests, then C2 / C3 A/B against the v_dot4 kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-mf}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab.sh ${TAG}_c2 mf0 mf1 mf2 mf0 mf1 mf2 > gpurun_out/${TAG}_c2.txt 2>&1 || exit $?
AB_ARGS="--mixed --no-extras --images 4096 --unique 512 --steps 20" bash scripts/gpu_ab.sh ${TAG}_c3 mf0 mf1 mf2 mf0 mf1 mf2 > gpurun_out/${TAG}_c3.txt 2>&1 || exit $?
