#!/bin/bash
# Coefficient-buffer decoder session: GPU tests, per-scan phases (instrumented build),
# and the progressive route study.  usage: scripts/gpu_prog2.sh TAG [ks] [routes]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-p2}
KS=${2:-0,16}
ROUTES=${3:-device,side}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python scripts/prog_phases.py > gpurun_out/${TAG}_prog_phases.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/route_study.py --batches 60 --warm 20 --side-ahead 24 --ks $KS --routes $ROUTES \
  > gpurun_out/${TAG}_route.jsonl 2> gpurun_out/${TAG}_route.err || exit $?
cat gpurun_out/${TAG}_route.jsonl
