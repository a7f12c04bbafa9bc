#!/bin/bash
# cProfile of one host-fed bench leg in its own process (main thread: launches + waits).
# usage: scripts/prof_leg.sh TAG e2e|c2_prog
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
TAG=$1; LEG=$2
timeout -k 10 600 python scripts/prof_leg.py gpurun_out/${TAG}_${LEG}.prof $LEG --procs 16 --steps 20 --warmup 5 \
  > gpurun_out/${TAG}_${LEG}.json 2> gpurun_out/${TAG}_${LEG}_prof.txt || exit $?
head -c 600 gpurun_out/${TAG}_${LEG}.json; echo
