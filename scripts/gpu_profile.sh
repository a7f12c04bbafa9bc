#!/bin/bash
# Profiling session: depth-1 rocprofv3 kernel summaries (C2, C3), FETCH / WRITE PMC passes,
# SQ instruction counters, k_huff1 phase split (instrumented build).
# usage: scripts/gpu_profile.sh TAG [prof,pmc,sq,phases]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r5p}
WHAT=${2:-prof,pmc,sq,phases}
has() { [[ ",$WHAT," == *",$1,"* ]]; }
if has prof; then
  bash scripts/gpu_session.sh $TAG prof || exit $?
fi
if has pmc; then
  bash scripts/gpu_session.sh $TAG pmc || exit $?
fi
if has sq; then
  bash scripts/gpu_sq.sh $TAG || exit $?
fi
if has phases; then
  timeout -k 10 300 python -u scripts/huff_phases.py > gpurun_out/${TAG}_huff_phases_c2.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/huff_phases.py --mixed > gpurun_out/${TAG}_huff_phases_c3.txt 2>&1 || exit $?
  cat gpurun_out/${TAG}_huff_phases_c2.txt gpurun_out/${TAG}_huff_phases_c3.txt
fi
exit 0
