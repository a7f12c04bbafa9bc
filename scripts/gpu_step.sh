#!/bin/bash
# Run one GPU step under its own time limit; stop the chain at anything fault-like:
# abort/segv/timeout exit codes, or a HIP memory-access error in the output.
# usage: scripts/gpu_step.sh <timeout_s> <log> -- cmd...
set -u
t=$1; log=$2; shift 3
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "rc=$rc" >> "$log"
if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|hipErrorLaunchFailure|GPU core dump" "$log"; then
  echo "GPU FAULT reported in $log" >&2; exit 98
fi
case $rc in
  0|1|2|5) exit 0 ;;      # pass / test failures / usage / no tests: safe to continue
  *) echo "FAULT-LIKE EXIT $rc in: $*" >&2; exit 99 ;;
esac
