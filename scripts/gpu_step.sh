#!/bin/bash
# Run GPU steps in order; stop at the first fault-like exit (abort/segv/timeout/kill).
# usage: scripts/gpu_step.sh <timeout_s> <log> -- cmd...   (chain several with ;)
set -u
t=$1; log=$2; shift 3
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "rc=$rc" >> "$log"
case $rc in
  0|1|2|5) exit 0 ;;      # pass / test failures / usage / no tests: safe to continue
  *) echo "FAULT-LIKE EXIT $rc in: $*" >&2; exit 99 ;;
esac
