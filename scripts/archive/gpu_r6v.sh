# two-thread prefetcher: the full GPU suite, then the c2_prog leg four times
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${R6TAG:-r6v}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
R6TAG=${R6TAG:-r6v} bash scripts/gpu_prog_ab.sh plan1:X=1 plan2:X=1 plan3:X=1 plan4:X=1 || exit 1
