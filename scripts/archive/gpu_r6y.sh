# containers written into the batches' own HBM copies (no merge copy): side-route / round-6 GPU
# tests, the full GPU suite, then the c2_prog leg three times
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6y
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
R6TAG=r6y bash scripts/gpu_prog_ab.sh plan1:X=1 plan2:X=1 plan3:X=1 || exit 1
