# small side pools to the wave decoder: side-route GPU tests, then the c2_prog leg three times
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${R6TAG:-r6o}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 250 --timeout-method thread -p no:cacheprovider tests/test_gpu_round6.py \
  tests/test_gpu_round3.py -k "lane or damaged or side_route or dropin" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
R6TAG=${R6TAG:-r6o} bash scripts/gpu_prog_ab.sh plan1:X=1 plan2:X=1 plan3:X=1 plan4:X=1 || exit 1
