#!/bin/bash
# A/B of k_hresize register budget (6 waves per SIMD, spills) against the default
# variant with both, then C2 / C3 bench legs per variant (interleaved, two rounds)
# usage: scripts/gpu_ab_wgs.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r6hr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
DINO_INGEST_LIB=build/lib_hr6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_round5.py -k "b512" -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
for rep in 1 2; do
  for v in default hr6; do
    if [ $v = default ]; then LIB=dataloader_amd/libdino_ingest.so; else LIB=build/lib_$v.so; fi
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > $OUT/c2_${v}_$rep.json 2> $OUT/c2_${v}_$rep.err || exit $?
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --mixed --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
      > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    python - $OUT/c2_${v}_$rep.json $OUT/c3_${v}_$rep.json $v <<'EOF'
import json, sys
a, b = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:3])
k = lambda d, n: d.get("kernels_ms_per_step", {}).get(n)
print(sys.argv[3], "C2", a["value"], "hresize", k(a, "k_hresize"),
      "| C3", b["value"], "hresize", k(b, "k_hresize"), flush=True)
EOF
  done
done
exit 0
