#!/bin/bash
# A/B of k_color quads per lane per iteration (2) and k_idct entries prefetched per lane (8)
# (B = 512 parity on each variant first), then C2 / C3 bench legs per variant (interleaved, two rounds)
# usage: scripts/archive/gpu_ab_cb.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r6cb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for L in cb2 pre8; do
  DINO_INGEST_LIB=build/lib_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_round5.py -k "b512" -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    > $OUT/gputests_$L.log 2>&1 || { tail -30 $OUT/gputests_$L.log; exit 1; }
  tail -1 $OUT/gputests_$L.log
done
for rep in 1 2; do
  for v in default cb2 pre8; do
    if [ $v = default ]; then LIB=dataloader_amd/libdino_ingest.so; else LIB=build/lib_$v.so; fi
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > $OUT/c2_${v}_$rep.json 2> $OUT/c2_${v}_$rep.err || exit $?
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --mixed --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
      > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    python - $OUT/c2_${v}_$rep.json $OUT/c3_${v}_$rep.json $v <<'EOF'
import json, sys
a, b = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:3])
k = lambda d, n: d.get("kernels_ms_per_step", {}).get(n)
print(sys.argv[3], "C2", a["value"], "color", k(a, "k_color"), "idct", k(a, "k_idct"),
      "| C3", b["value"], "color", k(b, "k_color"), "idct", k(b, "k_idct"), flush=True)
EOF
  done
done
exit 0
