#!/bin/bash
# A/B of the contiguous-band work mapping of k_color / k_idct (round 6) against the
# grid-strided one: GPU parity tests on the default build, then C2 / C3 bench legs per
# variant (interleaved, two rounds) and FETCH / WRITE passes at C3 for the two ends.
# usage: scripts/gpu_ab_band.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r6ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
for rep in 1 2; do
  for v in default strided colband idctband; do
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
for v in default strided; do
  if [ $v = default ]; then LIB=dataloader_amd/libdino_ingest.so; else LIB=build/lib_$v.so; fi
  export DINO_INGEST_LIB=$LIB
  BENCH="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --depth 1 --mixed --unique 1024 --images 4096"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${v}_fetch -o run --output-format csv -- $BENCH > $OUT/${v}_fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/${v}_write -o run --output-format csv -- $BENCH > $OUT/${v}_write.log 2>&1 || exit $?
  python scripts/pmc_traffic.py $OUT/${v}_fetch $OUT/${v}_write $OUT/pmc_c3_${v}.json || exit $?
  python -c "
import json; d = json.load(open('$OUT/pmc_c3_${v}.json'))
print('$v', {k: (round(d[k]['read_bytes_per_launch'] / 1e6), round(d[k]['write_bytes_per_launch'] / 1e6)) for k in ('k_color', 'k_idct')})"
done
unset DINO_INGEST_LIB
exit 0
