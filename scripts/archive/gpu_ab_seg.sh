# A/B of the Huffman segment size (2048 kbit default, 1536, 1024): C3 parity at B = 512 on the
# 1024 build, then C2 / C3 bench legs per variant, interleaved, two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/r6seg
mkdir -p $OUT
DINO_INGEST_LIB=build/lib_seg1m.so timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_round5.py -k "b512 or c3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in default seg1536 seg1m; do
    if [ $v = default ]; then LIB=dataloader_amd/libdino_ingest.so; else LIB=build/lib_$v.so; fi
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > $OUT/c2_${v}_$rep.json 2> $OUT/c2_${v}_$rep.err || exit $?
    DINO_INGEST_LIB=$LIB timeout -k 10 200 python bench.py --mixed --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
      > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    python - $OUT/c2_${v}_$rep.json $OUT/c3_${v}_$rep.json $v <<'PY'
import json, sys
a, b = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:3])
k = lambda d, n: d.get("kernels_ms_per_step", {}).get(n)
print(sys.argv[3], "C2", a["value"], "huff1", k(a, "k_huff1"), "| C3", b["value"], "huff1", k(b, "k_huff1"),
      "huff2", k(b, "k_huff2"), "huff3", k(b, "k_huff3"), flush=True)
PY
  done
done
exit 0
