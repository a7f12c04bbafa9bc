# the native feed's shard I/O modes (DINO_FEED_IO) at 8 ranks on the GPU box's host, twice each,
# alternated; then the e2e leg (1 rank, GPU) per mode
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${R6TAG:-r6i}
mkdir -p $OUT
for rep in 1 2; do
  for io in mmap index pread; do
    DINO_FEED_IO=$io timeout -k 10 120 python -u scripts/host_feed_study.py --ranks 8 --threads 2 --seconds 8 > $OUT/hf_${io}_$rep.json 2> $OUT/hf_${io}_$rep.err || { echo "hf $io failed"; tail -5 $OUT/hf_${io}_$rep.err; exit 1; }
    python - $io $OUT/hf_${io}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = [x["images_per_s"] for x in d["per_rank"]]
print(sys.argv[1], "min", min(r), "mean", round(sum(r) / len(r)), "sum", d["host_feeds_images_per_s_sum"],
      "GB/s", d["host_feeds_shm_read_GBs_sum"], "open_s", [round(x.get("feed", {}).get("open_s", 0), 2) for x in d["per_rank"]][:3])
PY
  done
done
for io in mmap pread; do
  DINO_FEED_IO=$io timeout -k 10 200 python -u bench.py --only-leg e2e --steps 98 --warmup 5 > $OUT/e2e_$io.json 2> $OUT/e2e_$io.err || { echo "e2e $io failed"; tail -5 $OUT/e2e_$io.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/e2e_$io.json').read().strip().splitlines()[-1]); print('$io e2e', d['e2e_images_per_s'], d.get('e2e_feed_stats'))"
done
