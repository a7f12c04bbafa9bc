# c2_prog leg under side-decoder settings (env A/B on one box); one JSON line per setting
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${R6TAG:-r6d}
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" DINO_SIDE_TIMING=1 timeout -k 10 240 python -u bench.py --only-leg c2_prog --steps ${STEPS:-96} --warmup 5 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$name" "$OUT/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = d["side"]
print(sys.argv[1], d["value"], "wait", s["per_batch_ms"]["wait_s"], "since_launch", s["per_batch_ms"]["since_launch_s"],
      "gpu_ms", sorted(s.get("gpu_ms_per_launch", []))[len(s.get("gpu_ms_per_launch", [1])) // 2], "launches", s["launches"])
PY
}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  run $name $(echo $envs | tr ',' ' ') || exit 1
done
