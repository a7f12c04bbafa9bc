#!/bin/bash
# A/B: the C2 and C3 bench lines (no CPU baseline, no extra legs) for every build/lib_<name>.so given,
# on one box; optionally the GPU tests first (TESTS=1, on the in-tree library).
# usage: [TESTS=1 [TESTLIB=name]] scripts/gpu_ab_c23.sh TAG name1 name2 ...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ "${TESTS:-0}" = 1 ]; then
  # TESTLIB=name: the tests run on build/lib_<name>.so instead of the in-tree library
  if [ -n "${TESTLIB:-}" ]; then export DINO_INGEST_LIB=build/lib_${TESTLIB}.so; fi
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_gputests.log
  unset DINO_INGEST_LIB
fi
for n in "$@"; do
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
    > gpurun_out/${TAG}_c2_$n.json 2> gpurun_out/${TAG}_c2_$n.err || exit $?
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 300 python bench.py --mixed --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
    --images 8192 --unique 1024 > gpurun_out/${TAG}_c3_$n.json 2> gpurun_out/${TAG}_c3_$n.err || exit $?
done
for n in "$@"; do
  for w in c2 c3; do
    python - "$n" "$w" gpurun_out/${TAG}_${w}_$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
k = d["kernels_ms_per_step"]
top = sorted(k.items(), key=lambda x: -x[1])[:6]
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d.get("serialized_ms_per_step"), " ".join(f"{a}={b:.3f}" for a, b in top))
PY
  done
done
