#!/bin/bash
# GPU tests of the coefficient-buffer path, then C2 with a share of progressive JPEGs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-pf}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "progressive or multiscan or damaged or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for f in 0.02 0.1; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --unique 512 --progressive-frac $f > gpurun_out/${TAG}_$f.json 2> gpurun_out/${TAG}_$f.err || exit $?
done
for f in 0.02 0.1; do python scripts/show_bench.py gpurun_out/${TAG}_$f.json; done
python - <<PY
import json
for f in ("0.02", "0.1"):
    for line in reversed(open(f"gpurun_out/${TAG}_{f}.json").read().strip().splitlines()):
        if line.startswith("{"):
            d = json.loads(line); print(f, "k_prog ms/step", d["kernels_ms_per_step"].get("k_prog")); break
PY
timeout -k 10 200 python scripts/prog_phases.py > gpurun_out/${TAG}_phases.txt 2>&1 || true
tail -16 gpurun_out/${TAG}_phases.txt
