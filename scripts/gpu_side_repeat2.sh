#!/bin/bash
# GPU tests, then the side route run 3 times in one process with HIP's default hardware queues.
set -o pipefail
TAG=${1:-srep2}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 400 python scripts/route_study.py --batch 512 --batches 160 --ks 32 --routes side --side-ahead 48 \
  --warm 70 --repeat 3 > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.err || exit $?
echo "default queues: $(python -c "import json,sys; print([json.loads(l)['images_per_s'] for l in open(sys.argv[1])])" gpurun_out/${TAG}.jsonl)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --legs c2_prog,e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('c2', d['value'], 'c2_prog', d['c2_prog']['value'], 'e2e', d['e2e']['e2e_images_per_s'])" gpurun_out/${TAG}_bench.json
