#!/bin/bash
# e2e timeline + C2 line with the role streams from torch's pool, from the least priority's
# pool (DINO_ROLE_STREAMS=low), and with 8 hardware queues per priority.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" DINO_TIMELINE=1 timeout -k 10 300 python bench.py --only-leg e2e --procs 16 > gpurun_out/rs_e2e_$tag.json 2> gpurun_out/rs_e2e_$tag.err || return $?
  mv gpurun_out/timeline_e2e.json gpurun_out/rs_tl_$tag.json
  env "$@" timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/rs_c2_$tag.json 2> gpurun_out/rs_c2_$tag.err || return $?
}
run torch DINO_ROLE_STREAMS=torch && run low DINO_ROLE_STREAMS=low && run q8 GPU_MAX_HW_QUEUES=8 || exit $?
for t in torch low q8; do
  echo "== $t"; head -c 120 gpurun_out/rs_e2e_$t.json; echo
  python scripts/e2e_timeline.py gpurun_out/rs_tl_$t.json | sed -n 1,4p
  python scripts/show_bench.py gpurun_out/rs_c2_$t.json
done
