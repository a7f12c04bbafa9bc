#!/bin/bash
# Round-4 closing call: A/B of the last candidates (record groups, checkpoint stride, the
# k_huff1 write threshold), then the GPU tests, smoke, the default bench line and the
# depth-1 rocprofv3 summaries on the in-tree library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS=1 TESTLIB=rec2 bash scripts/gpu_ab_c23.sh cz base rec2 cps16 fs6144 || exit $?
bash scripts/gpu_r4_final.sh r4x tests,bench,prof || exit $?
