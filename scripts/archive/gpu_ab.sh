#!/bin/bash
# A/B: the C2 bench line (no CPU baseline) for every build/lib_<name>.so given, on one box.
# usage: scripts/gpu_ab.sh TAG name1 name2 ...   (AB_ARGS: extra bench arguments, e.g. for C3)
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in "$@"; do
  DINO_INGEST_LIB=build/lib_$n.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline $AB_ARGS \
    > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || exit $?
done
for n in "$@"; do python scripts/show_bench.py gpurun_out/${TAG}_$n.json; done
