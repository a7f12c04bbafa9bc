#!/bin/bash
# SQ counters of k_pscan on a progressive-only workload (two passes of <= 8 SQ counters).
# usage: scripts/gpu_pscan_pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-pp}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES \
  -d gpurun_out/${TAG}_a -o run --output-format csv -- python3 scripts/prog_only.py > gpurun_out/${TAG}_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
  -d gpurun_out/${TAG}_b -o run --output-format csv -- python3 scripts/prog_only.py > gpurun_out/${TAG}_b.log 2>&1
python3 - "$TAG" <<'PY'
import csv, glob, collections, sys
tag = sys.argv[1]
for part in "ab":
    fs = glob.glob(f"gpurun_out/{tag}_{part}/**/run_counter_collection.csv", recursive=True)
    if not fs:
        print(part, "no data"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(fs[0])):
        for k in ("k_pscan", "k_pwalk"):
            if k in row["Kernel_Name"]:
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, d in acc.items():
        print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
PY
