#!/bin/bash
# SQ counters of k_prog on a progressive-only workload (one pass, 8 SQ counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/progpmc -o run --output-format csv -- python3 scripts/prog_only.py > gpurun_out/progpmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/progpmc/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f)):
    if "k_prog" in row["Kernel_Name"]:
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
for k, v in sorted(acc.items()):
    print(f"{k:20s} {v:.4g}")
PY
