#!/usr/bin/env python
"""Per-kernel mean (per dispatch) of every counter in rocprofv3 --pmc CSV dirs.

usage: pmc_counters.py DIR [DIR ...]   (prints a table; dispatch rows summed over instances)
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import short  # noqa: E402

per = defaultdict(float)
disp = defaultdict(set)
for d in sys.argv[1:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                per[(k, row["Counter_Name"])] += float(row["Counter_Value"])
                disp[(k, row["Counter_Name"])].add(row.get("Dispatch_Id"))
kern = sorted({k for k, _ in per})
ctrs = sorted({c for _, c in per})
print("kernel".ljust(16) + "".join(c[-18:].rjust(20) for c in ctrs))
for k in kern:
    print(k[:16].ljust(16) + "".join(
        (f"{per[(k, c)] / max(1, len(disp[(k, c)])):20.4g}" if (k, c) in per else " " * 20) for c in ctrs))
