#!/usr/bin/env python
"""Per-launch HBM traffic of every kernel from two rocprofv3 PMC passes.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON

FETCH_DIR / WRITE_DIR hold the ``*counter_collection.csv`` of a
``rocprofv3 --pmc FETCH_SIZE`` and a ``rocprofv3 --pmc WRITE_SIZE`` run of the
same bench command (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
Corrections follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts
TCC_EA0_RDREQ x 64 B while the fabric requests are 128 B, so the read bytes are
2 x FETCH_SIZE; WRITE_SIZE (KiB) is taken as is.  Both include Infinity-Cache
hits (the guide's caveat), so they bound HBM traffic from above.
"""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").strip()
    n = n.split("::")[-1] if n.startswith("dino::") else n
    return n.split("<")[0] if n.startswith("k_") else n[:60]


def load(d: str, counter: str) -> dict:
    per = defaultdict(list)
    files = list(Path(d).rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                key = (short(row["Kernel_Name"]), row.get("Dispatch_Id"))
                per[key].append(float(row["Counter_Value"]))
    out = defaultdict(list)
    for (k, _), vals in per.items():
        out[k].append(sum(vals))  # one value per dispatch (summed over XCD/instance rows)
    return out


def main() -> None:
    fd, wd, outp = sys.argv[1:4]
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    res = {"_note": "per-launch bytes; read = 2 x FETCH_SIZE(KiB) x 1024 (gfx950 correction), "
                    "write = WRITE_SIZE(KiB) x 1024; Infinity-Cache hits included (upper bound on HBM)"}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        rd = 2 * 1024 * sum(f) / len(f) if f else None
        wr = 1024 * sum(w) / len(w) if w else None
        res[k] = {"launches": max(len(f), len(w)),
                  "fetch_size_kib_raw": round(sum(f) / len(f), 1) if f else None,
                  "read_bytes_per_launch": round(rd) if rd is not None else None,
                  "write_bytes_per_launch": round(wr) if wr is not None else None,
                  "hbm_bytes_per_launch": round((rd or 0) + (wr or 0))}
    Path(outp).write_text(json.dumps(res, indent=1))
    for k, v in res.items():
        if not k.startswith("_"):
            print(f"{k:24s} {v['launches']:4d}  read {v['read_bytes_per_launch']}  write {v['write_bytes_per_launch']}")


if __name__ == "__main__":
    main()
