"""Reads gpurun_out/timeline_e2e.json (bench.py e2e leg with DINO_TIMELINE=1) and says what
paced each batch: the host (the copy was issued late), the copy, or the device.

Host stamps (perf_counter) and device stamps (HIP timing events) are aligned by the smallest
(copy start - copy issue) over the run (a copy never starts before it is issued)."""
import json
import sys


def main() -> int:
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/timeline_e2e.json"
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tl = json.load(open(path))
    rs = [r for r in tl if "c0" in r]
    off = min(r["c0"] - r["issue"] for r in rs)  # device time = host time + off
    rs = rs[skip:]
    busy = sorted((r["k0"], r["k1"]) for r in rs)
    span = busy[-1][1] - busy[0][0]
    idle, cur = 0.0, busy[0][1]
    for s, e in busy[1:]:
        if s > cur:
            idle += s - cur
        cur = max(cur, e)
    n = len(rs)
    print(f"{n} batches, {span / n * 1e3:.3f} ms per batch on the device span; "
          f"no batch running {idle / span:.1%} of it")
    acc = {"pull_wait": 0, "launch": 0, "issue_to_copy": 0, "copy": 0, "copy_to_kern": 0, "kern": 0}
    late = 0
    prev_k1 = {}
    rows = []
    for r in rs:
        issue_dev = r["issue"] + off
        acc["pull_wait"] += r["t0"] - r["pull"]
        acc["launch"] += r["t1"] - r["t0"]
        acc["issue_to_copy"] += r["c0"] - issue_dev
        acc["copy"] += r["c1"] - r["c0"]
        acc["copy_to_kern"] += r["k0"] - r["c1"]
        acc["kern"] += r["k1"] - r["k0"]
        # what the slot's kernels waited for: the copy (k0 ~ c1) or the slot's previous batch
        pk = prev_k1.get(r["slot"], -1)
        why = "copy" if r["c1"] >= pk else "slot"
        if why == "copy" and r["c1"] - r["c0"] < (r["k0"] - issue_dev) - 0.3e-3:
            late += 1
        prev_k1[r["slot"]] = r["k1"]
        rows.append((r["pull"] + off, r["t0"] + off, issue_dev, r["c0"], r["c1"], r["k0"], r["k1"], r["slot"], why))
    print("mean ms per batch:", {k: round(v / n * 1e3, 3) for k, v in acc.items()})
    print(f"batches whose kernels started on their copy's end: "
          f"{sum(1 for x in rows if x[-1] == 'copy')} of {n}")
    # kernels of a batch that start right as another slot's batch ends (within 30 us), while
    # neither its copy nor its own slot held it: the slots' streams share a hardware queue
    ends = [(x[6], x[7]) for x in rows]
    chained = 0
    for x in rows:
        if any(s != x[7] and 0 <= x[5] - e < 30e-6 for e, s in ends) and x[5] - x[4] > 30e-6:
            chained += 1
    print(f"batches starting on another slot's end: {chained} of {n}")
    t00 = rows[0][0]
    print(" pull     t0    issue   c0     c1     k0     k1   slot why (ms, device clock)")
    for x in rows[:40]:
        print(" ".join(f"{(v - t00) * 1e3:6.2f}" for v in x[:7]), x[7], x[8])
    return 0


if __name__ == "__main__":
    sys.exit(main())
