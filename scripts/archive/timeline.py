"""Device timeline of a traced run (rocprofv3 --kernel-trace --memory-copy-trace
--output-format csv): how busy the GPU is over the steady part of the run.

usage: python scripts/timeline.py <rocprofv3 output dir> [--skip-frac 0.3] [--marker k_huff1]

Prints, over the window from the first `marker` kernel after `skip-frac` of the run to the
last kernel: the union of kernel time, of copy time, the time with no kernel running, the
mean kernel concurrency, the copies' sizes / rates, and the idle gaps by length."""
import argparse
import csv
import glob
import os
import sys
from collections import Counter


def _rows(d: str, pat: str) -> list[dict]:
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def _union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip-frac", type=float, default=0.3)
    ap.add_argument("--marker", default="k_huff1")
    a = ap.parse_args()
    ks = _rows(a.dir, "*kernel_trace.csv")
    cs = _rows(a.dir, "*memory_copy_trace.csv")
    if not ks:
        print("no kernel trace under", a.dir)
        return 1
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
             r.get("Queue_Id", ""), r.get("Stream_Id", "")) for r in ks]
    kern.sort()
    marks = [k for k in kern if a.marker in k[2]]
    t_first = kern[0][0] + a.skip_frac * (kern[-1][1] - kern[0][0])
    m0 = next((k[0] for k in marks if k[0] >= t_first), t_first)
    t1 = max(k[1] for k in kern)
    win = [k for k in kern if k[0] >= m0]
    span = t1 - m0
    busy, gaps = _union([(s, e) for s, e, *_ in win])
    conc = sum(e - s for s, e, *_ in win) / max(1, busy)
    cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""),
           int(r.get("Bytes", r.get("Size", 0)) or 0)) for r in cs]
    cpw = [c for c in cp if c[0] >= m0]
    cbusy, _ = _union([(s, e) for s, e, *_ in cpw])
    n_mark = sum(1 for k in win if a.marker in k[2])
    print(f"window {span / 1e6:.2f} ms, {n_mark} x {a.marker}: {span / 1e6 / max(1, n_mark):.3f} ms per {a.marker}")
    print(f"kernel union {busy / 1e6:.2f} ms ({busy / span:.1%}), idle {(span - busy) / 1e6:.2f} ms, "
          f"mean concurrency while busy {conc:.2f}")
    print(f"copy union {cbusy / 1e6:.2f} ms ({cbusy / span:.1%}) over {len(cpw)} copies")
    by = Counter()
    for s, e, d, b in cpw:
        by[(d, b // (1 << 20))] += 1
    big = [c for c in cpw if c[3] >= 1 << 20]
    if big:
        rate = sum(c[3] for c in big) / max(1, sum(c[1] - c[0] for c in big))
        print(f"copies >= 1 MiB: {len(big)}, mean {sum(c[3] for c in big) / len(big) / 2**20:.1f} MiB, "
              f"{rate:.1f} GB/s while running, mean {sum(c[1] - c[0] for c in big) / len(big) / 1e3:.0f} us")
    hist = Counter()
    for g in gaps:
        hist[min(6, len(str(int(g // 1000))))] += g
    print("idle by gap length (us digits -> ms):",
          {f"<1e{k}us": round(v / 1e6, 3) for k, v in sorted(hist.items())})
    per = Counter()
    for s, e, n, *_ in win:
        per[n] += e - s
    print("kernel ms per", a.marker, {n: round(v / 1e6 / max(1, n_mark), 3) for n, v in per.most_common(14)})
    qs = Counter((q, st) for *_, q, st in win)
    print("queues/streams:", dict(qs.most_common(12)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
