"""When each H2D batch copy was asked for (hipMemcpyAsync on the host) and when it ran, from
a rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace csv directory; plus
the idle time of the device before each copy's first dependent kernel.

usage: python scripts/copy_lag.py <dir> [--min-mib 1]"""
import argparse
import csv
import glob
import os
import sys


def _rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=20, help="copies to skip (warm-up)")
    a = ap.parse_args()
    api = {r["Correlation_Id"]: r for r in _rows(a.dir, "*hip_api_trace.csv")}
    cps = _rows(a.dir, "*memory_copy_trace.csv")
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                for r in _rows(a.dir, "*kernel_trace.csv"))
    cps = sorted(cps, key=lambda r: int(r["Start_Timestamp"]))
    big = [r for r in cps if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 200_000]
    print(f"{len(big)} batch copies (> 200 us); api records {len(api)}")
    prev_end = None
    lags, idles = [], []
    for r in big[a.skip:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c = api.get(r["Correlation_Id"])
        call = int(c["Start_Timestamp"]) if c else None
        # device idle right before the copy's end: no kernel running in (e - 50 us, e)?
        running = [k for k in ks if k[0] < e and k[1] > s]
        busy = 0
        cur = s
        for k in sorted(running):
            ks_, ke = max(k[0], cur), min(k[1], e)
            if ke > ks_:
                busy += ke - ks_
                cur = ke
        idle = (e - s) - busy
        lag = (s - call) / 1e3 if call else float("nan")
        lags.append(lag)
        idles.append(idle / 1e3)
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        print(f"call->start {lag:8.1f} us  dur {(e - s) / 1e3:6.1f}  since prev copy {gap:8.1f}  "
              f"device idle during copy {idle / 1e3:7.1f} us  {c['Function'] if c else ''}")
    if lags:
        print(f"mean call->start {sum(lags) / len(lags):.1f} us, mean idle during copies {sum(idles) / len(idles):.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
