"""Reads a DINO_FEED_TRACE file (csrc/feed.hip) and splits the caller's waits in
dino_feed_next by what the packer was doing for that batch.

usage: python scripts/feed_trace.py <trace> [skip]"""
import sys


def main() -> int:
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    P, N = [], []
    for line in open(path):
        f = line.split()
        if f[0] == "P":
            P.append([float(x) for x in f[1:]])
        elif f[0] == "N":
            N.append([float(x) for x in f[1:]])
    P = P[skip:]
    blocking = [n for n in N if n[4] < 0][skip:]
    if not P or not blocking:
        print("empty trace")
        return 1
    k = len(P)
    ph = {"slot": 0.0, "samples": 0.0, "pack": 0.0, "relock": 0.0, "ready": 0.0, "between": 0.0}
    for i, r in enumerate(P):
        ph["slot"] += r[1] - r[0]
        ph["samples"] += r[2] - r[1]
        ph["pack"] += r[3] - r[2]
        ph["relock"] += r[4] - r[3]
        ph["ready"] += r[5] - r[4]
        if i:
            ph["between"] += r[0] - P[i - 1][5]
    span = P[-1][5] - P[0][0]
    print(f"packer: {k} batches, {span / k * 1e3:.3f} ms per batch; mean ms per batch:",
          {a: round(b / k * 1e3, 3) for a, b in ph.items()})
    w = [n[2] - n[0] for n in blocking]
    lw = [n[1] - n[0] for n in blocking]
    print(f"caller: {len(w)} blocking next() calls, mean wait {sum(w) / len(w) * 1e3:.3f} ms "
          f"(lock {sum(lw) / len(lw) * 1e3:.3f} ms), max {max(w) * 1e3:.2f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
