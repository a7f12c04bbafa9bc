#!/usr/bin/env python
"""Host-side copy bandwidth of the GPU box as the host half sees it (analysis aid, round 6):
the CPU quota this process gets (cgroup cpu.max, affinity), then dino_gather (the native
pack: 512 images of ~84 KB gathered into one buffer) with 1..32 copier threads, and N
concurrent gathers of 2 threads each (the 8-rank host study's shape: 8 feeds x 2 copiers).
No GPU work.  Prints one JSON line."""
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from dataloader_amd.tario import gather  # noqa: E402


def cpu_quota():
    out = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            out[p] = Path(p).read_text().strip()
        except OSError:
            pass
    return out


def main():
    rng = np.random.default_rng(0)
    n_img, img = 512, 84 * 1024
    # 4 distinct batches' worth of sources (more than the L3 of a CCD), as separate bytes objects
    srcs = [[rng.integers(0, 255, img, dtype=np.uint8).tobytes() for _ in range(n_img)] for _ in range(4)]
    batch_bytes = n_img * img

    def one_gather(dst, k, threads):
        gather(srcs[k % 4], dst, threads)

    res = {"quota": cpu_quota(), "batch_mb": round(batch_bytes / 1e6, 1), "single": {}, "concurrent": {}}
    dst = np.empty(batch_bytes + 4096, np.uint8)
    for threads in (1, 2, 4, 8, 16, 32):
        one_gather(dst, 0, threads)
        t0 = time.perf_counter()
        reps = 12
        for k in range(reps):
            one_gather(dst, k, threads)
        dt = time.perf_counter() - t0
        res["single"][threads] = round(reps * batch_bytes / dt / 1e9, 1)  # GB/s copied
    for feeds in (1, 2, 4, 8):
        dsts = [np.empty(batch_bytes + 4096, np.uint8) for _ in range(feeds)]
        reps = 8

        def run(f):
            for k in range(reps):
                one_gather(dsts[f], k + f, 2)

        ths = [threading.Thread(target=run, args=(f,)) for f in range(feeds)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        res["concurrent"][feeds] = round(feeds * reps * batch_bytes / dt / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
