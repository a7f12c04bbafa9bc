"""Per-kernel ms of bench logs (selected kernels): knock_show.py LOG..."""
import json
import sys

KS = ("k_huff1", "k_huff2", "k_huff3", "k_dcscan", "k_idct", "k_color", "k_hresize", "k_vert", "k_final")
for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = d["kernels_ms_per_step"]
            print(f"{f.split('/')[-1]:34s} {d['value']:9.1f} {d['ms_per_step']:7.3f} ser {d['serialized_ms_per_step']:7.3f}",
                  " ".join(f"{x[2:]}={k.get(x, 0):.3f}" for x in KS))
