"""Print the headline + Huffman kernel split of bench logs: show_bench.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = d["kernels_ms_per_step"]
            hk = {x: k[x] for x in k if x.startswith("k_h") and k[x] > 0.02}
            print(f"{f.split('/')[-1]:28s} {d['value']:9.1f} img/s {d['ms_per_step']:7.3f} ms  ser {d['serialized_ms_per_step']:7.3f}",
                  hk)
