#!/usr/bin/env python
"""cProfile of one host-fed bench leg in this process (bench imported as a module so that
its encoder pool can pickle its functions).  usage: prof_leg.py OUT.prof LEG [bench args]"""
import cProfile
import pstats
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402

if __name__ == "__main__":  # the encoder pool spawns workers that import this file
    out, leg = sys.argv[1], sys.argv[2]
    prof = cProfile.Profile()
    prof.enable()
    rc = bench.main(["--only-leg", leg] + sys.argv[3:])
    prof.disable()
    prof.dump_stats(out)
    st = pstats.Stats(out, stream=sys.stderr)
    st.sort_stats("tottime").print_stats(40)
    sys.exit(rc)
