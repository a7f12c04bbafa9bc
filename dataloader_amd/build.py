"""In-tree build of libdino_ingest.so (hipcc, gfx950).  Used by __graft_entry__.build()."""

from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OUT = PKG / "libdino_ingest.so"
SOURCES = [CSRC / "kernels.hip", CSRC / "capi.hip", CSRC / "feed.hip", CSRC / "tario.cpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-strict-aliasing",
         "-fno-gpu-flush-denormals-to-zero", "-Wall", "-Wno-unused-function", "-pthread"]


def needs_build() -> bool:
    if not OUT.exists():
        return True
    mt = OUT.stat().st_mtime
    deps = list(CSRC.glob("*")) + [PKG.parent / "include" / "dino_ingest.h"]
    return any(d.stat().st_mtime > mt for d in deps)


def build(force: bool = False, verbose: bool = True, out: Path = OUT, defines: tuple = ()) -> Path:
    if out == OUT and not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = out.with_suffix(".so.tmp")
    cmd = [hipcc, *FLAGS, *[f"-D{d}" for d in defines], "-o", str(tmp), *map(str, SOURCES)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out
