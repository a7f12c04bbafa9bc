#!/usr/bin/env python
"""Build A/B variants of the library under build/ (analysis aid): each argument is
name=DEFINE[,DEFINE...]; 'name=' builds the default."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from dataloader_amd import build as b  # noqa: E402

(ROOT / "build").mkdir(exist_ok=True)
for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    b.build(force=True, out=ROOT / "build" / f"lib_{name}.so", defines=tuple(d for d in defs.split(",") if d))
