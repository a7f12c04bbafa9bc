"""IDCT parity for out-of-range coefficients (damaged streams), CPU only.

Valid 8-bit JPEG data stays where libjpeg-turbo's C islow IDCT and its SIMD version
agree.  Damaged data can produce dequantised coefficients beyond 16 bits and
outputs beyond the range-limit table, where the x86 SIMD code Pillow runs wraps the
dequantisation, saturates pass 1 to int16 and clamps the output, while the C code
does not; idct.hpp restates the SIMD arithmetic, which k_idct runs for every block.  The test writer codes chosen coefficients (AC
categories up to 15, DC-only blocks with huge DC, random quant tables) and the
decode model must equal Pillow on every pixel; the same files run through the GPU
in tests/test_gpu_round2.py.
"""

from __future__ import annotations

import numpy as np
import pytest

from oracle import cpu_ref
from tests import jpeg_writer as jw
from tests.helpers import emu_decode

KINDS = ("small", "big", "dconly", "rowonly", "dense", "edge", "mix")


def extreme_coef_jpeg(rng, kind: str, nbw: int = 8, nbh: int = 8, color: bool = False) -> bytes:
    def block(k):
        b = np.zeros(64, np.int64)
        if k == "small":
            b[:] = rng.integers(-40, 41, 64) * (rng.random(64) < 0.3)
        elif k == "big":
            m = rng.random(64) < 0.1
            b[m] = rng.integers(-32767, 32768, int(m.sum()))
        elif k == "dconly":
            b[:8] = rng.integers(-3000, 3001, 8) * (rng.random(8) < 0.5)
        elif k == "rowonly":  # rows 1..7 zero: the SIMD DC-only shortcut with a large row 0
            b[:8] = rng.integers(-32767, 32768, 8)
        elif k == "dense":
            b[:] = rng.integers(-2000, 2001, 64)
        else:  # around the agreement bounds
            b[:] = rng.integers(-300, 301, 64) * (rng.random(64) < 0.5)
        b[0] = rng.integers(-16383, 16384)  # DC differences stay within category 15
        return b

    def hook(coefs, qts):
        out = []
        for c in coefs:
            bh, bw = c.shape[:2]
            n = np.zeros_like(c)
            for by in range(bh):
                for bx in range(bw):
                    n[by, bx] = block(kind if kind != "mix" else KINDS[int(rng.integers(0, 6))])
            out.append(n)
        return out, [rng.integers(1, 256, 64) for _ in qts]

    if color:
        img = np.zeros((nbh * 8, nbw * 8, 3), np.uint8)
        return jw.encode(img, [jw.scan((0, 1, 2))], samp=((1, 1), (1, 1), (1, 1)), coef_hook=hook)
    img = np.zeros((nbh * 8, nbw * 8), np.uint8)
    return jw.encode(img, [jw.scan((0,))], coef_hook=hook)


def extreme_cases(seed: int, n: int):
    rng = np.random.default_rng(seed)
    return [extreme_coef_jpeg(rng, KINDS[i % len(KINDS)], color=(i % 3 == 2)) for i in range(n)]


@pytest.mark.parametrize("mode,lanes", [(0, 1), (1, 16)])
def test_extreme_coefficients_match_pillow(emu, mode, lanes):
    for i, j in enumerate(extreme_cases(11, 28)):
        ref = cpu_ref.decode_rgb(j)
        assert ref is not None, i
        r, out, _ = emu_decode(emu, j, mode, lanes)
        assert r == 0
        np.testing.assert_array_equal(out, np.asarray(ref), err_msg=f"case {i} ({KINDS[i % len(KINDS)]})")
