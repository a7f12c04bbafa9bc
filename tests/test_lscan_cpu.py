"""The lane progressive decoder (lscan.hpp: lane_plan, lane_scan_decode with deferred
refinements, lane_apply_block) through the host emulator, bit-exact with Pillow, and its
eligibility rule (which images stay on the wave decoder).  CPU only."""

from __future__ import annotations

import numpy as np
import pytest

from dataloader_amd.synthetic import encode_jpeg, textured_rgb
from oracle import cpu_ref
from tests import jpeg_writer as jw
from tests.helpers import emu_decode

LANE = 4  # emu_decode mode: kind-1 images through the lane model (1 = left to the wave decoder)


def _lane_cases(rng):
    out = []
    for w, h in [(1, 1), (17, 9), (64, 64), (225, 333), (640, 480), (1111, 71)]:
        for sub in (0, 1, 2):
            out.append((f"pillow_prog_{w}x{h}_s{sub}",
                        encode_jpeg(textured_rgb(w, h, rng), quality=85, subsampling=sub, progressive=True)))
    out.append(("pillow_prog_gray", encode_jpeg(textured_rgb(300, 200, rng), progressive=True, gray=True)))
    out.append(("pillow_prog_q40", encode_jpeg(textured_rgb(300, 200, rng), progressive=True, quality=40)))
    out.append(("pillow_prog_q97", encode_jpeg(textured_rgb(213, 157, rng), progressive=True, quality=97)))
    for w, h in [(83, 61), (130, 97), (17, 9)]:
        img = textured_rgb(w, h, rng)
        out += [
            (f"jw_simple_{w}x{h}", jw.encode(img, jw.simple_progression(), progressive=True)),
            # four approximation levels of Y (3 AC refinement slots), DC refinements per component
            (f"jw_deep_{w}x{h}", jw.encode(img, jw.deep_progression(), progressive=True, quality=92)),
            (f"jw_deep_444_{w}x{h}", jw.encode(img, jw.deep_progression(), progressive=True, samp=((1, 1),) * 3)),
            (f"jw_gray_{w}x{h}", jw.encode(img.mean(-1).astype(np.uint8), jw.simple_progression(1), progressive=True)),
            # refinements of two bands of one component at the same level (shared mask words)
            (f"jw_split_bands_{w}x{h}", jw.encode(img, [
                jw.scan((0, 1, 2), 0, 0, 0, 0), jw.scan((0,), 1, 9, 0, 1), jw.scan((0,), 10, 63, 0, 1),
                jw.scan((1,), 1, 63, 0, 0), jw.scan((2,), 1, 63, 0, 0),
                jw.scan((0,), 10, 63, 1, 0), jw.scan((0,), 1, 9, 1, 0)], progressive=True)),
        ]
    return out


def test_lane_model_bit_exact(emu):
    rng = np.random.default_rng(61)
    for name, j in _lane_cases(rng):
        ref = cpu_ref.decode_rgb(j)
        assert ref is not None, name
        r, out, _ = emu_decode(emu, j, LANE, 1)
        assert r == 0, (name, r)
        np.testing.assert_array_equal(out, np.asarray(ref), err_msg=name)


@pytest.mark.parametrize("cut", [0.2, 0.55, 0.8])
def test_lane_model_damaged_scans(emu, cut):
    """Entropy bytes overwritten inside a scan (insufficient data, bad codes, runs past the
    band): the lane model keeps Pillow's output."""
    rng = np.random.default_rng(62)
    j = bytearray(encode_jpeg(textured_rgb(160, 120, rng), quality=90, progressive=True))
    pos = int(len(j) * cut)
    for k in range(pos, min(pos + 40, len(j) - 4)):
        if j[k] != 0xFF and j[k - 1] != 0xFF:
            j[k] = (j[k] * 37 + 11) & 0x7F
    j = bytes(j)
    ref = cpu_ref.decode_rgb(j)
    r, out, _ = emu_decode(emu, j, LANE, 1)
    if ref is None:
        assert r != 0
    else:
        assert r == 0
        np.testing.assert_array_equal(out, np.asarray(ref))


def test_lane_plan_leaves_irregular_images_to_the_wave_decoder(emu):
    rng = np.random.default_rng(63)
    img = textured_rgb(48, 40, rng)
    rst = encode_jpeg(textured_rgb(64, 48, rng), progressive=True, restart_mcus=2)
    seq = jw.encode(img, jw.sequential_per_component())
    five_refines = jw.encode(img, [jw.scan((0, 1, 2), 0, 0, 0, 0), jw.scan((0,), 1, 63, 0, 5)] +
                             [jw.scan((0,), 1, 63, a + 1, a) for a in range(4, -1, -1)] +
                             [jw.scan((1,), 1, 63, 0, 0), jw.scan((2,), 1, 63, 0, 0)], progressive=True)
    for name, j in (("restart", rst), ("sequential", seq), ("five_ac_refines", five_refines)):
        assert cpu_ref.decode_rgb(j) is not None, name
        assert emu_decode(emu, j, LANE, 1)[0] == 1, name  # not taken: the wave decoder's images
        r, out, _ = emu_decode(emu, j, 0, 1)              # ... which decodes them
        assert r == 0, name
        np.testing.assert_array_equal(out, np.asarray(cpu_ref.decode_rgb(j)), err_msg=name)
