"""Multi-scan JPEGs (tests/jpeg_writer.py) through the coefficient-buffer decode model
(progressive.hpp, the code k_prog runs) — bit-exact with Pillow / libjpeg-turbo, and the
host pre-screen's classification of the cases it leaves to Pillow.  CPU only."""

from __future__ import annotations

import numpy as np
import pytest

from dataloader_amd import fallback
from dataloader_amd.engine import pack_jpegs
from dataloader_amd.synthetic import textured_rgb
from oracle import cpu_ref
from tests import jpeg_writer as jw
from tests.helpers import emu_decode


def multiscan_cases(rng, sizes=((83, 61), (17, 9), (1, 1), (130, 97))):
    out = []
    for w, h in sizes:
        img = textured_rgb(w, h, rng)
        gray = img.mean(-1).astype(np.uint8)
        out += [
            (f"seq_per_comp_{w}x{h}", jw.encode(img, jw.sequential_per_component())),
            (f"seq_order_{w}x{h}", jw.encode(img, [jw.scan((2,)), jw.scan((0,)), jw.scan((1,))], samp=((2, 1), (1, 1), (1, 1)))),
            (f"seq_partial_il_{w}x{h}", jw.encode(img, [jw.scan((0,)), jw.scan((2, 1))], quality=60)),
            (f"seq_il_21_{w}x{h}", jw.encode(img, [jw.scan((0,)), jw.scan((2, 1))], samp=((1, 1), (1, 1), (1, 1)))),
            (f"seq_rst_{w}x{h}", jw.encode(img, jw.sequential_per_component(), restart=[2, 0, 5])),
            (f"prog_simple_rst_{w}x{h}", jw.encode(img, jw.simple_progression(), progressive=True, restart=3)),
            (f"prog_deep_{w}x{h}", jw.encode(img, jw.deep_progression(), progressive=True, quality=92)),
            (f"prog_deep_444_{w}x{h}", jw.encode(img, jw.deep_progression(), progressive=True, samp=((1, 1),) * 3)),
            (f"prog_deep_422_rst_{w}x{h}", jw.encode(img, jw.deep_progression(), progressive=True,
                                                     samp=((2, 1), (1, 1), (1, 1)),
                                                     restart=[1, 2, 3, 4, 0, 1, 7, 2, 2, 3, 1, 9, 1, 1, 4, 2])),
            (f"gray_seq_{w}x{h}", jw.encode(gray, [jw.scan((0,))], restart=1)),
            (f"gray_prog_{w}x{h}", jw.encode(gray, jw.simple_progression(1), progressive=True)),
            # a DQT between scans for a table already latched (allowed: libjpeg keeps the latched copy)
            (f"prog_dqt_latched_{w}x{h}", jw.encode(img, jw.simple_progression(), progressive=True,
                                                    before_scan={3: jw.dqt_segment(0, 30)})),
        ]
    return out


def test_multiscan_model_bit_exact(emu):
    rng = np.random.default_rng(8)
    for name, j in multiscan_cases(rng):
        ref = cpu_ref.decode_rgb(j)
        assert ref is not None, name
        r, out, st = emu_decode(emu, j, 0, 1)
        assert r == 0, (name, r)
        np.testing.assert_array_equal(out, np.asarray(ref), err_msg=name)


def test_prescreen_leaves_smoothed_and_relatched_files_to_pillow():
    rng = np.random.default_rng(9)
    img = textured_rgb(64, 48, rng)
    smoothed = jw.encode(img, jw.unrefined_progression(), progressive=True)
    # a DQT redefining the chroma table before the chroma components' first scan
    relatch = jw.encode(img, [jw.scan((0,), 0, 0, 0, 0), jw.scan((0,), 1, 63, 0, 0), jw.scan((1, 2), 0, 0, 0, 0),
                              jw.scan((1,), 1, 63, 0, 0), jw.scan((2,), 1, 63, 0, 0)], progressive=True,
                        before_scan={2: jw.dqt_segment(1, 20, chroma=True)})
    ok = jw.encode(img, jw.simple_progression(), progressive=True)
    buf, off = pack_jpegs([smoothed, relatch, ok], pin=False)
    info, _, _ = fallback.probe(buf.data_ptr(), off.numpy(), 3, 16384)
    assert list(info[:, 0]) == [1, 1, 0]
    assert cpu_ref.decode_rgb(smoothed) is not None and cpu_ref.decode_rgb(relatch) is not None


@pytest.mark.parametrize("cut", [0.3, 0.7, 0.97])
def test_truncated_multiscan_files(emu, cut):
    rng = np.random.default_rng(10)
    j = jw.encode(textured_rgb(70, 50, rng), jw.deep_progression(), progressive=True)
    t = j[: int(len(j) * cut)]
    assert cpu_ref.decode_rgb(t) is None          # no EOI: Pillow reports a truncated file
    assert emu_decode(emu, t, 0, 1)[0] == -2


def test_scan_component_order_rule(emu):
    """libjpeg-turbo get_sos: scan component k must be a frame component at index >= k, so
    (1, 0, 2) and (0, 2, 1) are errors (Pillow raises -> the reference zero-fills) while
    (2, 1) after a scan of 0 decodes."""
    rng = np.random.default_rng(12)
    img = textured_rgb(40, 24, rng)
    for comps, ok in (((1, 0, 2), False), ((0, 2, 1), False), ((0, 1, 2), True)):
        j = jw.encode(img, [jw.scan(comps)], samp=((1, 1),) * 3)
        ref = cpu_ref.decode_rgb(j)
        assert (ref is not None) == ok
        r, out, _ = emu_decode(emu, j, 0, 1)
        if ok:
            assert r == 0
            np.testing.assert_array_equal(out, np.asarray(ref))
        else:
            assert r < 0
