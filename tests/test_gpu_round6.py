"""Round-6 GPU parity: the lane decoder of progressive JPEGs (k_plscan + k_papply,
lscan.hpp) bit-exact with Pillow in batches of several 64-image groups, next to the wave
decoder's images (k_pscan) in the same batch.  Tolerances: bit-exact (decode)."""

from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from dataloader_amd import fallback
from dataloader_amd.engine import IngestEngine, pack_jpegs
from dataloader_amd.synthetic import encode_jpeg, textured_rgb
from oracle import cpu_ref
from tests import jpeg_writer as jw
from tests.test_lscan_cpu import _lane_cases

pytestmark = pytest.mark.gpu

LANE_FLAG_OFF = 776  # PHdr::lane (dino_debug_region 6)


def _wave_cases(rng):
    img = textured_rgb(48, 40, rng)
    five = jw.encode(img, [jw.scan((0, 1, 2), 0, 0, 0, 0), jw.scan((0,), 1, 63, 0, 5)] +
                     [jw.scan((0,), 1, 63, a + 1, a) for a in range(4, -1, -1)] +
                     [jw.scan((1,), 1, 63, 0, 0), jw.scan((2,), 1, 63, 0, 0)], progressive=True)
    return [encode_jpeg(textured_rgb(64, 48, rng), progressive=True, restart_mcus=2),
            jw.encode(img, jw.sequential_per_component()), five]


def _engine(dev, n: int, lane: bool) -> IngestEngine:
    """An engine whose progressive images take the lane decoder (DINO_PROG_LANE=1, read when
    the context is created) or the wave decoder."""
    old = os.environ.get("DINO_PROG_LANE")
    os.environ["DINO_PROG_LANE"] = "1" if lane else "0"
    try:
        return IngestEngine(dev, max_batch=n, max_views=1, max_crop_size=8)
    finally:
        if old is None:
            os.environ.pop("DINO_PROG_LANE")
        else:
            os.environ["DINO_PROG_LANE"] = old


def _decode(dev, jpegs, lane: bool):
    eng = _engine(dev, len(jpegs), lane)
    hb, off = pack_jpegs(jpegs, pin=True)
    info, ws, _ = fallback.probe(hb.data_ptr(), off.numpy(), len(jpegs), 0)
    assert (info[:, 0] == 0).all(), info[:, 0]
    eng.reserve(ws, 0)
    st = eng.decode(hb.to(dev), off.to(dev), len(jpegs)).cpu().numpy()
    torch.cuda.synchronize()
    flags = []  # PHdr::lane of each kind-1 image, -1 for the others
    for i in range(len(jpegs)):
        if info[i, 3] == 1:
            h = eng.debug_region(i, 6, 832).cpu().numpy()
            flags.append(int(h[LANE_FLAG_OFF:LANE_FLAG_OFF + 4].view(np.int32)[0]))
        else:
            flags.append(-1)
    rgb = [eng.copy_rgb(i, int(info[i, 1]), int(info[i, 2])).cpu().numpy() for i in range(len(jpegs))]
    eng.close()
    return st, flags, rgb


def test_lane_decoder_groups_bit_exact(gpu_device):
    """150 progressive files of every lane-eligible flavour (Pillow's script at three
    samplings and sizes 1x1 .. 1111x71, libjpeg-default and deep scripts with up to three AC
    refinement slots, split refinement bands, grayscale) in three 64-image groups, mixed
    with baseline files and the wave decoder's images (restart intervals, sequential
    multi-scan, five AC refinements): every image bit-exact with Pillow, the lane flag set
    exactly on the eligible ones; the same batch on the wave decoder alone gives the same
    pixels."""
    rng = np.random.default_rng(601)
    lane_src = [j for _, j in _lane_cases(rng)]
    wave_src = _wave_cases(rng)
    base = [encode_jpeg(textured_rgb(320, 240, rng)), encode_jpeg(textured_rgb(97, 203, rng))]
    jpegs, expect = [], []
    k = 0
    while len(jpegs) < 150:
        jpegs.append(lane_src[k % len(lane_src)])
        expect.append(1)
        if k % 17 == 5:
            jpegs.append(wave_src[(k // 17) % len(wave_src)])
            expect.append(0)
        if k % 23 == 7:
            jpegs.append(base[(k // 23) % len(base)])
            expect.append(-1)
        k += 1
    st, lane, rgb = _decode(gpu_device, jpegs, True)
    assert (st[:, 0] == 0).all(), st[:, 0]
    assert lane == expect, [(i, a, b) for i, (a, b) in enumerate(zip(lane, expect)) if a != b][:8]
    bad = []
    for i, j in enumerate(jpegs):
        ref = np.asarray(cpu_ref.decode_rgb(j))
        if not np.array_equal(rgb[i], ref):
            bad.append((i, expect[i], int((rgb[i] != ref).sum())))
    assert not bad, bad[:10]
    st0, lane0, rgb0 = _decode(gpu_device, jpegs, False)
    assert (st0[:, 0] == 0).all()
    assert all(v in (0, -1) for v in lane0)
    assert all(np.array_equal(a, b) for a, b in zip(rgb, rgb0))


@pytest.mark.parametrize("lane", [True, False], ids=["lane", "wave"])
def test_damaged_progressive_scans_both_decoders(gpu_device, lane):
    """Damaged entropy bytes inside progressive scans (bad codes, insufficient data, AC runs
    past the band into the next band's coefficients, which orders adjacent-band scans,
    progressive.hpp scan_write_end) on the lane and the wave decoder: Pillow's pixels, or
    zero-fill where Pillow raises."""
    rng = np.random.default_rng(602)
    jpegs = []
    for t in range(70):
        j = bytearray(encode_jpeg(textured_rgb(160 + t, 120, rng), quality=90, progressive=True))
        pos = int(len(j) * (0.15 + 0.8 * (t % 10) / 10))
        for k in range(pos, min(pos + 30 + t, len(j) - 4)):
            if j[k] != 0xFF and j[k - 1] != 0xFF:
                j[k] = (j[k] * 37 + 11 + t) & 0x7F
        jpegs.append(bytes(j))
    dev = gpu_device
    eng = _engine(dev, len(jpegs), lane)
    hb, off = pack_jpegs(jpegs, pin=True)
    info, ws, _ = fallback.probe(hb.data_ptr(), off.numpy(), len(jpegs), 0)
    eng.reserve(ws, 0)
    st = eng.decode(hb.to(dev), off.to(dev), len(jpegs)).cpu().numpy()
    bad = []
    for i, j in enumerate(jpegs):
        ref = cpu_ref.decode_rgb(j)
        if ref is None:
            if st[i, 0] == 0:
                bad.append((i, "decoded where Pillow raises"))
            continue
        if st[i, 0] != 0:
            bad.append((i, "status", int(st[i, 0])))
            continue
        got = eng.copy_rgb(i, int(st[i, 1]), int(st[i, 2])).cpu().numpy()
        if not np.array_equal(got, np.asarray(ref)):
            bad.append((i, int((got != np.asarray(ref)).sum())))
    eng.close()
    assert not bad, bad[:10]
