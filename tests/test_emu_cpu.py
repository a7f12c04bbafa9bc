"""CPU checks of the device algorithms, run through the host emulator.

tests/emu/emu.cpp compiles the same __host__ __device__ functions the HIP
kernels call (dataloader_amd/csrc/*.hpp) for the CPU and drives them with the
kernels' lane/phase structure (tests/emu/models.hpp).  Checked against Pillow
(decode, pixel ops, resize), the oracle (views) and the mask transcription.
"""

from __future__ import annotations

import ctypes
import io
import json
import random
from pathlib import Path

import numpy as np
import pytest
import torch
from PIL import Image

from dataloader_amd.params import VIEW_PARAMS_DTYPE, DinoAugConfig
from dataloader_amd.synthetic import encode_jpeg, textured_rgb
from oracle import cpu_ref
from oracle.masking_ref import RefMaskingGenerator
from tests.helpers import dc_extremes_rgb, P, emu_augment, emu_decode, emu_resized_crop, params_to_record, record_to_params

GOLD = Path(__file__).resolve().parent / "golden"
ONE_LEVEL = 1.0 / 255.0 / min(cpu_ref.IMAGENET_STD)


@pytest.fixture(scope="module")
def allrgb():
    idx = np.arange(1 << 24, dtype=np.uint32)
    a = np.stack([(idx >> 16) & 255, (idx >> 8) & 255, idx & 255], -1).astype(np.uint8)
    return a.reshape(4096, 4096, 3)


def test_rgb_hsv_l_exhaustive(emu, allrgb):
    """All 2^24 colours: RGB->HSV, HSV->RGB, RGB->L bit-exact with Pillow's Convert.c."""
    im = Image.fromarray(allrgb, "RGB")
    out = np.zeros((1 << 24) * 3, np.uint8)
    emu.emu_rgb_to_hsv_all(out.ctypes.data_as(P))
    np.testing.assert_array_equal(out.reshape(-1, 3), np.asarray(im.convert("HSV")).reshape(-1, 3))
    emu.emu_hsv_to_rgb_all(out.ctypes.data_as(P))
    np.testing.assert_array_equal(out.reshape(-1, 3),
                                  np.asarray(Image.fromarray(allrgb, "HSV").convert("RGB")).reshape(-1, 3))
    lo = np.zeros(1 << 24, np.uint8)
    emu.emu_rgb_to_l_all(lo.ctypes.data_as(P))
    np.testing.assert_array_equal(lo, np.asarray(im.convert("L")).reshape(-1))


def test_blend_matches_pillow(emu):
    a = np.repeat(np.arange(256, dtype=np.uint8), 256).reshape(256, 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256).reshape(256, 256)
    A = Image.fromarray(np.stack([a] * 3, -1))
    Bi = Image.fromarray(np.stack([b] * 3, -1))
    rng = np.random.default_rng(0)
    alphas = list(np.float32(rng.uniform(0.2, 1.8, 40))) + [np.float32(x) for x in (0.0, 0.5, 1.0, 1.8, 0.2)]
    for al in alphas:
        o = np.zeros(65536, np.uint8)
        emu.emu_blend_table(ctypes.c_float(al), o.ctypes.data_as(P))
        np.testing.assert_array_equal(o.reshape(256, 256), np.asarray(Image.blend(A, Bi, float(al)))[..., 0])


def test_normalize_and_casts(emu):
    px = np.arange(256, dtype=np.uint8)
    for m, s in zip(cpu_ref.IMAGENET_MEAN, cpu_ref.IMAGENET_STD):
        bf = np.zeros(256, np.uint16)
        f32 = np.zeros(256, np.float32)
        emu.emu_normalize(px.ctypes.data_as(P), 256, ctypes.c_float(m), ctypes.c_float(s), bf.ctypes.data_as(P),
                          f32.ctypes.data_as(P))
        ref = (torch.from_numpy(px).float().div(255) - torch.tensor(m, dtype=torch.float32)) / torch.tensor(
            s, dtype=torch.float32)
        np.testing.assert_array_equal(f32, ref.numpy())
        np.testing.assert_array_equal(bf, ref.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16))
    x = (torch.randn(10000) * 4).to(torch.bfloat16).float().numpy()
    o = np.zeros(x.size, np.uint8)
    emu.emu_fp8(x.ctypes.data_as(P), x.size, o.ctypes.data_as(P))
    np.testing.assert_array_equal(o, torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy())


def _zoo():
    rng = np.random.default_rng(7)
    out = []
    for (w, h) in [(64, 64), (225, 333), (17, 9), (8, 8), (1, 1), (640, 480), (33, 17)]:
        for sub in (0, 1, 2):
            out.append(encode_jpeg(textured_rgb(w, h, rng), quality=85, subsampling=sub))
    out.append(encode_jpeg(textured_rgb(200, 150, rng), gray=True))
    out.append(encode_jpeg(textured_rgb(320, 240, rng), restart_mcus=7))
    out.append(encode_jpeg(textured_rgb(99, 77, rng), quality=30))
    out.append(encode_jpeg(textured_rgb(99, 77, rng), quality=100))
    for sub, q in ((0, 95), (2, 95), (2, 50)):
        out.append(encode_jpeg(dc_extremes_rgb(160, 96, rng), quality=q, subsampling=sub))
    return out


@pytest.mark.parametrize("mode,lanes", [(0, 1), (1, 3), (1, 64), (1, 256), (2, 7), (2, 512), (3, 100), (3, 1024)])
def test_decode_bit_exact_vs_pillow(emu, mode, lanes):
    for j in _zoo():
        r, out, _ = emu_decode(emu, j, mode, lanes)
        assert r == 0
        np.testing.assert_array_equal(out, np.asarray(cpu_ref.decode_rgb(j)))


def test_decode_golden(emu):
    meta = json.loads((GOLD / "meta.json").read_text())
    for name in meta["jpegs"]:
        r, out, _ = emu_decode(emu, (GOLD / f"{name}.jpg").read_bytes(), 1, 16)
        assert r == 0, name
        np.testing.assert_array_equal(out, np.load(GOLD / f"{name}.rgb.npy"), err_msg=name)


def _damaged_streams(rng):
    """Valid entropy data cut mid-scan with the EOI kept (libjpeg: insufficient_data ->
    the MCU finishes from zero bits, later MCUs of the segment stay zero) and restart
    markers renumbered / dropped / duplicated (jpeg_resync_to_restart): Pillow decodes
    all of them (with warnings)."""
    out = []
    for sub in (0, 1, 2):
        for rst_mcus in (0, 5):
            base = encode_jpeg(textured_rgb(160, 120, rng), quality=85, subsampling=sub, restart_mcus=rst_mcus)
            sos = base.index(b"\xff\xda")
            s0 = sos + 2 + int.from_bytes(base[sos + 2:sos + 4], "big")
            for frac in (0.03, 0.3, 0.61, 0.97):
                cut = s0 + int((len(base) - 2 - s0) * frac)
                cut -= base[cut - 1] == 0xFF
                out.append((f"cut{sub}{rst_mcus}_{frac}", base[:cut] + b"\xff\xd9"))
    base = encode_jpeg(textured_rgb(200, 136, rng), quality=80, subsampling=2, restart_mcus=3)
    rst = [i for i in range(len(base) - 1) if base[i] == 0xFF and 0xD0 <= base[i + 1] <= 0xD7]
    for k in (0, len(rst) // 2, len(rst) - 1):
        for nv in (1, 2, 7):
            b = bytearray(base)
            b[rst[k] + 1] = 0xD0 + ((b[rst[k] + 1] - 0xD0 + nv) & 7)
            out.append((f"renum{k}_{nv}", bytes(b)))
        b = bytearray(base)
        del b[rst[k]:rst[k] + 2]
        out.append((f"drop{k}", bytes(b)))
        b = bytearray(base)
        b[rst[k]:rst[k]] = bytes([0xFF, 0xD0 + (k & 7)])
        out.append((f"dup{k}", bytes(b)))
    return out


@pytest.mark.parametrize("mode,lanes", [(0, 1), (1, 64), (1, 300), (3, 1000)])
def test_damaged_streams_bit_exact_vs_pillow(emu, mode, lanes):
    for name, j in _damaged_streams(np.random.default_rng(1)):
        ref = cpu_ref.decode_rgb(j)
        assert ref is not None, name
        r, out, _ = emu_decode(emu, j, mode, lanes)
        assert r == 0, (name, r)
        np.testing.assert_array_equal(out, np.asarray(ref), err_msg=name)


def test_corrupt_bytes_all_decode_modes_vs_pillow(emu):
    """Bytes overwritten inside the scan: the speculative decode modes agree with the
    sequential one and with Pillow, including blocks whose dequantised coefficients
    leave the range where libjpeg-turbo's SIMD and C IDCTs agree (idct.hpp)."""
    from dataloader_amd.synthetic import make_jpeg
    rng = np.random.default_rng(5)
    base = make_jpeg(320, 240, 3)
    sos = base.index(b"\xff\xda")
    for k in range(6):
        b = bytearray(base)
        for _ in range(4):
            p = int(rng.integers(sos + 20, len(b) - 4))
            v = int(rng.integers(0, 255))
            if b[p - 1] != 0xFF and v != 0xFF:
                b[p] = v
        j = bytes(b)
        ref = cpu_ref.decode_rgb(j)
        outs = [emu_decode(emu, j, m, lanes) for m, lanes in ((0, 1), (1, 200), (1, 77), (3, 513))]
        for r, out, _ in outs:
            assert r == outs[0][0]
            np.testing.assert_array_equal(out, outs[0][1])
        if ref is not None:
            assert outs[0][0] == 0
            np.testing.assert_array_equal(outs[0][1], np.asarray(ref))


def test_speculative_sync_converges(emu):
    from dataloader_amd.synthetic import make_jpeg
    j = make_jpeg(640, 480, 11)
    r, out, st = emu_decode(emu, j, 1, 256)
    assert r == 0 and st[0] <= 8, f"sync rounds {st[0]}"


def test_corrupt_and_unsupported(emu):
    info = np.zeros(8, np.int32)
    for data, expect in [(b"not a jpeg", -1), (b"\xff\xd8\xff\xd9", -1), (b"", -1)]:
        buf = np.frombuffer(data + b"\0", np.uint8)
        assert emu.emu_parse(buf.ctypes.data_as(P), ctypes.c_int64(len(data)), info.ctypes.data_as(P)) == expect
    good = encode_jpeg(textured_rgb(200, 150, np.random.default_rng(0)))
    r, _, _ = emu_decode(emu, good[: len(good) * 4 // 5], 0, 1)  # truncated, no EOI: Pillow raises
    assert r == -2
    assert cpu_ref.decode_rgb(good[: len(good) * 4 // 5]) is None


def test_resized_crop_bit_exact(emu):
    rng = np.random.default_rng(1)
    gen = torch.Generator().manual_seed(1)
    rnd = random.Random(1)
    cfg = cpu_ref.AugCfg()
    for _ in range(25):
        W, H = int(rng.integers(20, 500)), int(rng.integers(20, 500))
        rgb = textured_rgb(W, H, rng)
        img = Image.fromarray(rgb)
        for spec in cpu_ref.view_table(cfg):
            p = cpu_ref.draw_params_like_cpubackend(W, H, spec, cfg, gen, rnd)
            ref = cpu_ref.resized_crop(img, p.crop_top, p.crop_left, p.crop_h, p.crop_w, p.out_size)
            if p.flip:
                ref = ref.transpose(Image.FLIP_LEFT_RIGHT)
            np.testing.assert_array_equal(emu_resized_crop(emu, rgb, params_to_record(p)), np.asarray(ref))


def test_augment_views_vs_oracle(emu):
    """Full view chain: bit-exact except gaussian blur (<= 1 uint8 level on <= 0.5 % of pixels)."""
    rng = np.random.default_rng(2)
    gen = torch.Generator().manual_seed(2)
    rnd = random.Random(2)
    cfg = cpu_ref.AugCfg()
    for _ in range(10):
        W, H = int(rng.integers(60, 400)), int(rng.integers(60, 400))
        rgb = textured_rgb(W, H, rng)
        img = Image.fromarray(rgb)
        for spec in cpu_ref.view_table(cfg):
            p = cpu_ref.draw_params_like_cpubackend(W, H, spec, cfg, gen, rnd)
            ref = cpu_ref.augment_one(b"", p, decoded=img, out_dtype=torch.float32)
            got = emu_augment(emu, rgb, params_to_record(p), cfg.mean, cfg.std, 1)
            d = (ref - got).abs()
            if p.blur:
                assert d.max() <= ONE_LEVEL + 1e-5 and (d > 0).float().mean() <= 0.005
            else:
                assert torch.equal(ref, got)


def test_masks_bit_exact_vs_transcription(emu):
    for grid, seed, n in [(14, 0, 5), (16, 1, 5), (37, 42, 3), (8, 5, 10)]:
        ref = RefMaskingGenerator(grid, py_rng=random.Random(seed), np_rng=np.random.RandomState(seed))
        py = np.asarray(random.Random(seed).getstate()[1], np.uint32)
        ks = np.random.RandomState(seed).get_state()
        npst = np.concatenate([np.asarray(ks[1], np.uint32), np.asarray([ks[2]], np.uint32)])
        out = np.zeros((n, grid * grid), np.uint8)
        emu.emu_masks(grid, grid, grid * grid // 2, 4, grid * grid // 2, ctypes.c_double(ref.log_aspect_ratio[0]),
                      ctypes.c_double(ref.log_aspect_ratio[1]), n, py.ctypes.data_as(P), npst.ctypes.data_as(P),
                      out.ctypes.data_as(P))
        for k in range(n):
            np.testing.assert_array_equal(out[k].astype(bool), ref(flat=True))


def test_sampler_records_valid(emu):
    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.params import make_aug_config
    cfg = make_aug_config(DINOAugConfig(), 224, 96, 0)
    out = np.zeros(10, VIEW_PARAMS_DTYPE)
    flips = jit = 0
    for s in range(300):
        W, H = 40 + (s * 37) % 900, 30 + (s * 53) % 700
        emu.emu_sample_params(ctypes.byref(cfg), ctypes.c_uint64(99), ctypes.c_uint64(s // 7), s, W, H, 1,
                              out.ctypes.data_as(P))
        for v, r in enumerate(out):
            p = record_to_params(r)
            assert p.out_size == (224 if v < 2 else 96)
            assert 0 <= p.crop_top and p.crop_top + p.crop_h <= H and 0 <= p.crop_left and p.crop_left + p.crop_w <= W
            assert sorted(p.order) == [0, 1, 2, 3] and p.ksize in (3, 5, 7, 9)
            if v == 0:
                assert p.blur            # blur_prob_global1 = 1.0
            if v != 1:
                assert not p.solarize    # solarize only on view 1
            flips += p.flip
            jit += p.jitter
    assert 0.4 < flips / 3000 < 0.6 and 0.72 < jit / 3000 < 0.88


def test_view_params_layout_matches_c():
    assert VIEW_PARAMS_DTYPE.itemsize == 80
    assert VIEW_PARAMS_DTYPE.fields["sigma"][1] == 48 and VIEW_PARAMS_DTYPE.fields["order"][1] == 28
    assert ctypes.sizeof(DinoAugConfig) == 4 * 29  # dino_aug_config: 29 x 32-bit fields


def test_progressive_bit_exact_vs_pillow(emu):
    """Progressive JPEGs (libjpeg's simple progression: DC first/refine, spectral bands,
    successive approximation) through the k_prog model: bit-exact vs Pillow, with and
    without restart intervals, every chroma sampling, gray, edge sizes."""
    rng = np.random.default_rng(4)
    n = 0
    for w, h in [(1, 1), (8, 8), (17, 9), (64, 64), (225, 333), (640, 480), (1111, 71)]:
        for sub in (0, 1, 2):
            for q, rst in ((50, 0), (85, 3), (95, 0)):
                j = encode_jpeg(textured_rgb(w, h, rng), quality=q, subsampling=sub, progressive=True,
                                restart_mcus=rst)
                b = np.frombuffer(j, np.uint8)
                info = np.zeros(8, np.int32)
                assert emu.emu_parse(b.ctypes.data_as(P), ctypes.c_int64(len(j)), info.ctypes.data_as(P)) == 0
                r, out, st = emu_decode(emu, j, 0, 1)
                assert r == 0 and st[0] >= 2, (w, h, sub, q, rst)
                np.testing.assert_array_equal(out, np.asarray(cpu_ref.decode_rgb(j)), err_msg=f"{w}x{h} s{sub} q{q}")
                n += 1
    j = encode_jpeg(textured_rgb(300, 200, rng), progressive=True, gray=True)
    r, out, _ = emu_decode(emu, j, 0, 1)
    assert r == 0
    np.testing.assert_array_equal(out, np.asarray(cpu_ref.decode_rgb(j)))
    # truncated progressive file (no EOI): Pillow raises, the walk reports TRUNCATED
    cut = j[: len(j) * 2 // 3]
    assert cpu_ref.decode_rgb(cut) is None
    assert emu_decode(emu, cut, 0, 1)[0] == -2
