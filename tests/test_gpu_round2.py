"""Round-2 GPU parity: the configs and edge semantics VERDICT r1 found untested.

* committed golden fixtures decoded / augmented through the C ABI (r1 set + the
  round-2 odd/large/progressive files + full-config 224/96 view records);
* progressive and raw-RGB inputs (k_prog, k_color's copy path) bit-exact;
* workspace capacity: greedy placement instead of cascading zero-fill, per-image
  DINO_IMG_NO_SPACE, and the product path (probe + reserve) rendering everything;
* host hand-over of the flavours the GPU does not decode (CMYK, arithmetic), and
  LeJEPA's black canvas for undecodable images (reference cpu.py:446-448);
* C3-shaped batches (short side 224-1600, 2 x 224 + 8 x 96, masks) and the C1 tar
  shard (256 x 256^2, B = 32) through the real feed, against the oracle;
* the reference's pinned CPUBackend assertions (tests/test_cpu_backend.py:146-223),
  device masks on non-square grids, iterator reset with batches in flight.
Tolerances: as tests/test_gpu_parity.py (bit-exact, blur <= 1 uint8 level on <= 0.5 %).
"""

from __future__ import annotations

import hashlib
import io
import json
import random
from pathlib import Path

import numpy as np
import pytest
import torch
from PIL import Image

from dataloader_amd.config import DINOAugConfig
from dataloader_amd.engine import IngestEngine, pack_jpegs, params_from_device, params_to_device
from dataloader_amd.params import OUT_BF16, OUT_FP32, VIEW_PARAMS_DTYPE, make_aug_config
from dataloader_amd.synthetic import encode_jpeg, make_jpeg, textured_rgb
from oracle import cpu_ref
from oracle.masking_ref import RefMaskingGenerator
from tests.helpers import record_to_params
from tests.test_gpu_parity import ONE_LEVEL, _check_views, _to_dev

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLD / "meta.json").read_text())


def _check_golden_views(jpegs, recs, views_npz, nv, sizes, got_views):
    k = 0
    for b in range(len(jpegs)):
        for v in range(nv):
            p = record_to_params(recs[b * nv + v])
            ref = torch.from_numpy(views_npz[f"arr_{k}"].copy()).view(torch.bfloat16).reshape(3, sizes[v], sizes[v])
            got = got_views[v][b].cpu()
            diff = (ref.float() - got.float()).abs()
            if p.blur:
                assert diff.max().item() <= ONE_LEVEL + 0.0161, (b, v)
                assert (diff > 0).float().mean().item() <= 0.005, (b, v)
            else:
                assert torch.equal(ref, got), (b, v, int((diff > 0).sum()))
            k += 1


def test_golden_fixtures_through_the_abi(gpu_device):
    names = META["jpegs"]
    r2 = META["jpegs_r2"]
    jpegs = [(GOLD / f"{n}.jpg").read_bytes() for n in names] + [(GOLD / f"{n}.jpg").read_bytes() for n in r2]
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    assert (info[:, 0] == 0).all(), info
    for i, n in enumerate(names):
        ref = np.load(GOLD / f"{n}.rgb.npy")
        got = eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy()
        np.testing.assert_array_equal(got, ref, err_msg=n)
    for i, (n, m) in enumerate(r2.items(), start=len(names)):
        got = eng.copy_rgb(i, m["width"], m["height"]).cpu().numpy()
        assert hashlib.sha256(got.tobytes()).hexdigest() == m["rgb_sha256"], n
    eng.close()
    # r1 records at the reference's small_aug_cfg (32 / 16, 2 + 2 views)
    cfg = DINOAugConfig(global_crop_size=32, local_crop_size=16, n_local_crops=2)
    recs = np.load(GOLD / "views.params.npy")
    eng = IngestEngine(gpu_device, max_batch=len(names), max_views=4, max_crop_size=32)
    d_bytes, d_off = _to_dev(jpegs[:len(names)], gpu_device)
    eng.decode(d_bytes, d_off, len(names))
    views = eng.augment(make_aug_config(cfg, 32, 16, OUT_BF16),
                        params_to_device(np.asarray(recs, VIEW_PARAMS_DTYPE), gpu_device))
    torch.cuda.synchronize()
    _check_golden_views(names, recs, np.load(GOLD / "views.bf16.npz"), 4, META["view_sizes"], views)
    eng.close()
    # round-2 records at the full DINOAugConfig (2 x 224 + 8 x 96)
    g = META["views224"]
    recs = np.load(GOLD / "views224.params.npy")
    sel = [(GOLD / f"{n}.jpg").read_bytes() for n in g["jpegs"]]
    eng = IngestEngine(gpu_device, max_batch=len(sel), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(sel, gpu_device)
    eng.decode(d_bytes, d_off, len(sel))
    views = eng.augment(make_aug_config(DINOAugConfig(), 224, 96, OUT_BF16), params_to_device(recs, gpu_device))
    torch.cuda.synchronize()
    _check_golden_views(sel, recs, np.load(GOLD / "views224.bf16.npz"), 10, g["view_sizes"], views)
    eng.close()


def _prog_zoo(rng):
    out = []
    for w, h in [(1, 1), (17, 9), (64, 64), (225, 333), (640, 480), (1111, 71), (1601, 1203)]:
        for sub in (0, 1, 2):
            out.append(encode_jpeg(textured_rgb(w, h, rng), quality=85, subsampling=sub, progressive=True))
    out.append(encode_jpeg(textured_rgb(640, 480, rng), progressive=True, restart_mcus=3))
    out.append(encode_jpeg(textured_rgb(333, 250, rng), progressive=True, restart_mcus=1, quality=95))
    out.append(encode_jpeg(textured_rgb(300, 200, rng), progressive=True, gray=True))
    out.append(encode_jpeg(textured_rgb(300, 200, rng), progressive=True, quality=40))
    return out


def test_progressive_and_raw_decode_bit_exact(gpu_device):
    """Progressive files (k_prog) mixed with baseline files and pre-decoded RGB containers
    in one batch: every image bit-exact with Pillow (raw: with its own pixels)."""
    from dataloader_amd.fallback import raw_container
    rng = np.random.default_rng(31)
    prog = _prog_zoo(rng)
    base = [encode_jpeg(textured_rgb(320, 240, rng)), encode_jpeg(textured_rgb(1024, 768, rng))]
    raws = [textured_rgb(37, 21, rng), textured_rgb(640, 480, rng)]
    jpegs = base[:1] + prog[:6] + [raw_container(raws[0])] + prog[6:] + base[1:] + [raw_container(raws[1])]
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    # unmarked, the containers are what Pillow sees: not a JPEG -> corrupt (no in-band magic)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    is_raw = np.array([j[:4] == b"DRGB" for j in jpegs])
    assert (info[is_raw, 0] == -1).all() and (info[~is_raw, 0] == 0).all(), info
    assert all(cpu_ref.decode_rgb(j) is None for j in np.array(jpegs, dtype=object)[is_raw])
    raw_mask = torch.from_numpy(is_raw.astype(np.uint8)).to(gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs), raw_mask=raw_mask).cpu().numpy()
    assert (info[:, 0] == 0).all(), info
    bad = []
    for i, j in enumerate(jpegs):
        if j[:4] == b"DRGB":
            ref = raws[0] if raws[0].nbytes + 16 == len(j) else raws[1]
        else:
            ref = np.asarray(cpu_ref.decode_rgb(j))
        got = eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy()
        if not np.array_equal(got, ref):
            bad.append((i, int((got != ref).sum())))
    eng.close()
    assert not bad, bad


def test_damaged_streams_through_the_abi(gpu_device):
    """Entropy data cut mid-scan with EOI kept (insufficient_data zero fill) and restart
    markers renumbered / dropped / duplicated (resync on the k_prog path) in one batch with
    clean images, bit-exact with Pillow, which decodes them all."""
    from tests.test_emu_cpu import _damaged_streams
    rng = np.random.default_rng(41)
    cases = _damaged_streams(rng) + [("clean", encode_jpeg(textured_rgb(640, 480, rng)))]
    jpegs = [j for _, j in cases]
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    bad = []
    for i, (name, j) in enumerate(cases):
        ref = np.asarray(cpu_ref.decode_rgb(j))
        if info[i, 0] != 0:
            bad.append((name, "status", int(info[i, 0])))
            continue
        got = eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy()
        if not np.array_equal(got, ref):
            bad.append((name, int((got != ref).sum())))
    eng.close()
    assert not bad, bad


def test_extreme_coefficients_through_k_idct(gpu_device):
    """Blocks whose coefficients leave the range where libjpeg-turbo's C and SIMD IDCTs
    agree (damaged data): k_idct's SIMD-arithmetic path, bit-exact with Pillow."""
    from tests.test_idct_simd_cpu import extreme_cases
    jpegs = extreme_cases(12, 28)
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    bad = []
    for i, j in enumerate(jpegs):
        ref = np.asarray(cpu_ref.decode_rgb(j))
        if info[i, 0] != 0:
            bad.append((i, "status", int(info[i, 0])))
            continue
        got = eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy()
        if not np.array_equal(got, ref):
            bad.append((i, int((got != ref).sum())))
    eng.close()
    assert not bad, bad


def test_writer_multiscan_cases_through_k_prog(gpu_device):
    """The test writer's multi-scan sequential files, non-default progression scripts,
    restart intervals per scan and mid-stream DQTs (tests/jpeg_writer.py) decoded by
    k_prog in one batch, bit-exact with Pillow; reordered interleaved scans that
    libjpeg rejects come back as zero-fill statuses like the reference's."""
    from tests import jpeg_writer as jw
    from tests.test_multiscan_cpu import multiscan_cases
    rng = np.random.default_rng(33)
    cases = multiscan_cases(rng, sizes=((83, 61), (1, 1), (130, 97), (517, 389)))
    img = textured_rgb(40, 24, rng)
    cases.append(("il_rev", jw.encode(img, [jw.scan((1, 0, 2))], samp=((1, 1),) * 3)))
    jpegs = [j for _, j in cases]
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    bad = []
    for i, (name, j) in enumerate(cases):
        ref = cpu_ref.decode_rgb(j)
        if ref is None:
            if info[i, 0] >= 0:
                bad.append((name, "status", int(info[i, 0])))
            continue
        ref = np.asarray(ref)
        if info[i, 0] != 0:
            bad.append((name, "status", int(info[i, 0])))
            continue
        got = eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy()
        if not np.array_equal(got, ref):
            bad.append((name, int((got != ref).sum())))
    eng.close()
    assert not bad, bad


def test_progressive_augmented_views(gpu_device):
    """The augment kernels on progressive-decoded images: views equal the oracle's."""
    rng = np.random.default_rng(32)
    jpegs = [encode_jpeg(textured_rgb(int(rng.integers(120, 700)), int(rng.integers(120, 700)), rng),
                         progressive=True, subsampling=int(rng.integers(0, 3))) for _ in range(6)]
    cfg = DINOAugConfig()
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    params = torch.empty(len(jpegs) * 10 * VIEW_PARAMS_DTYPE.itemsize, dtype=torch.uint8, device=gpu_device)
    views, info = eng.run_batch(d_bytes, d_off, len(jpegs), make_aug_config(cfg, 224, 96, OUT_BF16), seed=9,
                                batch_index=0, params_out=params)
    torch.cuda.synchronize()
    assert (info[:, 0].cpu() == 0).all()
    _check_views(jpegs, views, params_from_device(params), 10, torch.bfloat16, cfg.mean, cfg.std)
    eng.close()


def test_decode_workspace_greedy_no_cascade(gpu_device):
    """an image that does not fit the decode workspace is reported
    DINO_IMG_NO_SPACE and the later (small) images still decode bit-exact."""
    rng = np.random.default_rng(33)
    small = [encode_jpeg(textured_rgb(96, 64, rng)) for _ in range(4)]
    big = encode_jpeg(textured_rgb(1600, 1200, rng))
    jpegs = [small[0], big, small[1], small[2], big, small[3]]
    eng = IngestEngine(gpu_device, max_batch=len(jpegs), max_views=10, max_crop_size=224,
                       workspace_bytes=8 << 20)  # far below one 1600x1200 image (~25 MiB)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    assert list(info[:, 0]) == [0, 3, 0, 0, 3, 0], info[:, 0]
    for i in (0, 2, 3, 5):
        ref = np.asarray(cpu_ref.decode_rgb(jpegs[i]))
        np.testing.assert_array_equal(eng.copy_rgb(i, ref.shape[1], ref.shape[0]).cpu().numpy(), ref)
    # the same batch after dino_reserve to the probe's figure: everything decodes
    from dataloader_amd import fallback
    buf, off = pack_jpegs(jpegs, pin=False)
    pinfo, ws, _ = fallback.probe(buf.data_ptr(), off.numpy(), len(jpegs), 16384)
    assert (pinfo[:, 0] == 0).all()
    eng.reserve(ws, 0)
    info = eng.decode(d_bytes, d_off, len(jpegs)).cpu().numpy()
    assert (info[:, 0] == 0).all()
    ref = np.asarray(cpu_ref.decode_rgb(big))
    np.testing.assert_array_equal(eng.copy_rgb(4, 1600, 1200).cpu().numpy(), ref)
    eng.close()


def _eval_source(jpegs):
    class Src:
        _batch_size = len(jpegs)
        _resolution_src = None

        def __call__(self):
            return jpegs
    return Src()


def test_eval_tall_images_augment_workspace(gpu_device):
    """Eval uses the whole image as its crop box, so images taller than ~1.4k px
    overflowed their augment-workspace share.  The bare engine now places views greedily
    and reports the ones it cannot hold (DINO_IMG_NO_SPACE via dino_batch_info); the
    product pipeline (probe + reserve) renders all of them bit-exact."""
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import EvalAugSpec, PipelineConfig, recipe_aug_config
    from dataloader_amd.pipeline import MI355XPipelineIterator
    rng = np.random.default_rng(34)
    sizes = [(1200, 1600), (1600, 2400), (900, 2000), (640, 480)]
    jpegs = [encode_jpeg(textured_rgb(w, h, rng), quality=80) for w, h in sizes]
    spec = EvalAugSpec(crop_size=224)
    acfg = recipe_aug_config(spec)
    eng = IngestEngine(gpu_device, max_batch=4, max_views=1, max_crop_size=224)
    ccfg = make_aug_config(acfg, 224, 224, OUT_FP32)
    d_bytes, d_off = _to_dev(jpegs, gpu_device)
    eng.decode(d_bytes, d_off, 4)
    params = eng.sample_params(ccfg, 0, 0)
    views = eng.augment(ccfg, params)
    info = eng.batch_info(torch.empty(4, 4, dtype=torch.int32, device=gpu_device)).cpu().numpy()
    torch.cuda.synchronize()
    for b, j in enumerate(jpegs):
        if info[b, 0] == 0:
            assert torch.equal(views[0][b].cpu(), cpu_ref.eval_one(j, 224, out_dtype=torch.float32)), b
        else:
            assert info[b, 0] == 3 and torch.count_nonzero(views[0][b]) == 0
    eng.close()
    pipe = MI355XBackend().build_pipeline(_eval_source(jpegs), spec, PipelineConfig(output_dtype="fp32"), None)
    out = next(MI355XPipelineIterator(pipe, spec.output_map, 4))[0]["view_0"].cpu()
    stats = pipe.flush_stats()
    for b, j in enumerate(jpegs):
        assert torch.equal(out[b], cpu_ref.eval_one(j, 224, out_dtype=torch.float32)), sizes[b]
    # the backend-built pipeline keeps gpu_queue batches in flight: every launched one is counted
    assert set(stats["status"]) == {0} and stats["status"][0] == stats["images"] == 4 * stats["batches"]
    pipe.close()


def _cmyk(w, h, rng):
    img = Image.fromarray(rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8), "CMYK")
    b = io.BytesIO()
    img.save(b, format="JPEG", quality=90)
    return b.getvalue()


@pytest.mark.parametrize("route", ["device", "auto", "host"])
def test_pipeline_hands_unsupported_flavours_to_pillow(gpu_device, route):
    """CMYK and arithmetic-coded files (not decoded by the GPU) go through Pillow on the
    host and are augmented on the GPU; the progressive file decodes in k_prog
    (``multiscan_route="device"``) or in the Pillow worker pool ("auto": one such image
    in the batch; "host"); a corrupt file is zero-filled.  Every view equals the
    oracle's on every route; nothing is silently dropped."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    rng = np.random.default_rng(35)
    good = encode_jpeg(textured_rgb(300, 200, rng))
    arith = bytearray(encode_jpeg(textured_rgb(200, 160, rng)))
    k = arith.index(b"\xff\xc0")
    arith[k + 1] = 0xC9
    jpegs = [good, _cmyk(240, 180, rng), encode_jpeg(textured_rgb(256, 300, rng), progressive=True), bytes(arith),
             b"\xff\xd8\xff corrupt", _cmyk(97, 131, rng)]
    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32, n_local_crops=3)
    pipe = MI355XAugPipeline(lambda: jpegs, cfg, len(jpegs), seed=4, out_dtype="fp32", depth=1,
                             multiscan_route=route, host_workers=2)
    it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], len(jpegs))
    out = next(it)[0]
    torch.cuda.synchronize()
    recs = pipe.last_params()
    stats = pipe.flush_stats()
    nv = cfg.n_views
    for b, j in enumerate(jpegs):
        img = cpu_ref.decode_rgb(j)
        for v in range(nv):
            p = record_to_params(recs[b * nv + v])
            got = out[f"view_{v}"][b].cpu()
            if img is None:
                assert torch.count_nonzero(got) == 0, (b, v)
                continue
            ref = cpu_ref.augment_one(j, p, cfg.mean, cfg.std, out_dtype=torch.float32, decoded=img)
            tol = ONE_LEVEL + 1e-6 if p.blur else 0.0
            assert (ref - got).abs().max().item() <= tol, (b, v)
    # two CMYK + the arithmetic file (+ the progressive file off the device route)
    assert stats["host_decoded"] == (3 if route == "device" else 4)
    n_ok = sum(cpu_ref.decode_rgb(j) is not None for j in jpegs)
    assert stats["status"][0] == n_ok and sum(n for s, n in stats["status"].items() if s > 0) == 0
    pipe.close()


def test_lejepa_undecodable_image_is_a_black_canvas(gpu_device):
    """Reference CPULeJEPAPipeline (cpu.py:446-448) substitutes Image.new("RGB", (224, 224))
    for an undecodable image: its context and target views are -mean/std per channel, not 0."""
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import LeJEPAAugSpec, PipelineConfig
    from dataloader_amd.pipeline import MI355XPipelineIterator
    rng = np.random.default_rng(36)
    jpegs = [make_jpeg(300, 240, 1), b"definitely not a jpeg", make_jpeg(200, 260, 2)]
    spec = LeJEPAAugSpec(n_target_views=2)

    class Src:
        _batch_size = 3
        _resolution_src = None

        def __call__(self):
            return jpegs

    for dtype, tdt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        pipe = MI355XBackend().build_pipeline(Src(), spec, PipelineConfig(output_dtype=dtype, seed=3), None)
        out = next(MI355XPipelineIterator(pipe, spec.output_map, 3))[0]
        torch.cuda.synchronize()
        recs = pipe.last_params()
        black = Image.new("RGB", (224, 224))
        nv = len(spec.output_map)
        for v, name in enumerate(spec.output_map):
            p = record_to_params(recs[1 * nv + v])
            assert p.crop_top + p.crop_h <= 224 and p.crop_left + p.crop_w <= 224
            ref = cpu_ref.augment_one(b"", p, spec.mean, spec.std, out_dtype=tdt, decoded=black)
            assert torch.equal(out[name][1].cpu(), ref), (dtype, name)
            assert torch.count_nonzero(ref.float()) == ref.numel()
        pipe.close()
    del rng


def _c3_sizes(rng, n):
    sizes = [(1600, 1250), (1300, 1733)]  # two images with short side > 1200
    while len(sizes) < n:
        short = int(rng.integers(224, 1601))
        long_ = int(round(short * rng.uniform(1.0, 4.0 / 3.0)))
        sizes.append((long_, short) if rng.random() < 0.5 else (short, long_))
    return sizes


def test_c3_mixed_resolution_parity(gpu_device):
    """C3-shaped batch (short side 224-1600, 2 x 224 + 8 x 96 views, bf16, iBOT masks) through
    the product pipeline: every view matches the oracle replay of its record; the batch's
    mask matches the reference generator (device path, grid 16 x 16, target 128)."""
    from dataloader_amd.masking import MaskingGenerator
    from dataloader_amd.pipeline import MI355XAugPipeline
    rng = np.random.default_rng(37)
    sizes = _c3_sizes(rng, 16)
    jpegs = [encode_jpeg(textured_rgb(w, h, rng), quality=85) for w, h in sizes]
    cfg = DINOAugConfig()
    pipe = MI355XAugPipeline(lambda: jpegs, cfg, len(jpegs), seed=17, depth=1)
    out = pipe.run_one_batch()
    torch.cuda.synchronize()
    recs = pipe.last_params()
    assert (pipe.last_status() == 0).all()
    views = [out[f"view_{v}"] for v in range(cfg.n_views)]
    assert views[0].shape == (16, 3, 224, 224) and views[9].shape == (16, 3, 96, 96)
    _check_views(jpegs, views, recs, cfg.n_views, torch.bfloat16, cfg.mean, cfg.std)
    gen = MaskingGenerator((16, 16), num_masking_patches=128, device=gpu_device)
    gen.seed(17)
    ref = RefMaskingGenerator((16, 16), num_masking_patches=128, py_rng=random.Random(17),
                              np_rng=np.random.RandomState(17))
    got = gen.generate(3).cpu().numpy()
    for k in range(3):
        np.testing.assert_array_equal(got[k], ref(flat=True))
    pipe.close()


def test_c1_tar_shard_through_native_feed(gpu_device, tmp_path):
    """C1: one WebDataset tar shard of 256 textured 256 x 256 JPEGs (reference fixture layout,
    tests/fixtures/__init__.py:80-139) in the /dev/shm cache format, B = 32, full
    DINOAugConfig (n_local_crops = 8), through ShardBatchFeeder -> dino_gather -> H2D ->
    Stage 3 with two batches in flight; checked view-by-view against the oracle."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    from dataloader_amd.synthetic import make_dataset
    from dataloader_amd.tario import ShardBatchFeeder, ShmShardCache
    jpegs = make_dataset(256, 256, 256, seed=1)
    import tarfile
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
        for i, data in enumerate(jpegs):
            for name, blob in ((f"sample_{i:06d}.jpg", data),
                               (f"sample_{i:06d}.json", json.dumps({"quality_score": 1.0}).encode())):
                ti = tarfile.TarInfo(name)
                ti.size = len(blob)
                tf.addfile(ti, io.BytesIO(blob))
    cache = ShmShardCache(job_id="c1test", base_dir=tmp_path)
    cache.put("/c1/shard-00000.tar", buf.getvalue())
    cfg = DINOAugConfig()
    B = 32
    pipe = MI355XAugPipeline(ShardBatchFeeder(cache, ["/c1/shard-00000.tar"], B, nthreads=4), cfg, B, seed=21,
                             depth=2)
    it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], B)
    outs = []
    for k, out in enumerate(it):
        if k in (0, 7):  # keep two batches for the full comparison
            outs.append((k, {n: t.clone() for n, t in out[0].items()}))
    torch.cuda.synchronize()
    assert len(outs) == 2 and pipe._batch_index == 8
    stats = pipe.flush_stats()
    assert stats["images"] == 256 and stats["status"] == {0: 256}
    pipe.close()
    # replay: the records of batch k are the Philox draws of (seed, k); recompute them on a
    # fresh engine from the same bytes
    eng = IngestEngine(gpu_device, max_batch=B, max_views=10, max_crop_size=224)
    for k, out in outs:
        sel = jpegs[k * B:(k + 1) * B]
        d_bytes, d_off = _to_dev(sel, gpu_device)
        eng.decode(d_bytes, d_off, B)
        recs = params_from_device(eng.sample_params(make_aug_config(cfg, 224, 96, OUT_BF16), 21, k))
        _check_views(sel, [out[f"view_{v}"] for v in range(10)], recs, 10, torch.bfloat16, cfg.mean, cfg.std)
    eng.close()
    cache.close(remove=True)


def test_reference_cpu_backend_pins(gpu_device):
    """Reference tests/test_cpu_backend.py:146-223 restated on the HIP path: small_aug_cfg
    shapes [B,3,32,32] / [B,3,16,16], dynamic resolution, finite values, bf16 dtype,
    corrupt JPEG -> all-zero views, close semantics."""
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import DinoV2AugSpec, PipelineConfig, ResolutionSource
    cfg = DINOAugConfig(global_crop_size=32, local_crop_size=16, n_local_crops=2, max_global_crop_size=64,
                        max_local_crop_size=32)
    res = ResolutionSource(32, 16)
    state = {"n": 0}

    def source():
        state["n"] += 1
        batch = [np.frombuffer(make_jpeg(64, 64, 100 * state["n"] + i), np.uint8) for i in range(4)]
        if state["n"] == 2:
            batch[2] = np.frombuffer(b"\x00\x01 not a jpeg", np.uint8)
        return batch
    source._batch_size = 4
    source._resolution_src = res
    be = MI355XBackend()
    spec = DinoV2AugSpec(aug_cfg=cfg)
    pipe = be.build_pipeline(source, spec, PipelineConfig(device_id=0, seed=0), None)
    out = pipe.run_one_batch()
    assert [tuple(out[f"view_{i}"].shape) for i in range(4)] == [(4, 3, 32, 32)] * 2 + [(4, 3, 16, 16)] * 2
    assert all(t.dtype == torch.bfloat16 and torch.isfinite(t.float()).all() for t in out.values())
    res.set(64, 32)
    out = pipe.run_one_batch()
    assert tuple(out["view_0"].shape) == (4, 3, 64, 64) and tuple(out["view_3"].shape) == (4, 3, 32, 32)
    torch.cuda.synchronize()
    assert all(torch.count_nonzero(out[f"view_{i}"][2]) == 0 for i in range(4))
    assert all(torch.count_nonzero(out[f"view_{i}"][0]) > 0 for i in range(4))
    pipe.close()
    pipe.close()
    with pytest.raises(RuntimeError, match="close"):
        pipe.run_one_batch()


def test_device_masks_non_square(gpu_device):
    from dataloader_amd.masking import MaskingGenerator
    for grid, kw in (((10, 12), {"num_masking_patches": 40}), ((10, 16), {"num_masking_patches": 75}),
                     ((1, 1), {"num_masking_patches": 1, "min_num_patches": 1}),
                     ((8, 8), {"num_masking_patches": 0}), ((90, 90), {})):
        ref = RefMaskingGenerator(grid, py_rng=random.Random(5), np_rng=np.random.RandomState(5), **kw)
        g = MaskingGenerator(grid, device=gpu_device, **kw)
        g.seed(5)
        got = g.generate(4).cpu().numpy()
        for k in range(4):
            np.testing.assert_array_equal(got[k], ref(flat=True), err_msg=str(grid))


def test_iterator_reset_with_batches_in_flight(gpu_device):
    """reset() with batches still queued never hands over a stale slot: the next batch is
    the source's next one, bit-identical to a serial pipeline at the same batch index."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32, n_local_crops=2)
    B = 6
    batches = [[make_jpeg(160 + 8 * k, 120, 10 * k + i) for i in range(B)] for k in range(8)]
    src = iter(batches)
    pipe = MI355XAugPipeline(lambda: next(src), cfg, B, seed=8, depth=3)
    it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], B)
    next(it)          # batches 0, 1, 2 enqueued; 0 handed over
    it.reset()        # 1 and 2 dropped while in flight
    got = {k: v.clone() for k, v in next(it)[0].items()}  # batches 3, 4, 5 enqueued; 3 handed over
    torch.cuda.synchronize()
    pipe.close()
    ser = MI355XAugPipeline(lambda: batches[3], cfg, B, seed=8, depth=1)
    ser._batch_index = 3
    ref = ser.run_one_batch()
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    ser.close()


def test_user_aug_spec_decode_only(gpu_device):
    """UserAugSpec (reference CPUUserAugPipeline, cpu.py:484-500): decode + Resize(decode_size)
    + normalise on the GPU, then aug_fn on the device tensor; bit-exact vs the oracle; a batch
    whose images resize to different shapes raises like the reference's torch.stack; an
    undecodable image contributes zeros; a missing view raises ValueError (DALI iterator)."""
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import PipelineConfig, UserAugSpec
    rng = np.random.default_rng(40)
    calls = []

    def aug_fn(x):
        calls.append((tuple(x.shape), x.dtype, x.device.type))
        return {"a": x, "b": x.flip(-1)}

    def src_of(jpegs):
        class Src:
            _batch_size = len(jpegs)
            _resolution_src = None

            def __call__(self):
                return jpegs
        return Src()

    be = MI355XBackend()
    for dtype, tdt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        spec = UserAugSpec(aug_fn=aug_fn, _output_map=["a", "b"], decode_size=256, warn_not_dali=False)
        jpegs = [encode_jpeg(textured_rgb(w, h, rng), progressive=p) for (w, h), p in
                 (((640, 480), False), ((320, 240), True), ((800, 600), False), ((1024, 768), False),
                  ((341, 256), False))]
        pipe = be.build_pipeline(src_of(jpegs), spec, PipelineConfig(output_dtype=dtype), None)
        out = next(be.build_pipeline_iterator(pipe, spec, spec.output_map, len(jpegs)))[0]
        torch.cuda.synchronize()
        assert calls[-1] == ((5, 3, 256, 341), tdt, "cuda")
        for b, j in enumerate(jpegs):
            ref = cpu_ref.decode_only_one(j, 256, spec.mean, spec.std, out_dtype=tdt)
            assert torch.equal(out["a"][b].cpu(), ref), (dtype, b)
        pipe.close()
    spec = UserAugSpec(aug_fn=aug_fn, _output_map=["a"], decode_size=64, warn_not_dali=False)
    sq = [encode_jpeg(textured_rgb(s, s, rng)) for s in (100, 64, 300)] + [b"corrupt"]
    pipe = be.build_pipeline(src_of(sq), spec, PipelineConfig(output_dtype="fp32"), None)
    out = next(be.build_pipeline_iterator(pipe, spec, spec.output_map, 4))[0]["a"].cpu()
    for b, j in enumerate(sq):
        assert torch.equal(out[b], cpu_ref.decode_only_one(j, 64, spec.mean, spec.std, out_dtype=torch.float32)), b
    assert torch.count_nonzero(out[3]) == 0
    pipe.close()
    mixed = [encode_jpeg(textured_rgb(640, 480, rng)), encode_jpeg(textured_rgb(480, 640, rng))]
    pipe = be.build_pipeline(src_of(mixed), spec, PipelineConfig(output_dtype="fp32"), None)
    with pytest.raises(RuntimeError, match="equal size"):
        next(be.build_pipeline_iterator(pipe, spec, spec.output_map, 2))
    pipe.close()
    spec_bad = UserAugSpec(aug_fn=lambda x: {"a": x}, _output_map=["a", "zzz"], decode_size=64, warn_not_dali=False)
    pipe = be.build_pipeline(src_of(sq[:3]), spec_bad, PipelineConfig(output_dtype="fp32"), None)
    with pytest.raises(ValueError, match="zzz"):
        next(be.build_pipeline_iterator(pipe, spec_bad, spec_bad.output_map, 3))
    pipe.close()
