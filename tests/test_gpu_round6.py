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
    """An engine whose progressive images take the lane decoder or the wave decoder
    (dino_ctx_set_prog_decoder)."""
    eng = IngestEngine(dev, max_batch=n, max_views=1, max_crop_size=8)
    eng.set_prog_decoder(lane)
    return eng


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
    # dino_copy_rgb_packed (the side decoder's containers): every image, in reverse order, into
    # one buffer at odd and 16-byte aligned offsets, gaps left untouched
    import ctypes
    sizes = [int(info[i, 1]) * int(info[i, 2]) * 3 for i in range(len(jpegs))]
    order = list(range(len(jpegs)))[::-1]
    offs, pos = [], 0
    for k, i in enumerate(order):
        pos += 16 + (k & 1)
        offs.append(pos)
        pos += sizes[i]
    big = torch.full((pos + 16,), 0xA5, dtype=torch.uint8, device=dev)
    d_idx = torch.tensor(order, dtype=torch.int32, device=dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    assert eng.lib.dino_copy_rgb_packed(eng._ctx, len(order), ctypes.c_void_p(d_idx.data_ptr()),
                                        ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(big.data_ptr()), 0,
                                        eng._s()) == 0
    torch.cuda.synchronize()
    hb_big = big.cpu().numpy()
    for k, i in enumerate(order):
        if st[i, 0] == 0:  # (an image that did not decode is skipped)
            assert np.array_equal(hb_big[offs[k]:offs[k] + sizes[i]], rgb[i].reshape(-1)), i
        assert (hb_big[offs[k] - 16 - (k & 1):offs[k]] == 0xA5).all(), i
    # absolute destinations (null base) with the container header written in front
    from dataloader_amd import _lib as L
    big.fill_(0xA5)
    d_abs = d_off + big.data_ptr()
    torch.cuda.synchronize()
    assert eng.lib.dino_copy_rgb_packed(eng._ctx, len(order), ctypes.c_void_p(d_idx.data_ptr()),
                                        ctypes.c_void_p(d_abs.data_ptr()), None, L.COPY_HEADER, eng._s()) == 0
    torch.cuda.synchronize()
    hb_big = big.cpu().numpy()
    for k, i in enumerate(order):
        if st[i, 0] == 0:
            assert np.array_equal(hb_big[offs[k]:offs[k] + sizes[i]], rgb[i].reshape(-1)), i
            hdr = hb_big[offs[k] - 16:offs[k]].copy().view("<u4")
            assert list(hdr) == [L.RAW_MAGIC, int(info[i, 1]), int(info[i, 2]), 0], (i, hdr)
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


# ----------------------------------------------------------------------------- the drop-in route at B = 512
B = 512


class _Recording:
    """A callable source with the reference's conventions (_batch_size, _resolution_src;
    _ReaderAdapter.__call__, shard_reader.py:346-376) that keeps every batch it hands out."""

    def __init__(self, src):
        self._src = src
        self._batch_size = src._batch_size
        self._resolution_src = None
        self.batches = []

    def __call__(self):
        b = self._src()
        self.batches.append(b)
        return b


def _check_handed(pipe, out, batch_jpegs, k, sample_rng, tdtype, n_sampled=36):
    """The batch just handed over by the iterator (its slot still holds it): every decode
    bit-exact with Pillow, >= 32 sampled images x 10 views against the oracle replay of their
    records (tests/test_gpu_parity.py _check_views: bit-exact except blur)."""
    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.engine import params_from_device
    from dataloader_amd.params import RECORD_BYTES
    from tests.test_gpu_parity import _check_views
    torch.cuda.synchronize()
    sl = pipe._handed
    assert sl.batch_index == k
    info = sl.info.cpu().numpy()
    assert (info[:, 0] == 0).all(), np.unique(info[:, 0], return_counts=True)
    bad = []
    for i, j in enumerate(batch_jpegs):
        arr = np.asarray(cpu_ref.decode_rgb(j))
        assert (info[i, 1], info[i, 2]) == (arr.shape[1], arr.shape[0]), i
        got = sl.engine.copy_rgb(i, arr.shape[1], arr.shape[0]).cpu().numpy()
        if not np.array_equal(got, arr):
            bad.append((i, int((got != arr).sum())))
    assert not bad, f"batch {k}: decode mismatches (image, bytes): {bad[:16]}"
    cfg = DINOAugConfig()
    nv = cfg.n_views
    recs = params_from_device(sl.params[: B * nv * RECORD_BYTES])
    views = [out[0][name] for name in pipe._names]
    assert all(v.dtype == tdtype and v.shape[0] == B for v in views)
    prog = [i for i, j in enumerate(batch_jpegs) if b"\xff\xc2" in j[:4096]]
    pick = list(range(8)) + list(range(B - 16, B)) + prog[:6]
    rest = [i for i in range(B) if i not in pick]
    pick += [int(x) for x in sample_rng.choice(rest, size=max(0, n_sampled - len(set(pick))), replace=False)]
    pick = sorted(set(pick))
    assert len(pick) >= 32
    sel_views = [v[pick] for v in views]
    sel_recs = np.concatenate([recs[b * nv:(b + 1) * nv] for b in pick])
    worst = _check_views([batch_jpegs[b] for b in pick], sel_views, sel_recs, nv, tdtype, cfg.mean, cfg.std)
    assert worst <= 0.005
    return len(pick), len(prog)


@pytest.mark.parametrize("fp8", [False, True], ids=["bf16", "fp8"])
def test_dropin_side_route_b512_from_a_host_source(gpu_device, fp8):
    """MI355XBackend.build_pipeline + build_pipeline_iterator, as DINODataLoader
    drives them (PipelineConfig.gpu_queue 3 batches in flight), from a host list source with one
    progressive JPEG in 16 (the default route: prefetch thread -> dino_gather_probe -> side
    look-ahead staged in HBM -> side decoder -> raw containers merged into the batch), at
    B = 512: a batch with its progressive images checked whole against Pillow and 36 sampled
    images x 10 views against the oracle; FP8 (PipelineConfig.dali_fp8_output, memory.py:193-214)
    the same way."""
    import bench
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import DINOAugConfig, DinoV2AugSpec, PipelineConfig
    uniq = bench.make_unique(256, 640, 480, 1, False, 16)
    uniq_prog = bench.make_unique(32, 640, 480, 31, False, 16, 1.0)
    src = _Recording(bench._ProgMixSource(uniq, uniq_prog, B, 1.0 / 16, 80))
    pcfg = PipelineConfig(device_id=0, seed=77, gpu_queue=3, dali_fp8_output=fp8)
    backend = MI355XBackend()
    spec = DinoV2AugSpec(aug_cfg=DINOAugConfig())
    pipe = backend.build_pipeline(src, spec, pcfg, None)
    try:
        assert pipe._multiscan_route == "side" and pipe.depth == 3
        it = backend.build_pipeline_iterator(pipe, spec, spec.output_map, B)
        k_check = 6
        for k in range(k_check + 1):
            out = next(it)
        n, n_prog = _check_handed(pipe, out, src.batches[k_check], k_check, np.random.default_rng(8),
                                  torch.float8_e4m3fn if fp8 else torch.bfloat16)
        assert n_prog == B // 16
        st = pipe.flush_stats()
        assert st["side_decoded"] >= (k_check + 1) * (B // 16) and st["host_decoded"] == 0
        assert set(st["status"]) == {0}
        # the default look-ahead (256 batches, a source without a metadata FIFO) puts the side
        # contexts on the lane decoder (progside.side_plan)
        assert pipe._side_ahead == 256 and st["side_lanes"] is True and pipe._side.lane_launches > 0
    finally:
        pipe.close()


def test_dropin_native_feed_b512(gpu_device, tmp_path):
    """the e2e path's host half (/dev/shm shard-cache files, reference
    shard_cache.py:584-609 -> NativeShardFeed: C++ openers + packer, pinned slots, probe) through
    MI355XBackend.build_pipeline + build_pipeline_iterator at B = 512, depth 3: a batch that
    straddles two shards checked whole against Pillow and 36 images x 10 views against the
    oracle."""
    import bench
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import DINOAugConfig, DinoV2AugSpec, PipelineConfig
    from dataloader_amd.tario import NativeShardFeed, ShmShardCache
    uniq = bench.make_unique(256, 640, 480, 3, False, 16)
    per = 700
    n_shards = 8
    order = [uniq[(k * 7919 + i) % len(uniq)] for k in range(n_shards) for i in range(per)]
    blobs = [bench.make_shards(order[k * per:(k + 1) * per], per)[0] for k in range(n_shards)]
    cache = ShmShardCache(job_id=f"r6_dropin_{os.getpid()}", base_dir="/dev/shm", max_gb=16.0)
    paths = [f"/synthetic/r6/shard-{k:05d}.tar" for k in range(n_shards)]
    try:
        for p, blob in zip(paths, blobs):
            cache.put(p, blob)
        feed = NativeShardFeed(cache, paths, B, nthreads=8, slots=6, shuffle=False)
        pcfg = PipelineConfig(device_id=0, seed=78, gpu_queue=3)
        backend = MI355XBackend()
        spec = DinoV2AugSpec(aug_cfg=DINOAugConfig())
        pipe = backend.build_pipeline(feed, spec, pcfg, None)
        try:
            assert pipe._feed and pipe.depth == 3
            it = backend.build_pipeline_iterator(pipe, spec, spec.output_map, B)
            k_check = 5  # images 2560 .. 3071: shards 3 and 4
            for k in range(k_check + 1):
                out = next(it)
            _check_handed(pipe, out, order[k_check * B:(k_check + 1) * B], k_check, np.random.default_rng(9),
                          torch.bfloat16)
            st = pipe.flush_stats()
            assert set(st["status"]) == {0} and st["host_decoded"] == 0
        finally:
            pipe.close()
            feed.close()
    finally:
        cache.close(remove=True)


def test_role_streams_released_before_exit(gpu_device, tmp_path):
    """a process that used depth-3 pipelines (role streams from
    dino_stream_create) ends with those streams destroyed by the pipeline module's atexit hook,
    before library finalization, and exits 0 -- whether it closed its pipeline or not."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    script = tmp_path / "child.py"
    script.write_text(f"""
import atexit, sys
sys.path.insert(0, {str(root)!r})
# registered before the pipeline module's hook, so it runs after it (atexit is LIFO)
atexit.register(lambda: print("left", len(sys.modules["dataloader_amd.pipeline"]._RAW_ROLE_STREAMS), flush=True))
import torch
from dataloader_amd import pipeline as P
from dataloader_amd.config import DINOAugConfig
from dataloader_amd.engine import pack_jpegs
from dataloader_amd.synthetic import make_jpeg
jp = [make_jpeg(96, 80, s) for s in range(8)]
hb, off = pack_jpegs(jp, pin=True)
dev = torch.device("cuda", 0)
pipe = P.MI355XAugPipeline(None, DINOAugConfig(global_crop_size=64, local_crop_size=32, n_local_crops=2), 8,
                           depth=3)
for k in range(4):
    pipe.run_device_batch(hb.to(dev), off.to(dev), 8)
torch.cuda.synchronize()
assert P._RAW_ROLE_STREAMS, "no dino_stream_create role stream was made"
if sys.argv[1] == "close":
    pipe.close()
""")
    for mode in ("close", "leave_open"):
        r = subprocess.run([sys.executable, str(script), mode], capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (mode, r.stderr[-2000:])
        assert "left 0" in r.stdout, (mode, r.stdout[-500:])
