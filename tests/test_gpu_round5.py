"""Round-5 GPU tests.

* The bench's own B = 512 path, pinned against the oracle: the C2 and C3
  data generators of ``bench.py`` through ``run_device_batch`` at depth 3, as ``run_leg``
  drives it; every image of a full 512-image batch decodes bit-exact with Pillow (the
  reference's own decoder, cpu.py:251), and >= 32 sampled images x 10 views match
  ``cpu_ref.augment_one`` bit for bit except blur, including the last images
  of the batch, whose views are the last ``k_hresize`` work items placed.
* Output reuse with a caller that keeps one output tensor itself.
* Pipelines alive together take different role streams.
"""

from __future__ import annotations

import random

import numpy as np
import pytest
import torch

from dataloader_amd.config import DINOAugConfig
from oracle import cpu_ref
from oracle.masking_ref import RefMaskingGenerator
from tests.test_gpu_parity import _check_views

pytestmark = pytest.mark.gpu

B = 512
DEPTH = 3


def _run_bench_pattern(uniq, mixed: bool, n_batches: int, masks: bool):
    """bench.run_leg's access pattern: the distinct encodes tiled into one device-resident
    buffer, batch k = images [kB, (k+1)B) of it, one output set per in-flight slot, depth 3."""
    from dataloader_amd.engine import pack_jpegs
    from dataloader_amd.masking import MaskingGenerator
    from dataloader_amd.pipeline import MI355XAugPipeline
    cfg = DINOAugConfig()
    n_img = n_batches * B
    jp = [uniq[i % len(uniq)] for i in range(n_img)]
    hb, off = pack_jpegs(jp, pin=True)
    dev = torch.device("cuda", 0)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    pipe = MI355XAugPipeline(None, cfg, B, seed=1234, out_dtype="bf16", device=0, max_image_dim=0, depth=DEPTH,
                             workspace_bytes=B * (40 << 20) if mixed else 0)
    ccfg = pipe._cfg(*pipe._sizes())
    views = [sl.engine.alloc_views(ccfg, B) for sl in pipe._slots]
    mg = None
    if masks:
        mg = MaskingGenerator((16, 16), num_masking_patches=128, device=dev)
        mg.seed(1234)
    got_masks = []
    for k in range(n_batches):
        pipe.run_device_batch(d_bytes, d_off[k * B:(k + 1) * B + 1], B, views=views[k % DEPTH])
        if mg is not None:
            got_masks.append(mg.generate(1).expand(B, -1))
    torch.cuda.synchronize()
    return pipe, jp, views, got_masks


def _check_slot(pipe, jp, views, k: int, sample_rng, n_sampled: int):
    """Batch k (still held by its slot): every decode vs Pillow, sampled images x 10 views vs
    the oracle replay of their records."""
    from dataloader_amd.engine import params_from_device
    from dataloader_amd.params import RECORD_BYTES
    cfg = DINOAugConfig()
    nv = cfg.n_views
    sl = pipe._slots[k % DEPTH]
    assert sl.batch_index == k
    info = sl.info.cpu().numpy()
    assert (info[:, 0] == 0).all(), np.unique(info[:, 0], return_counts=True)
    batch = jp[k * B:(k + 1) * B]
    bad = []
    for i, j in enumerate(batch):
        ref = cpu_ref.decode_rgb(j)
        arr = np.asarray(ref)
        assert (info[i, 1], info[i, 2]) == (arr.shape[1], arr.shape[0]), i
        got = sl.engine.copy_rgb(i, arr.shape[1], arr.shape[0]).cpu().numpy()
        if not np.array_equal(got, arr):
            bad.append((i, int((got != arr).sum())))
    assert not bad, f"batch {k}: decode mismatches (image, n bytes): {bad[:16]}"
    recs = params_from_device(sl.params[: B * nv * RECORD_BYTES])
    # the last 16 images (their views are the last work items k_vsizes / k_vplan place), the
    # first 8, the largest 4 and random others
    px = np.asarray([int(info[i, 1]) * int(info[i, 2]) for i in range(B)])
    pick = list(range(8)) + list(range(B - 16, B)) + [int(x) for x in np.argsort(px)[-4:]]
    rest = [i for i in range(B) if i not in pick]
    pick += [int(x) for x in sample_rng.choice(rest, size=max(0, n_sampled - len(set(pick))), replace=False)]
    pick = sorted(set(pick))
    assert len(pick) >= 32
    sel_views = [v[pick] for v in views[k % DEPTH]]
    sel_recs = np.concatenate([recs[b * nv:(b + 1) * nv] for b in pick])
    worst = _check_views([batch[b] for b in pick], sel_views, sel_recs, nv, torch.bfloat16, cfg.mean, cfg.std)
    return len(pick), worst


@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_bench_b512_batches_match_the_oracle(gpu_device, workload):
    """the timed configuration itself (B = 512, depth 3, bench.py's generators)
    against the oracle; C3 includes multi-segment images (short side up to 1600 px) and the
    batch's iBOT masks."""
    import bench
    mixed = workload == "c3"
    procs = 16
    if mixed:
        uniq = bench.make_unique(1024, 0, 0, 11, True, procs)
    else:
        uniq = bench.make_unique(1024, 640, 480, 1, False, procs)
    n_batches = 6   # two rounds of the three slots; the last three stay in their slots
    pipe, jp, views, masks = _run_bench_pattern(uniq, mixed, n_batches, masks=mixed)
    try:
        rng = np.random.default_rng(5 if mixed else 4)
        if mixed:
            sizes = [bench.jpeg_meta(j) for j in jp[(n_batches - 1) * B:n_batches * B]]
            assert max(min(w, h) for w, h in sizes) > 1200  # multi-segment images are in the checked batch
        n, worst = _check_slot(pipe, jp, views, n_batches - 1, rng, 40)
        assert n >= 32 and worst <= 0.005
        if not mixed:  # C2: every decode of a second slot's batch too
            _check_slot(pipe, jp, views, n_batches - 2, rng, 32)
        if mixed:
            ref = RefMaskingGenerator((16, 16), num_masking_patches=128, py_rng=random.Random(1234),
                                      np_rng=np.random.RandomState(1234))
            for m in masks:
                want = np.asarray(ref(flat=True))
                got = m.cpu().numpy()
                np.testing.assert_array_equal(got[0], want)
                np.testing.assert_array_equal(got[-1], want)
    finally:
        pipe.close()


def test_output_kept_by_direct_reference_is_not_refilled(gpu_device):
    """a caller that keeps one output tensor itself (not a view of it, not
    the whole dict) still sees its data after later batches; the reuse check counts references
    against a baseline measured through the same code path, not a per-interpreter constant."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator, _REFS_PIPELINE_ONLY
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    assert 2 <= _REFS_PIPELINE_ONLY <= 8
    rng = np.random.default_rng(75)
    uniq = [encode_jpeg(textured_rgb(160, 120, rng)) for _ in range(6)]
    Bs, nb = 4, 9
    batches = [[uniq[(k + i) % 6] for i in range(Bs)] for k in range(nb)]

    class Src:
        _batch_size = Bs
        _resolution_src = None

        def __init__(self):
            self._it = iter(batches)

        def __call__(self):
            return next(self._it)

    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32)
    pipe = MI355XAugPipeline(Src(), cfg, Bs, seed=15, depth=3)
    it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], Bs)
    kept, snaps, ptrs = [], [], []
    for k, out in enumerate(it):
        d = out[0]
        torch.cuda.synchronize()
        ptrs.append(d["view_3"].data_ptr())
        if k % 3 == 0:
            kept.append(d["view_3"])                 # one direct reference to one output
            snaps.append(d["view_3"].clone())
        del out, d
    torch.cuda.synchronize()
    pipe.close()
    for a, s in zip(kept, snaps):
        assert torch.equal(a, s)
    assert len(set(ptrs)) < nb  # outputs nobody kept were refilled in place


def test_concurrent_pipelines_take_separate_role_streams(gpu_device):
    """two pipelines alive together (train + val loaders) launch on different slot
    streams; once both close, the next pipeline reuses the first set (the process's stream ->
    hardware-queue mapping stays that of the first pipeline)."""
    from dataloader_amd.pipeline import MI355XAugPipeline
    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32)
    a = MI355XAugPipeline(lambda: [], cfg, 4, depth=3)
    b = MI355XAugPipeline(lambda: [], cfg, 4, depth=3)
    sa = [sl.engine.stream.cuda_stream for sl in a._slots]
    sb = [sl.engine.stream.cuda_stream for sl in b._slots]
    assert not set(sa) & set(sb)
    a.close()
    c = MI355XAugPipeline(lambda: [], cfg, 4, depth=3)
    assert [sl.engine.stream.cuda_stream for sl in c._slots] == sa
    b.close()
    c.close()
    d = MI355XAugPipeline(lambda: [], cfg, 4, depth=3)
    assert [sl.engine.stream.cuda_stream for sl in d._slots] == sa
    d.close()


def test_pixel_ops_all_inputs_match_pillow(gpu_device):
    """The ColorJitter hue op's colour conversions on the device (division-free restatement,
    pixel_ops.hpp) over all 2^24 inputs: RGB -> HSV and HSV -> RGB equal Pillow's Convert.c,
    and the whole hue shift equals ``cpu_ref.adjust_hue`` (torchvision's PIL path) for
    shifts of both signs."""
    from PIL import Image
    from dataloader_amd import _lib
    lib = _lib.load()
    idx = np.arange(1 << 24, dtype=np.uint32)
    allc = np.stack([(idx >> 16) & 255, (idx >> 8) & 255, idx & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    im = Image.fromarray(allc, "RGB")
    out = torch.empty(3 << 24, dtype=torch.uint8, device=gpu_device)
    stream = torch.cuda.current_stream().cuda_stream

    def run(op, param=0):
        _lib.check(lib.dino_pixel_ops_all(op, param, out.data_ptr(), stream), "dino_pixel_ops_all")
        return out.cpu().numpy().reshape(4096, 4096, 3)

    np.testing.assert_array_equal(run(0), np.asarray(im.convert("HSV")))
    np.testing.assert_array_equal(run(1), np.asarray(Image.fromarray(allc, "HSV").convert("RGB")))
    for f in (-0.5, -0.1, 0.037, 0.25):
        np.testing.assert_array_equal(run(2, int(f * 255) & 0xFF), np.asarray(cpu_ref.adjust_hue(im, f)), err_msg=str(f))
