"""Round-4 GPU tests: the side route as the backend default, its host-buffer forms, stream
lifetime, and output-buffer reuse under caller-held views.

* ``MI355XBackend`` routes coefficient-buffer images (progressive / multi-scan) to the device
  side decoder by default (the GPU peer decodes every flavour on the device, reference
  pipeline.py:429-434); Pillow keeps only what the device decoder does not implement;
* the side route reads a page-locked spans batch (``ShardBatchFeeder(register=True)``) from
  its shard ranges and keeps each image's true length (it sliced a never-filled
  staging buffer and took lengths from offset gaps that hold tar headers);
* closing a side pipeline destroys its dedicated streams, and a new one works in the same
  process (the segfault at close, gpurun_out/ss2.err);
* a caller that keeps only a slice of an output keeps its data (reuse was decided
  on the tensor object's refcount, blind to views);
* the colour conversion's quad and band edge cases.
"""

from __future__ import annotations

import io
import json
import tarfile

import numpy as np
import pytest
import torch

from dataloader_amd.config import DINOAugConfig, DinoV2AugSpec, PipelineConfig
from dataloader_amd.synthetic import encode_jpeg, textured_rgb

pytestmark = pytest.mark.gpu


class _ListSource:
    def __init__(self, batches):
        self._it = iter(batches)
        self._batch_size = len(batches[0])
        self._resolution_src = None

    def __call__(self):
        return next(self._it)


def _collect(it):
    outs = [{k: v.clone() for k, v in out[0].items()} for out in it]
    torch.cuda.synchronize()
    return outs


def _mixed_batches(rng, B, nb, n_prog=2):
    uniq = [encode_jpeg(textured_rgb(200 + 8 * s, 150 + 6 * s, rng)) for s in range(5)]
    progs = [encode_jpeg(textured_rgb(180 + 12 * s, 140 + 8 * s, rng), progressive=True) for s in range(3)]
    batches = [[uniq[(k + i) % 5] for i in range(B)] for k in range(nb)]
    for k in range(nb):
        for t in range(n_prog):
            batches[k][(k + 3 * t) % B] = progs[(k + t) % 3]
    return batches


def test_backend_defaults_to_the_device_side_route(gpu_device):
    """The backend's pipeline decodes progressive files on the device (side route) and matches
    the in-batch device route bit for bit; no image goes to Pillow."""
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    rng = np.random.default_rng(70)
    B, nb = 8, 6
    batches = _mixed_batches(rng, B, nb)
    spec = DinoV2AugSpec(aug_cfg=DINOAugConfig(global_crop_size=96, local_crop_size=48))
    be = MI355XBackend(host_workers=2)
    pipe = be.build_pipeline(_ListSource(batches), spec, PipelineConfig(gpu_queue=6, seed=11), None)
    assert pipe._multiscan_route == "side"
    got = _collect(be.build_pipeline_iterator(pipe, spec, spec.output_map, B))
    st = pipe.flush_stats()
    pipe.close()
    assert st["side_decoded"] == 2 * nb and st["host_decoded"] == 0 and set(st["status"]) == {0}
    ref_pipe = MI355XAugPipeline(_ListSource(batches), spec.aug_cfg, B, seed=11, depth=3, multiscan_route="device")
    ref = _collect(MI355XPipelineIterator(ref_pipe, spec.output_map, B))
    ref_pipe.close()
    assert len(ref) == len(got) == nb
    for k, (a, b) in enumerate(zip(ref, got)):
        for name in a:
            assert torch.equal(a[name], b[name]), (k, name)


def _shards(samples, per_shard):
    shards = []
    for s0 in range(0, len(samples), per_shard):
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w") as tf:
            for i in range(s0, min(len(samples), s0 + per_shard)):
                for name, data in ((f"sample_{i:06d}.jpg", samples[i]),
                                   (f"sample_{i:06d}.json", json.dumps({"i": i, "pad": "x" * (i % 7)}).encode())):
                    ti = tarfile.TarInfo(name)
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))
        shards.append(buf.getvalue())
    return shards


def test_side_route_reads_page_locked_spans_batches(gpu_device, tmp_path):
    """a page-locked spans batch (never packed) with progressive images on the
    side route: the side decoder reads the images from their shard ranges, and the merged batch
    keeps every image's true length (the gap to the next image holds tar headers and a JSON
    sidecar).  Views equal the packed feed on the in-batch device route, and the native feed on
    the side route."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    from dataloader_amd.tario import NativeShardFeed, ShardBatchFeeder, ShmShardCache
    rng = np.random.default_rng(71)
    B, nb = 8, 6
    samples = [j for b in _mixed_batches(rng, B, nb) for j in b]
    shards = _shards(samples, 20)  # batches straddle shards
    cache = ShmShardCache(job_id="side_spans", base_dir=tmp_path)
    paths = [f"/d/p-{k}.tar" for k in range(len(shards))]
    for p, t in zip(paths, shards):
        cache.put(p, t)
    cfg = DINOAugConfig(global_crop_size=96, local_crop_size=48)
    names = [f"view_{i}" for i in range(cfg.n_views)]

    def run(src, route):
        pipe = MI355XAugPipeline(src, cfg, B, seed=12, depth=3, multiscan_route=route, host_workers=2, side_ahead=3)
        outs = _collect(MI355XPipelineIterator(pipe, names, B))
        st = pipe.flush_stats()
        pipe.close()
        return outs, st

    packed = ShardBatchFeeder(cache, paths, B, nthreads=2, register=False)
    ref, st0 = run(packed, "device")
    packed.close()
    locked = ShardBatchFeeder(cache, paths, B, nthreads=2, register=True)
    got, st1 = run(locked, "side")
    locked.close()
    assert locked.register_error is None and not locked._reg
    feed = NativeShardFeed(cache, paths, B, nthreads=2, slots=4)
    nat, st2 = run(feed, "side")
    feed.close()
    assert len(ref) == len(got) == len(nat) == nb
    assert st1["side_decoded"] == st2["side_decoded"] == 2 * nb and st0["side_decoded"] == 0
    assert set(st0["status"]) == set(st1["status"]) == set(st2["status"]) == {0}
    for k in range(nb):
        for name in ref[k]:
            assert torch.equal(ref[k][name], got[k][name]), (k, name, "spans")
            assert torch.equal(ref[k][name], nat[k][name]), (k, name, "native feed")
    cache.close(remove=True)


def test_side_pipeline_close_destroys_streams_and_reopens(gpu_device):
    """a side pipeline is created, run and closed, three times in one process;
    every close destroys its dedicated streams (no stream is left alive for the process),
    every run gives the same views, and every pipeline launches on the same slot streams."""
    from dataloader_amd import progside
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    rng = np.random.default_rng(72)
    B, nb = 8, 4
    batches = _mixed_batches(rng, B, nb, n_prog=3)
    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32)
    names = [f"view_{i}" for i in range(cfg.n_views)]
    base = progside.live_streams()
    runs = []
    slot_streams = []
    for _ in range(3):
        pipe = MI355XAugPipeline(_ListSource(batches), cfg, B, seed=13, depth=2, multiscan_route="side",
                                 host_workers=2, side_ahead=2)
        # every pipeline reuses the process's role streams (pipeline.role_stream): the same
        # hardware-queue mapping as the first pipeline's
        slot_streams.append([sl.engine.stream.cuda_stream for sl in pipe._slots])
        outs = _collect(MI355XPipelineIterator(pipe, names, B))
        assert pipe.flush_stats()["side_decoded"] == 3 * nb
        assert progside.live_streams() > base
        pipe.close()
        assert progside.live_streams() == base
        runs.append(outs)
        del pipe, outs
        torch.cuda.empty_cache()
    for outs in runs[1:]:
        for a, b in zip(runs[0], outs):
            for name in a:
                assert torch.equal(a[name], b[name]), name
    assert slot_streams[0] == slot_streams[1] == slot_streams[2]


def test_kept_slice_of_an_output_is_not_refilled(gpu_device):
    """a caller that keeps only a view (slice / chunk) of a batch's output
    still sees its data after later batches; outputs nobody references are refilled."""
    from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator
    rng = np.random.default_rng(73)
    uniq = [encode_jpeg(textured_rgb(160, 120, rng)) for _ in range(6)]
    B, nb = 4, 9
    batches = [[uniq[(k + i) % 6] for i in range(B)] for k in range(nb)]
    cfg = DINOAugConfig(global_crop_size=64, local_crop_size=32)
    pipe = MI355XAugPipeline(_ListSource(batches), cfg, B, seed=14, depth=3)
    it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], B)
    kept, snaps, ptrs = [], [], []
    for k, out in enumerate(it):
        d = out[0]
        torch.cuda.synchronize()
        ptrs.append(d["view_0"].data_ptr())
        if k % 2 == 0:  # keep a slice of view_0 and a chunk of view_5 only
            kept.append((d["view_0"][:2], d["view_5"].chunk(2)[1]))
            snaps.append((d["view_0"][:2].clone(), d["view_5"].chunk(2)[1].clone()))
        del out, d
    torch.cuda.synchronize()
    pipe.close()
    for (a, b), (sa, sb) in zip(kept, snaps):
        assert torch.equal(a, sa) and torch.equal(b, sb)
    assert len(set(ptrs)) < nb  # the batches nobody kept were refilled in place


def test_colour_quads_and_band_edges_bit_exact(gpu_device):
    """k_idct + k_color over widths of every residue mod 4 (4:2:0 quads that wrap a row), heights
    that end inside an 8-row band, the smallest fancy-upsampled chroma (3 samples wide) next to
    box-upsampled 2-sample chroma, baseline, restart-interval and progressive files, and other
    samplings in the same batch: bit-exact with Pillow (the round-4 fused k_ycolor was measured
    slower and removed; these are its edge cases on the kernels that remain)."""
    from tests.test_gpu_parity import _to_dev
    from dataloader_amd.engine import IngestEngine
    from oracle import cpu_ref
    rng = np.random.default_rng(404)
    cases = []
    for w, h in ((2304, 17), (2305, 9), (2303, 23), (2302, 8), (2301, 31), (5, 5), (4, 4), (6, 3), (13, 11),
                 (641, 479), (96, 1), (1, 40)):
        cases.append((f"base_{w}x{h}", encode_jpeg(textured_rgb(w, h, rng), quality=90, subsampling=2)))
    cases.append(("prog_1000x9", encode_jpeg(textured_rgb(1000, 9, rng), subsampling=2, progressive=True)))
    cases.append(("prog_333x250", encode_jpeg(textured_rgb(333, 250, rng), subsampling=2, progressive=True)))
    cases.append(("rst_777x333", encode_jpeg(textured_rgb(777, 333, rng), subsampling=2, restart_mcus=5)))
    cases.append(("s422_300x200", encode_jpeg(textured_rgb(300, 200, rng), subsampling=1)))
    cases.append(("s444_301x201", encode_jpeg(textured_rgb(301, 201, rng), subsampling=0)))
    cases.append(("gray_250x90", encode_jpeg(textured_rgb(250, 90, rng), gray=True)))
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
