"""C-ABI surface and host-side logic (CPU only: no compute calls)."""

from __future__ import annotations

import ctypes
import re
import struct
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent


def test_library_exports_every_header_symbol():
    from dataloader_amd import _lib
    header = (ROOT / "include" / "dino_ingest.h").read_text()
    declared = set(re.findall(r"^(?:int|const char\*)\s+(dino_\w+)\(", header, flags=re.M))
    assert declared, "no declarations parsed"
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in dino_ingest.h but not exported"
    assert declared == set(_lib.exported_symbols())
    assert lib.dino_abi_version() == _lib.ABI_VERSION == 4


def test_ctx_create_fails_loudly_without_gpu():
    from dataloader_amd import _lib
    from dataloader_amd.engine import IngestEngine
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.DinoError):
        IngestEngine(0, max_batch=4)


def test_bad_arguments_rejected_before_any_launch():
    from dataloader_amd import _lib
    from dataloader_amd.params import DinoLimits
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.dino_ctx_create(0, ctypes.byref(DinoLimits(0, 10, 224, 4096, 0)), ctypes.byref(ctx)) == -1
    assert b"max_batch" in lib.dino_last_error()
    assert lib.dino_ctx_create(0, ctypes.byref(DinoLimits(4, 10, 2048, 4096, 0)), ctypes.byref(ctx)) == -1
    assert b"max_crop_size" in lib.dino_last_error()
    assert lib.dino_decode(None, None, None, None, 1, None, None) == -1
    assert lib.dino_masks(0, 4, 2, 1, 2, 0.0, 1.0, 1, None, None, None, None) == -1


def test_pack_jpegs_offsets():
    from dataloader_amd.engine import pack_jpegs
    items = [b"abc", np.frombuffer(b"\x01\x02", np.uint8), b"", b"zzzz"]
    buf, off = pack_jpegs(items, pin=False)
    assert off.tolist() == [0, 3, 5, 5, 9]
    assert bytes(buf[:9].numpy()) == b"abc\x01\x02zzzz"


def test_config_mirrors_reference_defaults():
    from dataloader_amd.config import DINOAugConfig, DinoV2AugSpec, PipelineConfig, ResolutionSource
    c = DINOAugConfig()
    assert (c.global_crop_size, c.local_crop_size, c.n_views) == (224, 96, 10)
    assert c.max_global_crop_size == 224 and c.max_local_crop_size == 96
    assert c.crop_size_at_epoch(5) == 224
    c2 = DINOAugConfig(resolution_schedule=[(10, 448), (0, 224)])
    assert c2.crop_size_at_epoch(3) == 224 and c2.crop_size_at_epoch(10) == 448
    spec = DinoV2AugSpec(aug_cfg=DINOAugConfig(n_local_crops=2))
    assert spec.output_map == ["view_0", "view_1", "view_2", "view_3"]
    assert spec.split_views([1, 2, 3, 4]) == ([1, 2], [3, 4]) and spec.supports_masking
    r = ResolutionSource(32, 16)
    r.set(64, 32)
    g, l = r()
    assert (int(g), int(l)) == (64, 32) and g.dtype == np.int32
    assert PipelineConfig().output_dtype == "bf16"


def test_backend_protocol_surface():
    from dataloader_amd.backend import MI355XBackend
    be = MI355XBackend()
    assert be.name == "mi355x" and be.supports_gpu and be.supports_fp8
    for m in ("build_shard_cache", "build_pipeline", "build_pipeline_iterator", "build_h2d_stream",
              "build_fp8_formatter", "init_distributed"):
        assert callable(getattr(be, m))
    env = be.init_distributed(rank=2, world_size=8, local_rank=2, local_world_size=8)
    assert (env.rank, env.world_size, env.topology.is_nvl72) == (2, 8, False)

    class CustomSpec:  # unsupported spec types raise TypeError like CPUBackend (cpu.py:708-709)
        pass
    from dataloader_amd.config import PipelineConfig
    with pytest.raises(TypeError):
        be.build_pipeline(lambda: [], CustomSpec(), PipelineConfig())


def test_shard_cache_lru(tmp_path):
    """build_shard_cache gives the node-shared /dev/shm cache (reference dali_backend.py:85-105):
    reference file format, LRU eviction over the budget, background prefetch, a shard larger
    than the whole budget raises ([FIX-EVICT-EARLY])."""
    from dataloader_amd import tario
    from dataloader_amd.backend import MI355XBackend
    cache = MI355XBackend().build_shard_cache(job_id="lru", node_master=True, max_gb=100 / (1 << 30),
                                              prefetch_window=2, timeout_s=5.0, warn_threshold=0.5,
                                              base_dir=tmp_path / "shm")
    assert isinstance(cache, tario.ShmShardCache) and cache.node_master and cache.shard_timeout_s == 5.0
    paths = []
    for i in range(3):
        p = tmp_path / f"s{i}.tar"
        p.write_bytes(bytes([i]) * 40)
        paths.append(str(p))
    with pytest.warns(RuntimeWarning, match="utilisation"):
        for p in paths:
            assert cache.get(p) == bytes([paths.index(p)]) * 40
    assert cache.utilisation <= 1.0
    assert not tario.is_ready(cache.path_of(paths[0])) and tario.is_ready(cache.path_of(paths[2]))  # evicted
    with cache.get_view(paths[-1]) as mv:
        assert bytes(mv[:1]) == b"\x02"
    raw = cache.path_of(paths[2]).read_bytes()
    assert struct.unpack("QQ", raw[:16]) == (40, tario.READY_MAGIC) and raw[16:] == b"\x02" * 40
    cache.prefetch(paths[0])                               # background load, then a blocking get
    assert cache.get(paths[0]) == b"\x00" * 40
    big = tmp_path / "big.tar"
    big.write_bytes(b"x" * 200)
    with pytest.raises(RuntimeError, match="exceeds the entire shm budget"):
        cache.get(str(big))
    cache.close(remove=True)


def test_masking_generator_validation_matches_reference():
    from dataloader_amd.masking import MaskingGenerator
    with pytest.raises(ValueError):
        MaskingGenerator(4, num_masking_patches=17)
    with pytest.raises(ValueError):
        MaskingGenerator(4, num_masking_patches=-1)
    with pytest.raises(ValueError):
        MaskingGenerator(8, num_masking_patches=30, min_num_patches=31, max_num_patches=30)
    MaskingGenerator(8, num_masking_patches=0)  # min > max allowed when target == 0
    g = MaskingGenerator((10, 16))
    assert g.get_shape() == (10, 16) and g.num_masking_patches == 80 and "10x16" in repr(g)


def _doc_blocks(lang: str) -> list[str]:
    import re
    text = (ROOT / "INTEGRATION.md").read_text()
    return re.findall(r"```" + lang + r"\n(.*?)```", text, flags=re.S)


def _header_params() -> dict[str, int]:
    """Parameter count of every function the header declares."""
    import re
    hdr = (ROOT / "include" / "dino_ingest.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(dino_\w+)\s*\(([^;{]*?)\)\s*;", hdr, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_integration_c_examples_compile_against_the_header(tmp_path):
    """every C example of INTEGRATION.md compiles against include/dino_ingest.h."""
    import subprocess
    blocks = _doc_blocks("c")
    assert len(blocks) >= 2
    for k, code in enumerate(blocks):
        src = tmp_path / f"example_{k}.c"
        src.write_text(code)
        r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Werror", "-I", str(ROOT / "include"),
                            str(src)], capture_output=True, text=True)
        assert r.returncode == 0, f"INTEGRATION.md C block {k}:\n{r.stderr}"


def test_integration_ctypes_argtypes_match_header_and_binding():
    """Every ``lib.<fn>.argtypes = [...]`` of INTEGRATION.md has the header's parameter count and
    _lib.py's, and _lib.py binds every header function with the header's count."""
    import re

    from dataloader_amd import _lib
    lib = _lib.load()
    params = _header_params()
    for name in _lib.exported_symbols():
        assert name in params, name
        assert len(getattr(lib, name).argtypes) == params[name], (name, getattr(lib, name).argtypes, params[name])
    seen = 0
    for code in _doc_blocks("python"):
        for m in re.finditer(r"lib\.(dino_\w+)\.argtypes\s*=\s*\[(.*?)\]\n", code, flags=re.S):
            items = [x for x in re.split(r",(?![^()]*\))", m.group(2).replace("\n", " ")) if x.strip()]
            assert len(items) == params[m.group(1)], (m.group(1), len(items), params[m.group(1)])
            seen += 1
    assert seen >= 3


def test_backend_side_look_ahead_fits_the_metadata_fifo():
    """The side route pulls max(PipelineConfig.cpu_queue, 256) batches ahead (DALI's CPU prefetch
    queue, reference config.py:166), never more than the source's metadata FIFO holds
    (_ReaderAdapter._meta_queue, 64 slots, shard_reader.py:98, 357-375: an overflow raises)."""
    import queue

    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import PipelineConfig

    class Src:
        def __init__(self, n):
            self._meta_queue = queue.Queue(maxsize=n)

    from dataloader_amd.pipeline import MI355XAugPipeline

    be = MI355XBackend()
    # worst case pulled and not handed over: look-ahead + prefetch queue (1 + min(ahead, 4)) +
    # the batches being packed (PACK_THREADS) + the puller's queue (RAW_AHEAD) and the batch it
    # holds + the batches in flight; one FIFO entry stays spare
    from dataloader_amd.pipeline import PACK_THREADS, RAW_AHEAD
    assert RAW_AHEAD == 2 and PACK_THREADS == 1
    assert MI355XAugPipeline.pulled_bound(3, 1, 48) == 48 + 5 + 1 + 3 + 3
    assert be.SIDE_AHEAD == 256
    assert be.side_look_ahead(PipelineConfig(), Src(64), 3) == 64 - 3 - 7 - 3
    assert be.side_look_ahead(PipelineConfig(), object(), 3) == 256
    assert be.side_look_ahead(PipelineConfig(), Src(20), 3) == 20 - 3 - 7 - 3
    assert be.side_look_ahead(PipelineConfig(cpu_queue=60), Src(64), 3) == 64 - 3 - 7 - 3
    assert be.side_look_ahead(PipelineConfig(cpu_queue=300), object(), 3) == 300
    assert MI355XBackend(side_ahead=8).side_look_ahead(PipelineConfig(), Src(64), 3) == 8
    assert MI355XBackend(side_ahead=80).side_look_ahead(PipelineConfig(), Src(64), 3) == 64 - 3 - 7 - 3
    for cap in (12, 20, 64):
        for depth in (1, 3, 6):
            for cq in (1, 16, 60, 200):
                a = be.side_look_ahead(PipelineConfig(cpu_queue=cq), Src(cap), depth)
                if a > 1:
                    assert MI355XAugPipeline.pulled_bound(depth, be.PREFETCH, a) + 1 <= cap, (cap, depth, cq)


def test_side_plan_follows_the_look_ahead(monkeypatch):
    """The side decoder runs the lane decoder on pools of 4096 when the look-ahead holds two
    such pools in flight (>= 128 batches), the wave decoder on pools of 512 otherwise (a source
    whose metadata FIFO caps the look-ahead); DINO_SIDE_DECODER / DINO_SIDE_MAX override."""
    from dataloader_amd import progside
    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import PipelineConfig

    monkeypatch.delenv("DINO_SIDE_DECODER", raising=False)
    monkeypatch.delenv("DINO_SIDE_MAX", raising=False)
    be = MI355XBackend()
    assert progside.side_plan(be.side_look_ahead(PipelineConfig(), object(), 3)) == (True, 4096)

    class Fifo:
        def __init__(self):
            import queue
            self._meta_queue = queue.Queue(maxsize=64)

    assert progside.side_plan(be.side_look_ahead(PipelineConfig(), Fifo(), 3)) == (False, 512)
    assert progside.side_plan(127) == (False, 512) and progside.side_plan(128) == (True, 4096)
    monkeypatch.setenv("DINO_SIDE_DECODER", "wave")
    assert progside.side_plan(256) == (False, 512)
    monkeypatch.setenv("DINO_SIDE_DECODER", "lanes")
    monkeypatch.setenv("DINO_SIDE_MAX", "1024")
    assert progside.side_plan(8) == (True, 1024)


def test_side_look_ahead_engages_only_with_coefficient_buffer_images():
    """on the side route the look-ahead (up to side_ahead batches pulled ahead and
    staged in HBM) is engaged only while progressive images are about: a stream of baseline
    batches is pulled one at a time and never staged; a batch with a progressive image arms it
    for side_ahead batches (the batches already ahead are staged too); then it disengages."""
    from collections import deque

    from dataloader_amd.pipeline import MI355XAugPipeline

    class PB:
        def __init__(self, k, prog):
            self.k, self.prog, self.side, self.staged = k, prog, None, False

    prog_at = {5, 6}
    src = iter(range(40))
    p = MI355XAugPipeline.__new__(MI355XAugPipeline)
    p._side_ahead, p._side_hot, p._ahead, p._source_end = 4, 0, deque(), False
    p._side = None
    p.host_seconds = {"wait": 0.0}
    p.stats = {}
    pulled = []

    def pull_one(block):
        k = next(src)
        pulled.append(k)
        return PB(k, k in prog_at)

    class Job:  # a side decode already finished
        pending = False

        def done(self):
            return True

    def side_submit(pb):
        pb.side = Job() if pb.prog else None

    def stage(pb):
        pb.staged = True

    p._pull_one, p._side_submit, p._stage_on_device = pull_one, side_submit, stage
    out = [p._pull_side() for _ in range(16)]
    assert [pb.k for pb in out] == list(range(16))           # order kept
    staged = {pb.k for pb in out if pb.staged}
    # cold: one at a time (batches 0-4 pulled only as they are handed out, never staged); batch 5
    # arms the look-ahead; it stays engaged for side_ahead batches after the last progressive one
    assert not staged & {0, 1, 2, 3, 4}
    assert {5, 6, 7, 8, 9} <= staged and max(staged) <= 6 + 4
    assert not staged & set(range(11, 16))
    assert pulled[:6] == [0, 1, 2, 3, 4, 5]


def test_side_look_ahead_fills_behind_a_running_side_decode():
    """A head batch whose side decode has not finished is not handed out while the look-ahead
    has room: further batches are pulled (blocking) behind it, so when the host half is the
    bottleneck the decode's latency is covered by later batches instead of stalling the launch."""
    from collections import deque

    from dataloader_amd.pipeline import MI355XAugPipeline

    class Job:
        pending = False

        def __init__(self):
            self.finished = False

        def done(self):
            return self.finished

    class PB:
        def __init__(self, k):
            self.k, self.side, self.staged = k, Job() if k == 0 else None, False

    src = iter(range(40))
    p = MI355XAugPipeline.__new__(MI355XAugPipeline)
    p._side_ahead, p._side_hot, p._ahead, p._source_end = 6, 0, deque(), False
    p._side = None
    p.host_seconds = {"wait": 0.0}
    p.stats = {}
    blocking = []

    def pull_one(block):
        blocking.append(block)
        return PB(next(src))

    p._pull_one, p._side_submit, p._stage_on_device = pull_one, lambda pb: None, lambda pb: None
    first = p._pull_side()
    assert first.k == 0 and len(p._ahead) == 5           # batches 1-5 pulled behind the busy head
    assert all(blocking)                                  # each of them waited for the host half
    first.side.finished = True
    assert [p._pull_side().k for _ in range(3)] == [1, 2, 3]


def test_output_set_reuse_check_sees_every_outside_reference():
    """The output ring reuses a set only when nothing outside the pipeline holds a tensor
    of it or its memory (pipeline._all_unshared; ADVICE r4: no assumed interpreter
    reference counts).  CPU tensors, same reference structure as a slot's."""
    from dataloader_amd import pipeline as P

    views = [torch.empty(4), torch.empty(4)]
    ring = [("key", views, None)]  # the ring's list holds the tensors
    outputs = {"a": views[0], "b": views[1]}  # one slot's outputs dict
    assert P._all_unshared(views, [1, 1])
    held = views[0]  # a direct reference kept by the caller
    assert not P._all_unshared(views, [1, 1])
    del held
    assert P._all_unshared(views, [1, 1])
    part = views[1][:2]  # a view of the memory
    assert not P._all_unshared(views, [1, 1])
    del part
    caller = dict(outputs)  # the caller's own dict of the batch
    assert not P._all_unshared(views, [1, 1])
    del caller
    assert P._all_unshared(views, [1, 1])
    del outputs  # no slot dict holds them any more
    assert P._all_unshared(views, [0, 0])
    assert ring
