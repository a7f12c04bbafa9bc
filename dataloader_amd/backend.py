"""``MI355XBackend`` — drop-in peer of ``CPUBackend`` / ``DALIBackend``.

Satisfies the structural ``BackendProtocol`` of reference
``src/dino_loader/backends/protocol.py:18-69`` so that
``DINODataLoader(..., backend=MI355XBackend())`` (reference loader.py:431-436)
runs Stage 3 on the GPU.  Method-by-method:

* ``name`` / ``supports_fp8`` / ``supports_gpu``     protocol.py:22-29
* ``build_shard_cache``   -> :class:`tario.ShmShardCache`, the node-shared /dev/shm cache
  the GPU peer builds (dali_backend.py:85-105 -> NodeSharedShardCache): the node master
  loads shards, the other ranks wait for its writes; the native feed reads its files
* ``build_pipeline``      -> :class:`MI355XAugPipeline` (dispatch as cpu.py:649-709):
  DinoV2 multi-crop, LeJEPA and Eval view recipes on the same kernels; UserAugSpec ->
  :class:`MI355XUserAugPipeline` (decode-only recipe, ``dino_resize_batch``, then aug_fn);
  anything else raises TypeError (cpu.py:708-709)
* ``build_pipeline_iterator`` -> :class:`MI355XPipelineIterator` (cpu.py:711-722)
* ``build_h2d_stream``    -> outputs are already device-resident: identity transfer
  that orders the consumer stream after the producer (memory.py:131-165 semantics)
* ``build_fp8_formatter`` -> HIP bf16->E4M3 cast (memory.py:168-214, scale 1)
* ``init_distributed``    -> rank bookkeeping only (no collective on this path)
"""

from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import TYPE_CHECKING, Any

import torch

from . import _lib
from .pipeline import MI355XAugPipeline, MI355XPipelineIterator

if TYPE_CHECKING:
    from .tario import ShmShardCache


class DeviceH2DStream:
    """Stage-4 transfer for device-resident views: no copy, only stream ordering."""

    def __init__(self, device: torch.device, topo: Any = None) -> None:
        self._device = torch.device(device)

    @contextlib.contextmanager
    def transfer(self, batch: dict[str, list[torch.Tensor]]):
        yield self.send(batch)

    def send(self, batch: dict[str, list[torch.Tensor]]) -> dict[str, list[torch.Tensor]]:
        return {k: [t if t.device == self._device else t.to(self._device, non_blocking=True) for t in v]
                for k, v in batch.items()}

    def wait(self) -> None:
        """Views are produced on the current stream: nothing to wait for."""


class HipFP8Formatter:
    """bf16 -> float8_e4m3fn with scale 1 (TE ``cast_to_fp8`` semantics, memory.py:193-214)."""

    def quantise(self, tensor: torch.Tensor) -> torch.Tensor:
        assert tensor.dtype not in (torch.float8_e4m3fn, torch.float8_e5m2), "already FP8"
        import ctypes

        src = tensor.to(torch.bfloat16).contiguous()
        out = torch.empty(src.shape, dtype=torch.float8_e4m3fn, device=src.device)
        lib = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream(src.device).cuda_stream)
        _lib.check(lib.dino_bf16_to_fp8(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                        src.numel(), stream), "dino_bf16_to_fp8")
        return out


@dataclass
class ClusterTopology:
    label: str = "MI355X-xGMI"
    gpus_per_node: int = 8
    has_pcie: bool = True
    has_infiniband: bool = False

    @property
    def is_nvl72(self) -> bool:
        return False

    @property
    def is_grace_blackwell(self) -> bool:
        return False


@dataclass
class DistribEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    topology: ClusterTopology | None = None

    def __post_init__(self) -> None:
        if self.topology is None:
            self.topology = ClusterTopology()


def _is_dinov2_spec(spec: Any) -> bool:
    return type(spec).__name__ == "DinoV2AugSpec" and hasattr(spec, "aug_cfg")


class MI355XBackend:
    """Backend whose Stage 3 runs as HIP kernels on an MI355X (gfx950).

    ``max_image_dim``: 0 (default) decodes any JPEG side on the device; a positive value
    hands larger JPEGs to Pillow.  ``max_in_flight`` caps ``PipelineConfig.gpu_queue``
    (DALI's prefetch_queue_depth, reference pipeline.py:317 / dali_backend.py:163-164):
    each in-flight batch owns a ctx (workspaces in HBM) and a HIP stream, and three
    already hide the latency-bound entropy decode (depth 2/3/4 measured);
    ``hbm_fraction`` further caps it so that the slots' workspaces stay a small share of
    the device memory the training process also needs."""

    # initial decode workspace per image of a backend-built slot; every batch is probed on
    # the host first and the workspace grows (stream-ordered) to what the batch needs
    WS_PER_IMAGE = 4 << 20

    def __init__(self, max_image_dim: int = 0, workspace_bytes: int = 0, max_in_flight: int = 3,
                 hbm_fraction: float = 0.15, host_workers: int | None = None, multiscan_route: str = "side",
                 side_ahead: int | None = None) -> None:
        self._max_image_dim = max_image_dim
        self._workspace_bytes = workspace_bytes
        self._max_in_flight = max(1, int(max_in_flight))
        self._hbm_fraction = float(hbm_fraction)
        self._host_workers = host_workers
        # progressive / multi-scan JPEGs: decoded on the device ahead of their batch ("side",
        # default; the GPU peer decodes every flavour on the device, reference pipeline.py:429-434);
        # Pillow only for what the device decoder does not implement (MI355XAugPipeline)
        self._multiscan_route = multiscan_route
        self._side_ahead = side_ahead  # None: SIDE_AHEAD (see side_look_ahead)

    # side look-ahead in batches.  Round 4 (scripts/route_study.py, B = 512 with 32 progressive:
    # 16 -> 84.8k img/s, 48 -> 92.2-94.9k; profiles/r04_side_ahead.jsonl): a wave-decoder pool
    # takes ~45 ms alone, so the look-ahead must cover several of them.  Round 6 (c2_prog,
    # profiles/r06_side_plan/): 256 batches let the side decoder run the lane decoder on pools
    # of 4096 images (progside.side_plan), which costs the batches less GPU time per image:
    # c2_prog 72k -> 89-112k img/s.  The look-ahead's batches wait in HBM (~43 MB per C2
    # batch, plus room for its progressive images' containers: ~19 GB of the 288 at 256 with 32
    # progressive images per batch)
    SIDE_AHEAD = 256
    PREFETCH = 1  # host-half batches prepared ahead by the pipeline's prefetch thread

    def side_look_ahead(self, pipeline_cfg: Any, source: Any, depth: int) -> int:
        """Batches the side route pulls ahead of their launch (DALI's CPU prefetch queue plays
        this role for the reference's GPU peer: ``PipelineConfig.cpu_queue`` batches pulled
        ahead, reference config.py:166, pipeline.py:317): ``max(cpu_queue, SIDE_AHEAD)``, capped
        so that everything pulled and not yet handed over (look-ahead + prefetch queue + batches
        in flight) fits the source's metadata FIFO (``_ReaderAdapter._meta_queue``, 64 slots,
        shard_reader.py:98, 357-375: an overflow raises).  The look-ahead's batches wait in HBM
        (MI355XAugPipeline._stage_on_device): 256 C2 batches with 32 progressive images each
        take ~19 GB of the 288 (their bytes and their containers)."""
        want = self._side_ahead if self._side_ahead is not None else \
            max(int(os.environ.get("DINO_SIDE_AHEAD", self.SIDE_AHEAD)),
                int(getattr(pipeline_cfg, "cpu_queue", 16) or 16))
        mq = getattr(source, "_meta_queue", None)
        cap = getattr(mq, "maxsize", 0) or 0
        if cap > 0:
            # the largest look-ahead whose worst case (MI355XAugPipeline.pulled_bound) leaves one
            # FIFO entry spare
            while want > 1 and MI355XAugPipeline.pulled_bound(depth, self.PREFETCH, want) + 1 > cap:
                want -= 1
        return max(1, int(want))

    def queue_depth(self, pipeline_cfg: Any, batch_size: int, n_views: int = 10, max_crop: int = 224) -> int:
        """Batches in flight for ``pipeline_cfg.gpu_queue``, capped by ``max_in_flight`` and by
        the slots' workspace footprint (decode + augment + crop planes) against the device's HBM."""
        want = max(1, int(getattr(pipeline_cfg, "gpu_queue", 1) or 1))
        depth = min(want, self._max_in_flight)
        per_slot = (self._workspace_bytes or batch_size * self.WS_PER_IMAGE) + \
            batch_size * n_views * (max_crop * 3 * 1024 + (256 << 10)) + batch_size * n_views * 3 * max_crop ** 2
        try:
            total = torch.cuda.get_device_properties(int(getattr(pipeline_cfg, "device_id", 0))).total_memory
            depth = max(1, min(depth, int(total * self._hbm_fraction // max(per_slot, 1))))
        except Exception:  # noqa: BLE001 - no device visible: the pipeline constructor reports it
            pass
        return depth

    @property
    def name(self) -> str:
        return "mi355x"

    @property
    def supports_fp8(self) -> bool:
        return True

    @property
    def supports_gpu(self) -> bool:
        return True

    def build_shard_cache(self, job_id: str = "mi355x", node_master: bool = True, max_gb: float = 1.0,
                          prefetch_window: int = 4, timeout_s: float = 30.0, warn_threshold: float = 0.85,
                          **kwargs: Any) -> "ShmShardCache":
        """The node-local /dev/shm shard cache (reference DALIBackend.build_shard_cache,
        dali_backend.py:85-105): ``/dev/shm/<job_id>/<sha1(path)[:16]>`` files in the reference's
        format, written by the node master (``node_master``: local rank 0, loader.py:467) and
        waited for by the other ranks for up to ``timeout_s`` seconds; ``max_gb`` budget with LRU
        eviction; ``prefetch_window`` concurrent background loads; a warning past
        ``warn_threshold`` of the budget.  ``base_dir`` (keyword, default /dev/shm) relocates it."""
        from .tario import ShmShardCache
        return ShmShardCache(job_id=job_id, node_master=node_master, max_gb=max_gb,
                             base_dir=kwargs.get("base_dir", "/dev/shm"), shard_timeout_s=timeout_s,
                             prefetch_window=prefetch_window, warn_threshold=warn_threshold)

    def build_pipeline(self, source: Any, aug_spec: Any, pipeline_cfg: Any, specs: Any = None) -> MI355XAugPipeline:
        """Dispatch as CPUBackend.build_pipeline (cpu.py:649-709): DinoV2 multi-crop, LeJEPA
        (context + targets) and Eval (resize + centre crop) run on the same kernels with their
        own view recipe; UserAugSpec decodes + resizes on the GPU and applies aug_fn."""
        kind = type(aug_spec).__name__
        if kind == "UserAugSpec":  # decode-only recipe + the user's aug_fn (cpu.py:469-503)
            from .pipeline import MI355XUserAugPipeline
            norm = None
            if getattr(pipeline_cfg, "fuse_normalization", False) and specs is not None:
                from .norm import NormTable
                norm = NormTable(aug_spec, specs)
                if hasattr(source, "register_dataset_index_callback"):
                    source.register_dataset_index_callback(norm.set_dataset_indices)
            return MI355XUserAugPipeline(source, aug_spec, getattr(source, "_batch_size", 1),
                                         out_dtype=pipeline_cfg.output_dtype, device=pipeline_cfg.device_id,
                                         max_image_dim=self._max_image_dim, workspace_bytes=self._workspace_bytes,
                                         norm=norm)
        if _is_dinov2_spec(aug_spec):
            aug_cfg = aug_spec.aug_cfg
            names = None
        elif kind in ("LeJEPAAugSpec", "EvalAugSpec"):
            from .config import recipe_aug_config
            aug_cfg = recipe_aug_config(aug_spec)
            names = list(aug_spec.output_map)
        else:
            raise TypeError(f"MI355XBackend: unsupported aug_spec type {kind}.")
        out = pipeline_cfg.output_dtype
        if getattr(pipeline_cfg, "dali_fp8_output", False) or getattr(aug_spec, "fp8_output", False):
            out = "fp8"
        norm = None
        if getattr(pipeline_cfg, "fuse_normalization", False) and specs is not None:
            # per-dataset mean/std as DALIBackend wires NormSource (dali_backend.py:142-153)
            from .norm import NormTable
            norm = NormTable(aug_cfg, specs)
            if hasattr(source, "register_dataset_index_callback"):
                source.register_dataset_index_callback(norm.set_dataset_indices)
        batch = getattr(source, "_batch_size", 1)
        max_crop = max(int(aug_cfg.max_global_crop_size or aug_cfg.global_crop_size),
                       int(aug_cfg.max_local_crop_size or aug_cfg.local_crop_size))
        depth = self.queue_depth(pipeline_cfg, batch, aug_cfg.n_views, max_crop)
        return MI355XAugPipeline(
            source=source,
            aug_cfg=aug_cfg,
            batch_size=batch,
            resolution_src=getattr(source, "_resolution_src", None) if names is None else None,
            seed=pipeline_cfg.seed,
            out_dtype=out,
            device=pipeline_cfg.device_id,
            max_image_dim=self._max_image_dim,
            workspace_bytes=self._workspace_bytes or batch * self.WS_PER_IMAGE,
            norm=norm,
            view_names=names,
            depth=depth,
            prefetch=self.PREFETCH,
            host_workers=self._host_workers,
            start_host_pool=True,
            multiscan_route=self._multiscan_route,
            side_ahead=self.side_look_ahead(pipeline_cfg, source, depth),
        )

    def build_pipeline_iterator(self, pipeline: Any, aug_spec: Any, output_map: list[str],
                                batch_size: int):
        from .pipeline import MI355XUserAugIterator, MI355XUserAugPipeline
        if isinstance(pipeline, MI355XUserAugPipeline):
            return MI355XUserAugIterator(pipeline, output_map)
        return MI355XPipelineIterator(pipeline, output_map, batch_size)

    def build_h2d_stream(self, device: Any, topo: Any) -> DeviceH2DStream:
        return DeviceH2DStream(device, topo)

    def build_fp8_formatter(self) -> HipFP8Formatter:
        return HipFP8Formatter()

    def init_distributed(self, rank: int = 0, world_size: int = 1, local_rank: int = 0, local_world_size: int = 1,
                         force_topology: str | None = None) -> DistribEnv:
        return DistribEnv(rank, world_size, local_rank, local_world_size)
