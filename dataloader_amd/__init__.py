"""dataloader_amd — MI355X-native Stage-3 ingest backend for DINO-style loaders.

Drop-in backend for the ``dino_loader`` backend abstraction (reference
``src/dino_loader/backends/protocol.py``): JPEG decode, random-resized crop x N,
colour jitter, grayscale, gaussian blur, solarize, normalize (bf16/fp32/fp8) and
iBOT masks as hand-written HIP kernels for gfx950.  See DESIGN.md.
"""

from .backend import MI355XBackend
from .config import DINOAugConfig, DinoV2AugSpec, NormStats, PipelineConfig, ResolutionSource
from .masking import MaskingGenerator
from .params import VIEW_PARAMS_DTYPE

__all__ = ["MI355XBackend", "DINOAugConfig", "DinoV2AugSpec", "NormStats", "PipelineConfig",
           "ResolutionSource", "MaskingGenerator", "VIEW_PARAMS_DTYPE"]
