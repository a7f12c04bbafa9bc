"""dataloader_amd — MI355X-native Stage-3 ingest backend for DINO-style loaders.

Drop-in backend for the ``dino_loader`` backend abstraction (reference
``src/dino_loader/backends/protocol.py``): JPEG decode, random-resized crop x N,
colour jitter, grayscale, gaussian blur, solarize, normalize (bf16/fp32/fp8) and
iBOT masks as hand-written HIP kernels for gfx950.  See DESIGN.md.

The public names are resolved on first access (PEP 562), so that a process that
only needs the host hand-over (``fallback.pillow_container`` in the Pillow worker
pool) does not import torch.
"""

from importlib import import_module

_EXPORTS = {
    "MI355XBackend": ".backend",
    "DINOAugConfig": ".config",
    "DinoV2AugSpec": ".config",
    "NormStats": ".config",
    "PipelineConfig": ".config",
    "ResolutionSource": ".config",
    "MaskingGenerator": ".masking",
    "VIEW_PARAMS_DTYPE": ".params",
}

__all__ = list(_EXPORTS)


def __getattr__(name):
    mod = _EXPORTS.get(name)
    if mod is None:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    value = getattr(import_module(mod, __name__), name)
    globals()[name] = value
    return value


def __dir__():
    return sorted(list(globals()) + __all__)
