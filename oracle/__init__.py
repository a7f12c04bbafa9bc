"""CPU oracle for the DINO Stage-3 hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker / the timed CPU
baseline.  The product path (``dataloader_amd``) never imports it and fails
loudly when its HIP library is missing.

Contents
--------
``cpu_ref``      restatement of ``CPUBackend._augment_one`` / ``CPUAugPipeline``
                 (reference ``src/dino_loader/backends/cpu.py:172-367``) with an
                 explicit per-view parameter record, built on PIL + numpy + torch.
``masking_ref``  transcription of ``MaskingGenerator``
                 (reference ``src/dino_loader/masking.py:60-269``).
``synth``        textured synthetic JPEG generator for fixtures and benchmarks.

Parity pinning: the reference itself cannot be imported
here (recorded denial) and its arithmetic lives in third-party
libraries (Pillow, torchvision).  Pillow *is* present and is called directly
for every PIL primitive the reference uses (decode, crop, bicubic resize,
ImageEnhance, HSV, L conversion, solarize).  torchvision is absent: its PIL-path
functions (RandomResizedCrop.get_params, ColorJitter order, gaussian_blur,
to_tensor/normalize) are restated on torch.  The reference's own tests pin no
pixel values, so crop parity w.r.t. the reference is "parity unpinned" beyond
those primitives; the mask transcription is pinned bit-exactly by construction
(it runs the interpreter's own ``random`` and ``numpy.random``).
"""
