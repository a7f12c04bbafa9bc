"""Host pre-screen (``dino_probe``) and the Pillow hand-over of ``fallback.py`` — no GPU.

The probe runs the device parser on the host; its status must agree with what the
reference does for each flavour: Pillow raises (negative -> zeros, as cpu.py:252-253)
or decodes (0 on the GPU path, 1 handed over to Pillow).  Workspace bytes must equal
the sum of the per-image plan (plan.hpp) and grow with the image.
"""

from __future__ import annotations

import io

import numpy as np
from PIL import Image

from dataloader_amd import fallback
from dataloader_amd.engine import pack_jpegs
from dataloader_amd.params import make_aug_config
from dataloader_amd.config import DINOAugConfig
from dataloader_amd.synthetic import encode_jpeg, textured_rgb
from oracle import cpu_ref


def _probe(jpegs, cfg=None, max_dim=0, raw_mask=None):
    buf, off = pack_jpegs(jpegs, pin=False)
    return fallback.probe(buf.data_ptr(), off.numpy(), len(jpegs), max_dim, cfg, raw_mask)


def _cmyk_jpeg(w, h, rng):
    img = Image.fromarray(rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8), "CMYK")
    b = io.BytesIO()
    img.save(b, format="JPEG", quality=90)
    return b.getvalue()


def _with_sof_byte(jpeg: bytes, marker: int | None = None, precision: int | None = None) -> bytes:
    k = jpeg.index(b"\xff\xc0")
    out = bytearray(jpeg)
    if marker is not None:
        out[k + 1] = marker
    if precision is not None:
        out[k + 4] = precision
    return bytes(out)


def test_probe_classifies_like_the_reference():
    rng = np.random.default_rng(3)
    base = encode_jpeg(textured_rgb(120, 80, rng))
    prog = encode_jpeg(textured_rgb(120, 80, rng), progressive=True)
    raw = fallback.raw_container(textured_rgb(33, 17, rng))
    cases = [
        (base, 0, 0),                                  # baseline
        (prog, 0, 1),                                  # progressive: GPU coefficient-buffer path
        (raw, 0, 2),                                   # pre-decoded RGB
        (_cmyk_jpeg(40, 24, rng), 1, None),            # CMYK: Pillow decodes, GPU does not
        (_with_sof_byte(base, marker=0xC9), 1, None),  # arithmetic SOF: left to Pillow
        (_with_sof_byte(base, precision=12), -1, None),  # Pillow: "cannot handle 12-bit layers"
        (b"not a jpeg", -1, None),
        (b"", -1, None),
        (prog[: len(prog) // 2], -2, None),            # truncated progressive: Pillow raises
    ]
    rm = np.array([k == 2 for _, _, k in cases], np.uint8)
    info, ws, aws = _probe([c for c, _, _ in cases], raw_mask=rm)
    for i, (data, want, kind) in enumerate(cases):
        assert info[i, 0] == want, (i, info[i])
        if kind is not None:
            assert info[i, 3] == kind
        if kind == 2:
            continue  # the raw container is this ABI's own input format
        ref = cpu_ref.decode_rgb(data)
        if want < 0:
            assert ref is None, i          # the reference zero-fills exactly these
        else:
            assert ref is not None, i
    assert ws > 0 and aws == 0
    # the container magic is never trusted in user data.  Unmarked, a blob that
    # starts with it is not a JPEG, exactly as Pillow sees it (the reference zero-fills)
    info, _, _ = _probe([raw])
    assert info[0, 0] == -1 and cpu_ref.decode_rgb(raw) is None


def test_probe_workspace_grows_with_images():
    rng = np.random.default_rng(5)
    small = [encode_jpeg(textured_rgb(64, 48, rng)) for _ in range(3)]
    big = small + [encode_jpeg(textured_rgb(1600, 1200, rng))]
    cfg = make_aug_config(DINOAugConfig(), 224, 96, 0)
    _, ws_s, aws_s = _probe(small, cfg)
    _, ws_b, aws_b = _probe(big, cfg)
    assert ws_b > ws_s + 1600 * 1200 * 3 and aws_b > aws_s
    # augment bound covers the widest crop of every view: >= H x S x 3 per view
    assert aws_b - aws_s >= 1200 * (2 * 224 + 8 * 96) * 3


def test_probe_limits():
    rng = np.random.default_rng(6)
    j = encode_jpeg(textured_rgb(300, 40, rng))
    info, _, _ = _probe([j], max_dim=256)
    assert info[0, 0] == 4  # DINO_IMG_LIMIT: the caller's ceiling, not a reference failure
    assert fallback.route_mask(info, True, "auto", 8)[0]  # ... handed to Pillow by the pipeline
    # the default has no side limit: very wide / tall JPEGs decode on the device
    wide = [encode_jpeg(textured_rgb(9000, 40, rng)), encode_jpeg(textured_rgb(24, 17000, rng))]
    info, _, _ = _probe(wide)
    assert (info[:, 0] == 0).all() and list(info[:, 1]) == [9000, 24] and list(info[:, 2]) == [40, 17000]
    # a header claiming > 2 x PIL.Image.MAX_IMAGE_PIXELS: Pillow raises DecompressionBombError
    bomb = bytearray(j)
    k = bomb.index(b"\xff\xc0")
    bomb[k + 5:k + 9] = (20000).to_bytes(2, "big") + (20000).to_bytes(2, "big")
    info, _, _ = _probe([bytes(bomb)])
    assert info[0, 0] == -4
    assert cpu_ref.decode_rgb(bytes(bomb)) is None


def test_hand_over_replaces_only_unsupported():
    rng = np.random.default_rng(7)
    good = encode_jpeg(textured_rgb(50, 40, rng))
    cmyk = _cmyk_jpeg(30, 20, rng)
    arith = _with_sof_byte(good, marker=0xC9)
    jpegs = [good, cmyk, arith, b"junk"]
    info, _, _ = _probe(jpegs)
    out, n, rm = fallback.hand_over(jpegs, info[:, 0])
    assert n == 2 and out[0] is good and out[3] == b"junk"
    for i in (1, 2):
        ref = cpu_ref.decode_rgb(jpegs[i])
        if ref is None:          # Pillow raised: travels as zero bytes (device: corrupt -> zeros)
            assert out[i] == b""
        else:
            w, h = ref.size
            assert out[i][16:] == np.asarray(ref).tobytes() and int.from_bytes(out[i][4:8], "little") == w
    info2, _, _ = _probe(out, raw_mask=rm)
    assert (info2[[0, 1], 0] == 0).all() and info2[1, 3] == 2


def test_route_mask_policies():
    """Coefficient-buffer images (kind 1) go to the host on "host", never on "device", and on
    "auto" only while the batch holds at most host_max of them; unsupported images always
    (when host_fallback); corrupt/truncated never (the device zero-fills them like the reference)."""
    rng = np.random.default_rng(8)
    base = encode_jpeg(textured_rgb(64, 48, rng))
    prog = encode_jpeg(textured_rgb(64, 48, rng), progressive=True)
    jpegs = [base, prog, _cmyk_jpeg(30, 20, rng), prog, prog[:100], b"junk"]
    info, _, _ = _probe(jpegs)
    m = lambda route, hmax=8, fb=True: list(fallback.route_mask(info, fb, route, hmax))  # noqa: E731
    assert m("device") == [False, False, True, False, False, False]
    assert m("host") == [False, True, True, True, False, False]
    assert m("auto") == m("host") and m("auto", hmax=2) == m("host")
    assert m("auto", hmax=1) == m("device")
    assert m("host", fb=False) == [False, True, False, True, False, False]


def test_hand_over_in_worker_pool_matches_serial():
    """The spawn-context Pillow pool returns the same containers as the in-process hand-over."""
    rng = np.random.default_rng(9)
    prog = [encode_jpeg(textured_rgb(70 + 9 * i, 50, rng), progressive=True) for i in range(3)]
    jpegs = [prog[0], _cmyk_jpeg(30, 20, rng), prog[1], b"\xff\xd8junk", prog[2]]
    info, _, _ = _probe(jpegs)
    mask = fallback.route_mask(info, True, "host", 0)
    assert list(mask) == [True, True, True, False, True]
    serial, n, rm = fallback.hand_over(jpegs, info[:, 0], mask)
    pool = fallback.HostDecoder(2)
    try:
        pooled, n2, rm2 = fallback.hand_over(jpegs, info[:, 0], mask, pool)
    finally:
        pool.close()
    assert n == n2 == 4 and pooled == serial and pooled[3] == jpegs[3] and (rm == rm2).all()
    info2, _, _ = _probe(pooled, raw_mask=rm)
    assert list(info2[:, 3]) == [2, 2, 2, -1, 2]


def test_host_decoder_falls_back_in_process(monkeypatch):
    """a pool that cannot start (e.g. spawned children that cannot import the
    training script's __main__) is reported at start() and the hand-over continues in
    this process with the same bytes."""
    import warnings
    rng = np.random.default_rng(10)
    cmyk = _cmyk_jpeg(30, 20, rng)
    dec = fallback.HostDecoder(2)

    class _Broken:
        def __init__(self, *a, **k):
            raise OSError("cannot start workers")
    import concurrent.futures
    monkeypatch.setattr(concurrent.futures, "ProcessPoolExecutor", _Broken)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        dec.start()
    assert any("in-process" in str(x.message) for x in w)
    assert dec.submit(cmyk).result() == fallback.pillow_container(cmyk)
    dec.close()
