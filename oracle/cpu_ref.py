"""CPU restatement of ``CPUBackend``'s DINOv2 multi-crop path (TEST INFRA ONLY).

Follows, op for op, reference ``src/dino_loader/backends/cpu.py``:

* ``_augment_one``           cpu.py:235-267  -> :func:`augment_one`
* ``_random_resized_crop``   cpu.py:172-183  -> :func:`resized_crop` (+ :func:`rrc_get_params`)
* ``_color_jitter``          cpu.py:194-207  -> :func:`color_jitter`
* ``_gaussian_blur``         cpu.py:210-220  -> :func:`gaussian_blur`
* ``_to_tensor_normalized``  cpu.py:223-232  -> :func:`to_tensor_normalized`
* ``CPUAugPipeline.run_one_batch`` view-param table cpu.py:325-341 -> :func:`view_table`,
  stacking cpu.py:362-367 -> :func:`run_batch`
* ``CPUEvalPipeline.run_one_batch`` cpu.py:395-413 (``_resize_shorter`` cpu.py:190-191,
  ``_center_crop`` cpu.py:186-187) -> :func:`eval_one`, :func:`eval_geometry`
* ``CPULeJEPAPipeline.run_one_batch`` cpu.py:435-461 -> :func:`lejepa_one` (views replayed
  from their :class:`ViewParams`, as the multi-crop ones)
* ``CPUUserAugPipeline.run_one_batch`` cpu.py:484-500 -> :func:`decode_only_one`

The reference draws every random quantity from process-global RNGs inside the
ops (torch global RNG for RandomResizedCrop/ColorJitter, Python ``random`` for
the coin flips and blur sigma).  Here every draw is an explicit field of
:class:`ViewParams`, so "same JPEG bytes + same ViewParams => same output" is a
checkable statement.  :func:`draw_params_like_cpubackend` reproduces the
reference's draw *order* from a ``torch.Generator`` + ``random.Random`` pair,
i.e. what a single-worker CPUBackend would have drawn.

torchvision (the reference's ``~=0.25`` pin) is not installed; its PIL-path
functions are restated on torch/PIL below, each citing the torchvision routine
it follows.  Pillow is the real thing (12.2.0 / libjpeg-turbo 3.1.4.1 here).
"""

from __future__ import annotations

import io
import math
import random
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image, ImageEnhance, ImageOps

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # reference config.py:271
IMAGENET_STD = (0.229, 0.224, 0.225)    # reference config.py:272

# ColorJitter op ids, torchvision ColorJitter.forward order semantics.
OP_BRIGHTNESS, OP_CONTRAST, OP_SATURATION, OP_HUE = 0, 1, 2, 3


@dataclass
class ViewParams:
    """Every random decision ``_augment_one`` makes for one (sample, view).

    Field names mirror ``dino_view_params`` in ``include/dino_ingest.h``.
    """

    out_size: int
    crop_top: int = 0        # RandomResizedCrop i
    crop_left: int = 0       # RandomResizedCrop j
    crop_h: int = 1
    crop_w: int = 1
    flip: bool = False
    jitter: bool = False
    order: tuple = (0, 1, 2, 3)
    brightness: float = 1.0
    contrast: float = 1.0
    saturation: float = 1.0
    hue: float = 0.0
    gray: bool = False
    blur: bool = False
    sigma: float = 1.0
    ksize: int = 3
    solarize: bool = False
    resize_w: int = 0        # resample target of the crop box (0 -> out_size)
    resize_h: int = 0
    out_x: int = 0           # view window inside the resampled box
    out_y: int = 0


@dataclass
class ViewSpec:
    """Per-view static config (reference ``_ViewAugParams``, cpu.py:153-164)."""

    crop_size: int
    scale: tuple
    blur_prob: float
    sol_prob: float


@dataclass
class AugCfg:
    """Subset of reference ``DINOAugConfig`` (config.py:243-272) the hot path reads."""

    global_crop_size: int = 224
    local_crop_size: int = 96
    n_global_crops: int = 2
    n_local_crops: int = 8
    global_crops_scale: tuple = (0.32, 1.0)
    local_crops_scale: tuple = (0.05, 0.32)
    blur_prob_global1: float = 1.0
    blur_prob_global2: float = 0.1
    blur_prob_local: float = 0.5
    solarize_prob: float = 0.2
    color_jitter_prob: float = 0.8
    grayscale_prob: float = 0.2
    blur_sigma_min: float = 0.1
    blur_sigma_max: float = 2.0
    brightness: float = 0.8
    contrast: float = 0.8
    saturation: float = 0.8
    hue: float = 0.2
    flip_prob: float = 0.5
    mean: tuple = field(default=IMAGENET_MEAN)
    std: tuple = field(default=IMAGENET_STD)


def view_table(cfg: AugCfg, global_size: int | None = None, local_size: int | None = None) -> list[ViewSpec]:
    """Reference cpu.py:325-341: view 0 blur p1, view 1 blur p2 + solarize, locals."""
    g = cfg.global_crop_size if global_size is None else global_size
    l = cfg.local_crop_size if local_size is None else local_size
    out = []
    for i in range(cfg.n_global_crops):
        out.append(ViewSpec(g, cfg.global_crops_scale,
                            cfg.blur_prob_global1 if i == 0 else cfg.blur_prob_global2,
                            cfg.solarize_prob if i == 1 else 0.0))
    for _ in range(cfg.n_local_crops):
        out.append(ViewSpec(l, cfg.local_crops_scale, cfg.blur_prob_local, 0.0))
    return out


# ---------------------------------------------------------------------------
# Decode (cpu.py:250-253)
# ---------------------------------------------------------------------------

def decode_rgb(jpeg_bytes: bytes) -> Image.Image | None:
    """``Image.open(BytesIO(b)).convert("RGB")``; ``None`` where the reference returns zeros."""
    try:
        return Image.open(io.BytesIO(bytes(jpeg_bytes))).convert("RGB")
    except Exception:  # noqa: BLE001 - mirrors cpu.py:252
        return None


# ---------------------------------------------------------------------------
# RandomResizedCrop (torchvision transforms.RandomResizedCrop.get_params / forward)
# ---------------------------------------------------------------------------

def rrc_get_params(width: int, height: int, scale, ratio, gen: torch.Generator):
    """torchvision ``RandomResizedCrop.get_params``: 10 tries, then central fallback."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=gen).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1], generator=gen)).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = torch.randint(0, height - h + 1, size=(1,), generator=gen).item()
            j = torch.randint(0, width - w + 1, size=(1,), generator=gen).item()
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def resized_crop(img: Image.Image, top: int, left: int, h: int, w: int, size: int) -> Image.Image:
    """torchvision ``F.resized_crop`` PIL path: ``crop`` then ``resize(BICUBIC)``."""
    img = img.crop((left, top, left + w, top + h))
    return img.resize((size, size), Image.BICUBIC)


# ---------------------------------------------------------------------------
# ColorJitter (torchvision ColorJitter.get_params/forward + _functional_pil)
# ---------------------------------------------------------------------------

def adjust_brightness(img, f):
    return ImageEnhance.Brightness(img).enhance(f)


def adjust_contrast(img, f):
    return ImageEnhance.Contrast(img).enhance(f)


def adjust_saturation(img, f):
    return ImageEnhance.Color(img).enhance(f)


def adjust_hue(img, hue_factor):
    """torchvision ``_functional_pil.adjust_hue``: uint8 wrap-add on PIL's H channel."""
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError(hue_factor)
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    np_h += np.uint8(int(hue_factor * 255) & 0xFF)   # == np.int8(x*255).view(uint8)
    h = Image.fromarray(np_h, "L")
    return Image.merge("HSV", (h, s, v)).convert("RGB")


def color_jitter(img, p: ViewParams):
    fns = {OP_BRIGHTNESS: (adjust_brightness, p.brightness),
           OP_CONTRAST: (adjust_contrast, p.contrast),
           OP_SATURATION: (adjust_saturation, p.saturation),
           OP_HUE: (adjust_hue, p.hue)}
    for op in p.order:
        fn, f = fns[int(op)]
        img = fn(img, f)
    return img


# ---------------------------------------------------------------------------
# Gaussian blur (torchvision F.gaussian_blur, PIL input -> tensor path)
# ---------------------------------------------------------------------------

def gaussian_kernel1d(ksize: int, sigma: float) -> torch.Tensor:
    """torchvision ``_functional_tensor._get_gaussian_kernel1d`` (float32)."""
    half = (ksize - 1) * 0.5
    x = torch.linspace(-half, half, steps=ksize, dtype=torch.float32)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    return pdf / pdf.sum()


def gaussian_blur(img: Image.Image, ksize: int, sigma: float) -> Image.Image:
    """``pil_to_tensor`` -> float32 reflect-pad depthwise conv2d -> round -> uint8 -> PIL."""
    t = torch.from_numpy(np.array(img, dtype=np.uint8, copy=True)).permute(2, 0, 1)
    k1 = gaussian_kernel1d(ksize, float(sigma))
    k2 = torch.mm(k1[:, None], k1[None, :])
    kernel = k2.expand(3, 1, ksize, ksize)
    x = t.unsqueeze(0).to(torch.float32)
    pad = ksize // 2
    x = F.pad(x, [pad, pad, pad, pad], mode="reflect")
    y = F.conv2d(x, kernel, groups=3)
    y = torch.round(y).to(torch.uint8).squeeze(0)
    return Image.fromarray(y.permute(1, 2, 0).contiguous().numpy(), "RGB")


def blur_ksize(sigma: float) -> int:
    """cpu.py:219."""
    return max(3, int(sigma * 4 + 1) | 1)


# ---------------------------------------------------------------------------
# to_tensor + normalize + cast (cpu.py:223-232)
# ---------------------------------------------------------------------------

def to_tensor_normalized(img: Image.Image, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                         out_dtype=torch.bfloat16) -> torch.Tensor:
    t = torch.from_numpy(np.array(img, dtype=np.uint8, copy=True)).permute(2, 0, 1).contiguous()
    t = t.to(torch.float32).div(255)
    m = torch.as_tensor(np.asarray(mean, dtype=np.float32).tolist(), dtype=torch.float32).view(-1, 1, 1)
    s = torch.as_tensor(np.asarray(std, dtype=np.float32).tolist(), dtype=torch.float32).view(-1, 1, 1)
    t = t.sub(m).div(s)
    if out_dtype == torch.float8_e4m3fn:
        # reference Stage 5: bf16 output, then TE cast_to_fp8 with scale 1 (memory.py:193-214)
        return t.to(torch.bfloat16).to(torch.float8_e4m3fn)
    return t.to(out_dtype)


# ---------------------------------------------------------------------------
# The per-view op chain (cpu.py:235-267)
# ---------------------------------------------------------------------------

def eval_geometry(w: int, h: int, crop_size: int) -> tuple[int, int, int, int]:
    """(new_w, new_h, left, top) of CPUEvalPipeline: torchvision ``Resize(int(crop * 256 / 224))``
    of the shorter side (``_compute_resized_output_size``: long side = int(size * long / short)),
    then ``CenterCrop`` offsets ``int(round((dim - crop) / 2.0))`` (torchvision F.center_crop)."""
    size = int(crop_size * 256 / 224)
    if w <= h:
        new_w, new_h = size, int(size * h / w)
    else:
        new_w, new_h = int(size * w / h), size
    return new_w, new_h, int(round((new_w - crop_size) / 2.0)), int(round((new_h - crop_size) / 2.0))


def eval_one(jpeg_bytes: bytes, crop_size: int, mean=IMAGENET_MEAN, std=IMAGENET_STD,
             out_dtype=torch.bfloat16, decoded: Image.Image | None = None) -> torch.Tensor:
    """CPUEvalPipeline for one sample (cpu.py:405-411): decode, resize shorter side (BICUBIC),
    centre crop, normalise; undecodable -> zeros."""
    img = decoded if decoded is not None else decode_rgb(jpeg_bytes)
    if img is None:
        return torch.zeros(3, crop_size, crop_size, dtype=out_dtype)
    new_w, new_h, left, top = eval_geometry(img.size[0], img.size[1], crop_size)
    img = img.resize((new_w, new_h), Image.BICUBIC)
    img = img.crop((left, top, left + crop_size, top + crop_size))
    return to_tensor_normalized(img, mean, std, out_dtype)


def decode_only_one(jpeg_bytes: bytes, decode_size: int, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                    out_dtype=torch.bfloat16) -> torch.Tensor:
    """CPUUserAugPipeline for one sample (cpu.py:491-497): decode, torchvision
    ``Resize(decode_size)`` of the shorter side (BICUBIC, geometry of eval_geometry),
    normalise; undecodable -> zeros (3, decode_size, decode_size)."""
    img = decode_rgb(jpeg_bytes)
    if img is None:
        return torch.zeros(3, decode_size, decode_size, dtype=out_dtype)
    w, h = img.size
    nw, nh = (decode_size, int(decode_size * h / w)) if w <= h else (int(decode_size * w / h), decode_size)
    if (nw, nh) != img.size:
        img = img.resize((nw, nh), Image.BICUBIC)
    return to_tensor_normalized(img, mean, std, out_dtype)


def lejepa_one(jpeg_bytes: bytes, params: list, mean=IMAGENET_MEAN, std=IMAGENET_STD,
               out_dtype=torch.bfloat16, decoded: Image.Image | None = None) -> list[torch.Tensor]:
    """CPULeJEPAPipeline for one sample (cpu.py:447-459), with its draws as records:
    context = RRC + ColorJitter + flip (flip commutes with the per-pixel jitter ops),
    targets = RRC only."""
    img = decoded if decoded is not None else decode_rgb(jpeg_bytes)
    return [augment_one(jpeg_bytes, p, mean, std, out_dtype, decoded=img) for p in params]


def augment_image(img: Image.Image, p: ViewParams) -> Image.Image:
    """All uint8 stages of ``_augment_one`` after decode, with explicit params."""
    if p.resize_w:  # a window of the resampled crop box (Eval: resize shorter side + centre crop)
        img = img.crop((p.crop_left, p.crop_top, p.crop_left + p.crop_w, p.crop_top + p.crop_h))
        if (p.resize_w, p.resize_h) != img.size:
            img = img.resize((p.resize_w, p.resize_h), Image.BICUBIC)
        img = img.crop((p.out_x, p.out_y, p.out_x + p.out_size, p.out_y + p.out_size))
    else:
        img = resized_crop(img, p.crop_top, p.crop_left, p.crop_h, p.crop_w, p.out_size)
    if p.flip:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    if p.jitter:
        img = color_jitter(img, p)
    if p.gray:
        img = img.convert("L").convert("RGB")
    if p.blur:
        img = gaussian_blur(img, p.ksize, p.sigma)
    if p.solarize:
        img = ImageOps.solarize(img, 128)
    return img


def augment_one(jpeg_bytes: bytes, p: ViewParams, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                out_dtype=torch.bfloat16, decoded: Image.Image | None = None) -> torch.Tensor:
    img = decoded if decoded is not None else decode_rgb(jpeg_bytes)
    if img is None:
        return torch.zeros(3, p.out_size, p.out_size, dtype=out_dtype)
    return to_tensor_normalized(augment_image(img, p), mean, std, out_dtype)


def run_batch(jpegs, params, mean=IMAGENET_MEAN, std=IMAGENET_STD, out_dtype=torch.bfloat16,
              decode_per_view: bool = False) -> dict[str, torch.Tensor]:
    """``{view_i: [B,3,S,S]}`` like ``CPUAugPipeline.run_one_batch`` (cpu.py:362-367).

    ``params[b][v]`` is the ViewParams of sample b, view v.  With
    ``decode_per_view`` every view re-decodes the JPEG exactly as cpu.py:251 does.
    """
    n_views = len(params[0])
    per_view: list[list[torch.Tensor]] = [[] for _ in range(n_views)]
    for b, jpg in enumerate(jpegs):
        img = None if decode_per_view else decode_rgb(jpg)
        for v in range(n_views):
            if decode_per_view:
                t = augment_one(jpg, params[b][v], mean, std, out_dtype)
            elif img is None:
                t = torch.zeros(3, params[b][v].out_size, params[b][v].out_size, dtype=out_dtype)
            else:
                t = augment_one(jpg, params[b][v], mean, std, out_dtype, decoded=img)
            per_view[v].append(t)
    return {f"view_{v}": torch.stack(ts) for v, ts in enumerate(per_view)}


# ---------------------------------------------------------------------------
# Reference draw order (what a single-worker CPUBackend draws)
# ---------------------------------------------------------------------------

def draw_params_like_cpubackend(width: int, height: int, spec: ViewSpec, cfg: AugCfg,
                                gen: torch.Generator, rnd: random.Random) -> ViewParams:
    """Consume ``gen`` (torch RNG) and ``rnd`` (Python random) in cpu.py's order."""
    i, j, h, w = rrc_get_params(width, height, spec.scale, (3 / 4, 4 / 3), gen)
    p = ViewParams(out_size=spec.crop_size, crop_top=i, crop_left=j, crop_h=h, crop_w=w)
    p.flip = rnd.random() < cfg.flip_prob                                      # cpu.py:256
    if not (rnd.random() > cfg.color_jitter_prob):                             # cpu.py:202
        p.jitter = True
        # torchvision ColorJitter.get_params: randperm(4) then four uniforms
        p.order = tuple(int(x) for x in torch.randperm(4, generator=gen))
        b = (max(0.0, 1 - cfg.brightness), 1 + cfg.brightness)
        c = (max(0.0, 1 - cfg.contrast), 1 + cfg.contrast)
        s = (max(0.0, 1 - cfg.saturation), 1 + cfg.saturation)
        hh = (-cfg.hue, cfg.hue)
        p.brightness = float(torch.empty(1).uniform_(b[0], b[1], generator=gen))
        p.contrast = float(torch.empty(1).uniform_(c[0], c[1], generator=gen))
        p.saturation = float(torch.empty(1).uniform_(s[0], s[1], generator=gen))
        p.hue = float(torch.empty(1).uniform_(hh[0], hh[1], generator=gen))
    p.gray = rnd.random() < cfg.grayscale_prob                                 # cpu.py:262
    if not (rnd.random() > spec.blur_prob):                                    # cpu.py:216
        p.blur = True
        p.sigma = rnd.uniform(cfg.blur_sigma_min, cfg.blur_sigma_max)         # cpu.py:218
        p.ksize = blur_ksize(p.sigma)
    if spec.sol_prob > 0 and rnd.random() < spec.sol_prob:                     # cpu.py:265
        p.solarize = True
    return p
