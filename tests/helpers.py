"""Shared test helpers: oracle <-> ABI record conversion, emulator binding."""

from __future__ import annotations

import ctypes
import io
import os
from pathlib import Path

import numpy as np

from dataloader_amd.params import VIEW_PARAMS_DTYPE
from oracle.cpu_ref import ViewParams

ROOT = Path(__file__).resolve().parent.parent
EMU_SO = ROOT / "tests" / "emu" / "libdino_emu.so"
P = ctypes.c_void_p


def record_to_params(rec) -> ViewParams:
    names = rec.dtype.names or ()

    def opt(k):  # records saved before the window fields existed (golden fixtures) have none
        return int(rec[k]) if k in names else 0

    return ViewParams(
        out_size=int(rec["out_size"]), crop_top=int(rec["crop_top"]), crop_left=int(rec["crop_left"]),
        crop_h=int(rec["crop_h"]), crop_w=int(rec["crop_w"]), flip=bool(rec["flip"]),
        jitter=bool(rec["jitter"]), order=tuple(int(x) for x in rec["order"]),
        brightness=float(rec["brightness"]), contrast=float(rec["contrast"]),
        saturation=float(rec["saturation"]), hue=float(rec["hue"]), gray=bool(rec["gray"]),
        blur=bool(rec["blur"]), sigma=float(rec["sigma"]), ksize=int(rec["ksize"]),
        solarize=bool(rec["solarize"]), resize_w=opt("resize_w"), resize_h=opt("resize_h"),
        out_x=opt("out_x"), out_y=opt("out_y"))


def params_to_record(p: ViewParams) -> np.ndarray:
    r = np.zeros((), VIEW_PARAMS_DTYPE)
    r["out_size"] = p.out_size
    r["crop_top"], r["crop_left"], r["crop_h"], r["crop_w"] = p.crop_top, p.crop_left, p.crop_h, p.crop_w
    r["flip"], r["jitter"], r["gray"], r["blur"], r["solarize"] = p.flip, p.jitter, p.gray, p.blur, p.solarize
    r["order"] = np.asarray(p.order, np.uint8)
    r["brightness"], r["contrast"], r["saturation"], r["hue"] = p.brightness, p.contrast, p.saturation, p.hue
    r["sigma"], r["ksize"] = p.sigma, p.ksize
    r["resize_w"], r["resize_h"], r["out_x"], r["out_y"] = p.resize_w, p.resize_h, p.out_x, p.out_y
    return r


def build_emu() -> ctypes.CDLL:
    src = ROOT / "tests" / "emu" / "emu.cpp"
    deps = [src, ROOT / "tests" / "emu" / "models.hpp", *sorted((ROOT / "dataloader_amd" / "csrc").glob("*.hpp"))]
    if not EMU_SO.exists() or EMU_SO.stat().st_mtime < max(d.stat().st_mtime for d in deps):
        # host-only: the emulator runs the device functions on the CPU (no device pass)
        cmd = (f"hipcc --cuda-host-only -O2 -ffp-contract=off -fPIC -shared -o {EMU_SO} {src}")
        if os.system(cmd) != 0:
            raise RuntimeError(f"emulator build failed: {cmd}")
    return ctypes.CDLL(str(EMU_SO))


def emu_decode(lib, jpeg: bytes, mode: int = 0, lanes: int = 1):
    from PIL import Image
    try:
        w, h = Image.open(io.BytesIO(jpeg)).size
    except Exception:  # noqa: BLE001
        w, h = 1, 1
    out = np.zeros(h * w * 3, np.uint8)
    st = np.zeros(4, np.int32)
    buf = np.frombuffer(jpeg, np.uint8)
    r = lib.emu_decode(buf.ctypes.data_as(P), ctypes.c_int64(len(jpeg)), mode, lanes,
                       out.ctypes.data_as(P), st.ctypes.data_as(P))
    return r, out.reshape(h, w, 3), st


def emu_augment(lib, rgb: np.ndarray, rec, mean, std, out_dtype: int = 0):
    import torch
    H, W, _ = rgb.shape
    S = int(rec["out_size"])
    rgb = np.ascontiguousarray(rgb)
    m = np.asarray(mean, np.float32)
    s = np.asarray(std, np.float32)
    recarr = np.asarray(rec, VIEW_PARAMS_DTYPE).reshape(1)
    if out_dtype == 0:
        out = np.zeros(3 * S * S, np.uint16)
    elif out_dtype == 1:
        out = np.zeros(3 * S * S, np.float32)
    else:
        out = np.zeros(3 * S * S, np.uint8)
    lib.emu_augment_view(rgb.ctypes.data_as(P), W, H, recarr.ctypes.data_as(P), m.ctypes.data_as(P),
                         s.ctypes.data_as(P), out_dtype, out.ctypes.data_as(P))
    t = torch.from_numpy(out.reshape(3, S, S).copy())
    if out_dtype == 0:
        return t.view(torch.bfloat16)
    if out_dtype == 2:
        return t.view(torch.float8_e4m3fn)
    return t


def emu_resized_crop(lib, rgb: np.ndarray, rec) -> np.ndarray:
    H, W, _ = rgb.shape
    S = int(rec["out_size"])
    rgb = np.ascontiguousarray(rgb)
    recarr = np.asarray(rec, VIEW_PARAMS_DTYPE).reshape(1)
    out = np.zeros(S * S * 3, np.uint8)
    lib.emu_resized_crop(rgb.ctypes.data_as(P), W, H, recarr.ctypes.data_as(P), out.ctypes.data_as(P))
    return out.reshape(S, S, 3)


def dc_extremes_rgb(w: int, h: int, rng, cell: int = 16) -> np.ndarray:
    """Saturated colour cells (black/white/blue/yellow/red/cyan) in cell x cell squares:
    neighbouring blocks differ by DC categories 10-11 in luma and chroma, whose chroma
    codes are longer than the DC lookahead (the decoder's slow path)."""
    pal = np.array([[0, 0, 0], [255, 255, 255], [0, 0, 255], [255, 255, 0], [255, 0, 0], [0, 255, 255]], np.uint8)
    idx = rng.integers(0, len(pal), size=((h + cell - 1) // cell, (w + cell - 1) // cell))
    img = pal[np.repeat(np.repeat(idx, cell, axis=0), cell, axis=1)[:h, :w]]
    return np.ascontiguousarray(img)
