"""Test infrastructure only (never imported by the product path): a numpy restatement of Pillow's
8-bit resampler (Pillow 12.2, src/libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc,
ImagingResampleHorizontal_8bpc / ImagingResampleVertical_8bpc, the bilinear and bicubic (a = -0.5)
filters) -- the operation behind the reference's image preprocessing (torchvision Resize on a PIL
image, misinfo_forensics.py:249-253, and CLIPImageProcessor's PIL resize).  Pinned against Pillow
itself, run in this container (tests/test_pil_resample_cpu.py: bit-exact on every case); the device
resampler (csrc/resize.hip) is checked against both.
"""
import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bilinear(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def _bicubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


FILTERS = {"bilinear": (_bilinear, 1.0), "bicubic": (_bicubic, 2.0)}


def coeffs(in_size: int, out_size: int, name: str):
    """Per output coordinate: (xmin, n) and n fixed-point weights (precompute_coeffs +
    normalize_coeffs_8bpc)."""
    f, sup = FILTERS[name]
    scale = float(in_size) / out_size
    fs = max(scale, 1.0)
    support = sup * fs
    ksize = int(math.ceil(support)) * 2 + 1
    bounds, kk = [], np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / fs
        xmin = max(int(center - support + 0.5), 0)
        n = min(int(center + support + 0.5), in_size) - xmin
        w = [f((x + xmin - center + 0.5) * ss) for x in range(n)]
        ww = 0.0
        for v in w:
            ww += v
        for x, v in enumerate(w):
            v = v / ww if ww != 0.0 else v
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds.append((xmin, n))
    return bounds, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize(img: np.ndarray, out_w: int, out_h: int, name: str) -> np.ndarray:
    """Image.resize((out_w, out_h), BILINEAR | BICUBIC) of a uint8 HxWxC array."""
    h, w, c = img.shape
    if (out_w, out_h) == (w, h):
        return img.copy()
    bh, kh = coeffs(w, out_w, name)
    bv, kv = coeffs(h, out_h, name)
    if out_w != w:  # horizontal pass over the rows the vertical pass reads
        y0, y1 = bv[0][0], bv[-1][0] + bv[-1][1]
        src = img.astype(np.int64)
        tmp = np.empty((y1 - y0, out_w, c), np.uint8)
        for xx in range(out_w):
            xmin, n = bh[xx]
            acc = np.full((y1 - y0, c), 1 << (PRECISION_BITS - 1), np.int64)
            for x in range(n):
                acc += src[y0:y1, xmin + x, :] * kh[xx, x]
            tmp[:, xx, :] = _clip8(acc)
        bv = [(a - y0, b) for a, b in bv]
    else:
        tmp = img
    if out_h == h:
        return tmp
    t = tmp.astype(np.int64)
    out = np.empty((out_h, tmp.shape[1], c), np.uint8)
    for yy in range(out_h):
        ymin, n = bv[yy]
        acc = np.full((tmp.shape[1], c), 1 << (PRECISION_BITS - 1), np.int64)
        for y in range(n):
            acc += t[ymin + y] * kv[yy, y]
        out[yy] = _clip8(acc)
    return out


def effnet_window(img: np.ndarray) -> np.ndarray:
    """misinfo_forensics.py:249-253 geometry: Resize((224, 224)) bilinear."""
    return resize(img, 224, 224, "bilinear")


def clip_window(img: np.ndarray) -> np.ndarray:
    """CLIPImageProcessor geometry: shortest edge -> 224 bicubic, centre crop 224."""
    h, w = img.shape[:2]
    if (w, h) == (224, 224):
        return img.copy()
    short, long_ = (w, h) if w <= h else (h, w)
    nl = int(224 * long_ / short)
    nw, nh = (224, nl) if w <= h else (nl, 224)
    r = resize(img, nw, nh, "bicubic")
    top, left = (nh - 224) // 2, (nw - 224) // 2
    return r[top:top + 224, left:left + 224]
