"""JPEG test inputs shared by tests/test_jpeg_cpu.py and tests/test_gpu_jpeg.py: encoded in the test
run by Pillow's encoder (deterministic), covering the decoder paths -- 4:2:0 / 4:2:2 / 4:4:4 /
grayscale, odd sizes and 1x1, optimised Huffman tables, restart intervals (per blocks and per MCU
rows), low and high quality, progressive files -- plus files the device path must hand back to
Pillow."""
import io

import numpy as np
from PIL import Image


def photo_like(w, h, seed=0):
    """Smooth gradients + texture + noise: coefficient statistics of a photo, not of white noise."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 3 + yy) % 256, (yy * 2 + 40) % 256, ((xx + yy) * 5) % 256], -1).astype(np.float64)
    tex = 40 * np.sin(xx[..., None] / 3.0 + np.array([0, 1, 2])) * np.cos(yy[..., None] / 5.0)
    a = base * 0.75 + tex + rng.normal(0, 12, (h, w, 3))
    return np.clip(a, 0, 255).astype(np.uint8)


def encode(a, mode="RGB", **kw):
    im = Image.fromarray(a)
    if mode != "RGB":
        im = im.convert(mode)
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


# (w, h, mode, save kwargs)
SUPPORTED = [
    (64, 48, "RGB", dict(quality=90, subsampling=2)),
    (65, 49, "RGB", dict(quality=75, subsampling=2)),
    (33, 17, "RGB", dict(quality=95, subsampling=1)),
    (40, 40, "RGB", dict(quality=50, subsampling=0)),
    (31, 23, "L", dict(quality=80)),
    (97, 61, "RGB", dict(quality=85, subsampling=2, optimize=True)),
    (8, 8, "RGB", dict(quality=100, subsampling=2)),
    (1, 1, "RGB", dict(quality=90)),
    (3, 5, "RGB", dict(quality=10, subsampling=2)),
    (300, 200, "RGB", dict(quality=90, subsampling=2, restart_marker_blocks=7)),
    (301, 203, "RGB", dict(quality=70, subsampling=1, restart_marker_rows=1)),
    (70, 50, "L", dict(quality=60, restart_marker_blocks=3)),
    (127, 129, "RGB", dict(quality=98, subsampling=0, optimize=True)),
]
LARGE = [(640, 480, "RGB", dict(quality=90, subsampling=2)), (1023, 767, "RGB", dict(quality=80, subsampling=1))]


# progressive (SOF2): Pillow's scan script has DC first / refine and AC first / refine scans with
# successive approximation, optimised tables per scan (DHT between scans)
PROGRESSIVE = [(w, h, m, dict(kw, progressive=True)) for w, h, m, kw in (
    (64, 48, "RGB", dict(quality=90, subsampling=2)),
    (65, 49, "RGB", dict(quality=75, subsampling=2)),
    (33, 17, "RGB", dict(quality=95, subsampling=1)),
    (40, 40, "RGB", dict(quality=50, subsampling=0)),
    (31, 23, "L", dict(quality=80)),
    (1, 1, "RGB", dict(quality=90)),
    (300, 200, "RGB", dict(quality=90, subsampling=2, restart_marker_blocks=7)),
    (127, 129, "RGB", dict(quality=98, subsampling=0)),
)]
LARGE_PROGRESSIVE = [(640, 480, "RGB", dict(quality=90, subsampling=2, progressive=True))]


def _cases(cases):
    return [(f"{w}x{h}-{m}-{kw}", encode(photo_like(w, h, seed=w * 31 + h), m, **kw)) for w, h, m, kw in cases]


def supported_jpegs(large=False, progressive=False):
    cases = SUPPORTED + (LARGE if large else [])
    if progressive:
        cases = cases + PROGRESSIVE + (LARGE_PROGRESSIVE if large else [])
    return _cases(cases)


def progressive_pairs():
    """(name, progressive file, sequential file of the same pixels and settings): the quantised
    coefficients of the two are the same (progression only changes the entropy coding)."""
    out = []
    for w, h, m, kw in PROGRESSIVE:
        a = photo_like(w, h, seed=w * 31 + h)
        seq = {k: v for k, v in kw.items() if k != "progressive"}
        out.append((f"{w}x{h}-{m}-{kw}", encode(a, m, **kw), encode(a, m, **seq)))
    return out


def unsupported_files():
    """Files the device path declines (MMF_EUNSUPPORTED or not JPEG): Pillow decodes them."""
    a = photo_like(48, 40, seed=5)
    seq = bytearray(encode(a, quality=90))
    i = seq.index(b"\xff\xc0")
    seq[i + 1] = 0xC3  # the same file relabelled lossless (SOF3)
    out = [("lossless", bytes(seq)),
           ("cmyk", encode(a, "CMYK", quality=90))]
    b = io.BytesIO()
    Image.fromarray(a).save(b, "PNG")
    out.append(("png", b.getvalue()))
    return out


def _segments(d: bytes):
    """(marker, start, end) of each marker segment before the first SOS's entropy data."""
    out, p = [], 2
    while p + 4 <= len(d):
        m = d[p + 1]
        L = (d[p + 2] << 8) | d[p + 3]
        out.append((m, p, p + 2 + L))
        if m == 0xDA:
            break
        p += 2 + L
    return out


def rgb_component_ids() -> bytes:
    """A 3-component file with no JFIF / Adobe marker whose component ids are 'R' 'G' 'B':
    libjpeg (default_decompress_parms) decodes it as RGB, without the YCbCr transform."""
    d = bytearray(encode(photo_like(40, 32, seed=9), quality=90, subsampling=0))
    segs = _segments(bytes(d))
    for m, a, b in segs:
        if m in (0xC0, 0xDA):
            ids = [a + 10 + 3 * i for i in range(3)] if m == 0xC0 else [a + 5 + 2 * i for i in range(3)]
            for k, i in enumerate(ids):
                d[i] = (82, 71, 66)[k]
    app0 = [(a, b) for m, a, b in segs if m == 0xE0]
    for a, b in reversed(app0):
        del d[a:b]
    return bytes(d)


def duplicate_sos_ids() -> bytes:
    """SOF ids 1, 2, 3 but SOS ids 1, 1, 1 (libjpeg: JERR_BAD_COMPONENT_ID)."""
    d = bytearray(encode(photo_like(32, 24, seed=4), quality=90))
    for m, a, b in _segments(bytes(d)):
        if m == 0xDA:
            for i in range(3):
                d[a + 5 + 2 * i] = 1
    return bytes(d)


def short_sos_at_eof() -> bytes:
    """A file ending in an SOS segment whose length field claims only the length itself (L = 2)."""
    d = encode(photo_like(16, 16, seed=2), quality=90)
    sos = [a for m, a, b in _segments(d) if m == 0xDA][0]
    return d[:sos] + b"\xff\xda\x00\x02"


def pillow_rgb(data: bytes) -> np.ndarray:
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
