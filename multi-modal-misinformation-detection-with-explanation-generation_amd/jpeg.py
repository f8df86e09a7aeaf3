"""Device JPEG decode for the host input stage.

The reference decodes every image with `Image.open(path).convert("RGB")`
(misinfo_forensics.py:255-258) -- Pillow's libjpeg-turbo on one host core.  Here the only serial
part, marker parsing + Huffman entropy decoding, runs in C on the host threads
(csrc/jpeg_host.cpp: mmf_jpeg_header / mmf_jpeg_entropy_packed, called through ctypes, which releases
the GIL); the quantised coefficients are packed sparse (per block a mask of the nonzero zigzag
positions + their values: ~0.35 MB for a 640x480 q90 photo instead of 0.92 MB of dense planes) into
a pinned staging buffer, one H2D copy moves them, and the device reconstructs the pixels (csrc/jpeg.hip: islow IDCT, fancy chroma upsampling, YCbCr -> RGB,
bit-exact with Pillow) as RGBX images that feed the Pillow-exact resampler (mmf_resize_pil).
Progressive files are decoded scan by scan into the same coefficients.  Files the C decoder does
not take (CMYK, 4:4:0, lossless / arithmetic / 12-bit, RGB-id files, files whose data ends before
the EOI marker, ...) report MMF_EUNSUPPORTED and are decoded by Pillow on the host, as before (so a
truncated file raises Pillow's "image file is truncated", as in the reference); so are images past
the device resampler's tap budget.
"""
from __future__ import annotations

import ctypes
import os
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np
import torch

from . import hip

INFO_LEN = 16
MMF_EUNSUPPORTED = -95
MMF_ERANGE = -34


def read_bytes(item) -> Optional[bytes]:
    """Encoded bytes of an image argument (bytes, or a path to a file), None for anything else
    (PIL images, arrays): those keep the Pillow path."""
    if isinstance(item, (bytes, bytearray, memoryview)):
        return bytes(item)
    if isinstance(item, (str, os.PathLike)) and os.path.isfile(item):
        with open(item, "rb") as f:
            return f.read()
    return None


def _align(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


class Staged:
    """One chunk's entropy-decoded JPEGs in a pinned buffer: which inputs, their header infos and
    the byte layout of the buffer (tables | infos | block bases | RGBX offsets | record offsets |
    block-record offsets | packed records)."""

    def __init__(self):
        self.index: List[int] = []  # positions (within the chunk) decoded by the device path
        self.infos = None
        self.slot = 0
        self.nbytes = 0
        self.sections = {}
        self.blocks = self.pixels = 0
        self.max_blocks = self.max_pixels = 0


class JpegStager:
    """Host half: headers + entropy decoding of a chunk into one of two pinned buffers (the other
    may still be feeding the previous chunk's H2D copy: each slot's copy is fenced by an event)."""

    guess_bytes_per_block = 64  # first sizing of a slot's packed section (grown when a chunk needs more)

    def __init__(self, workers: Optional[int] = None):
        self.lib = hip.load()
        self.workers = workers or min(16, len(os.sched_getaffinity(0)))
        self.buf = [None, None]
        self.copied = [None, None]  # torch.cuda.Event recorded after the H2D copy of each slot
        self.next_slot = 0
        self._pool = ThreadPoolExecutor(max_workers=self.workers)
        # decode a chunk in one C call on the library's threads (MMF_JPEG_BATCH=0: per file on the pool)
        self.batch_call = os.environ.get("MMF_JPEG_BATCH", "1") != "0"

    def close(self):
        self._pool.shutdown(wait=False)

    def stage(self, datas: List[Optional[bytes]]) -> Staged:
        st = Staged()
        lib = self.lib

        m = len(datas)
        if m == 0:
            return st
        hptrs = (ctypes.c_char_p * m)(*datas)  # None -> NULL: declined
        hlens = np.array([len(d) if d is not None else 0 for d in datas], np.int64)
        allinf = np.zeros((m, INFO_LEN), np.int32)
        hrc = np.zeros(m, np.int32)
        hip.check(lib.mmf_jpeg_header_batch(ctypes.cast(hptrs, ctypes.c_void_p), hlens.ctypes.data, m,
                                            allinf.ctypes.data, hrc.ctypes.data, self.workers), "mmf_jpeg_header_batch")
        ok = hrc == 0
        # images past mmf_resize_pil's tap budget (shortest side above ~5264 px) are decoded and
        # resampled by Pillow on the host (api._resize), like every other declined file
        for i in np.flatnonzero(ok):
            if not lib.mmf_resize_supported(int(allinf[i, 0]), int(allinf[i, 1])):
                ok[i] = False
        st.index = np.flatnonzero(ok).tolist()
        n = len(st.index)
        if n == 0:
            return st
        inf = np.ascontiguousarray(allinf[st.index])
        blocks = inf[:, 11].astype(np.int64)
        pixels = inf[:, 0].astype(np.int64) * inf[:, 1]
        coef_blocks = np.zeros(n, np.int64)
        coef_blocks[1:] = np.cumsum(blocks)[:-1]
        out_off = np.zeros(n, np.int64)
        out_off[1:] = np.cumsum(pixels * 4)[:-1]
        st.blocks, st.pixels = int(blocks.sum()), int(pixels.sum())
        st.max_blocks, st.max_pixels = int(blocks.max()), int(pixels.max())
        sec = {}
        off = 0
        for name, size in (("qt", n * 192 * 2), ("infos", n * INFO_LEN * 4), ("coef_blocks", n * 8),
                           ("out_off", n * 8), ("pk_off", n * 8), ("block_off", st.blocks * 4)):
            sec[name] = off
            off = _align(off + size)
        sec["packed"] = off
        st.sections, st.infos = sec, inf
        st.out_off = out_off
        slot = self.next_slot
        self.next_slot ^= 1
        st.slot = slot
        if self.copied[slot] is not None:
            self.copied[slot].synchronize()  # the previous H2D from this slot has finished
        # the packed records' size is known only after decoding: start from ~half the dense size
        guess = off + st.blocks * self.guess_bytes_per_block
        if self.buf[slot] is None or self.buf[slot].numel() < guess:
            self.buf[slot] = torch.empty(max(guess, 1 << 16) * 5 // 4, dtype=torch.uint8).pin_memory()
        host = self.buf[slot].numpy()
        host[sec["infos"]:sec["infos"] + n * INFO_LEN * 4] = inf.view(np.uint8).reshape(-1)
        host[sec["coef_blocks"]:sec["coef_blocks"] + n * 8] = coef_blocks.view(np.uint8)
        host[sec["out_off"]:sec["out_off"] + n * 8] = out_off.view(np.uint8)
        pk_off = np.zeros(n, np.int64)
        cursor = np.zeros(1, np.int64)
        b = host.ctypes.data
        dst, cap, cur = b + sec["packed"], self.buf[slot].numel() - sec["packed"], cursor.ctypes.data
        boff, qt, po = b + sec["block_off"], b + sec["qt"], pk_off.ctypes.data
        idx = st.index

        if self.batch_call:  # one C call for the chunk (GIL released; the library's own threads)
            ds = [datas[i] for i in idx]
            ptrs = (ctypes.c_char_p * n)(*ds)
            lens = np.array([len(d) for d in ds], np.int64)
            rcs_a = np.zeros(n, np.int32)
            hip.check(lib.mmf_jpeg_stage_packed_batch(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, dst,
                                                      cap, cur, boff, coef_blocks.ctypes.data, qt, po, self.workers,
                                                      rcs_a.ctypes.data), "mmf_jpeg_stage_packed_batch")
        else:  # one C call per file on the Python pool
            def entropy(k):
                d = datas[idx[k]]
                return lib.mmf_jpeg_stage_packed(d, len(d), dst, cap, cur, boff + int(coef_blocks[k]) * 4,
                                                 qt + k * 384, po + k * 8)
            rcs_a = np.array(list(self._pool.map(entropy, range(n))) if n > 1 else [entropy(0)], np.int32)
        rcs = rcs_a.tolist()
        overflow = [k for k, rc in enumerate(rcs) if rc == MMF_ERANGE]
        bad = [k for k, rc in enumerate(rcs) if rc not in (0, MMF_ERANGE)]
        if bad:  # (a header that parsed but a scan that did not: never seen; decode those on the host)
            raise hip.MMFError(f"mmf_jpeg_stage_packed failed for chunk positions {[st.index[k] for k in bad]}")
        total = sec["packed"] + int(cursor[0])
        if overflow:  # grow the slot, keep what was written, then place the records that did not fit
            old = self.buf[slot]
            keep = sec["packed"] + cap
            self.buf[slot] = torch.empty(total * 5 // 4, dtype=torch.uint8).pin_memory()
            host = self.buf[slot].numpy()
            host[:keep] = old.numpy()[:keep]
            b = host.ctypes.data
            for k in overflow:
                d = datas[idx[k]]
                used = ctypes.c_int64(0)
                scratch = np.empty(int(lib.mmf_jpeg_packed_bound(int(blocks[k]))), np.uint8)
                hip.check(lib.mmf_jpeg_entropy_packed(d, len(d), scratch.ctypes.data, scratch.size,
                                                      b + sec["block_off"] + int(coef_blocks[k]) * 4,
                                                      b + sec["qt"] + k * 384, ctypes.byref(used)),
                          "mmf_jpeg_entropy_packed")
                o = sec["packed"] + int(pk_off[k])
                host[o:o + used.value] = scratch[:used.value]
        host[sec["pk_off"]:sec["pk_off"] + n * 8] = pk_off.view(np.uint8)
        st.nbytes = total
        return st


def _reconstruct(lib, h, p, st: Staged, samples: int, rgbx: int) -> int:
    sec = st.sections
    return lib.mmf_jpeg_reconstruct(h, p + sec["packed"], p + sec["block_off"], p + sec["pk_off"], p + sec["qt"],
                                    p + sec["coef_blocks"], p + sec["infos"], p + sec["out_off"], len(st.index),
                                    st.max_blocks, st.max_pixels, samples, rgbx, hip.stream_ptr())


def device_windows(engine, stager: JpegStager, st: Staged):
    """Device half: H2D of the staged coefficients, reconstruction to RGBX, both towers' 224x224
    windows (Pillow-exact) -> (eff, clp) uint8 [n,224,224,3] device tensors for st.index."""
    lib, dev = engine.lib, engine.device
    n = len(st.index)
    src = stager.buf[st.slot][:st.nbytes].to(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    stager.copied[st.slot] = ev
    p = src.data_ptr()
    need = st.pixels * 4 + st.blocks * 64
    if getattr(engine, "_jpeg_dev", None) is None or engine._jpeg_dev.numel() < need:
        engine._jpeg_dev = torch.empty(need * 5 // 4, dtype=torch.uint8, device=dev)
    rgbx = engine._jpeg_dev.data_ptr()
    samples = rgbx + st.pixels * 4
    hip.check(_reconstruct(lib, engine.h, p, st, samples, rgbx), "mmf_jpeg_reconstruct")
    wh = np.ascontiguousarray(st.infos[:, :2]).reshape(-1)
    eff = torch.empty((n, 224, 224, 3), dtype=torch.uint8, device=dev)
    clp = torch.empty((n, 224, 224, 3), dtype=torch.uint8, device=dev)
    hip.check(lib.mmf_resize_pil(engine.h, rgbx, st.out_off.ctypes.data_as(ctypes.c_void_p),
                                 wh.ctypes.data_as(ctypes.c_void_p), n, 4, hip.ptr(eff), hip.ptr(clp),
                                 hip.stream_ptr()), "mmf_resize_pil")
    return eff, clp


def device_rgb(engine, stager: JpegStager, st: Staged) -> List[np.ndarray]:
    """Decoded pixels only (tests / tools): [h][w][3] uint8 host arrays for st.index."""
    dev = engine.device
    src = stager.buf[st.slot][:st.nbytes].to(dev)
    p = src.data_ptr()
    n = len(st.index)
    out = torch.empty(st.pixels * 4 + st.blocks * 64, dtype=torch.uint8, device=dev)
    hip.check(_reconstruct(engine.lib, engine.h, p, st, out.data_ptr() + st.pixels * 4, out.data_ptr()),
              "mmf_jpeg_reconstruct")
    host = out[:st.pixels * 4].cpu().numpy()
    res = []
    for k in range(n):
        w, h = int(st.infos[k, 0]), int(st.infos[k, 1])
        o = int(st.out_off[k])
        res.append(host[o:o + w * h * 4].reshape(h, w, 4)[..., :3].copy())
    return res
