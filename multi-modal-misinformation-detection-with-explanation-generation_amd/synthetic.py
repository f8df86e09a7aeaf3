"""Seeded synthetic inputs of the shapes the hot path consumes.

* RoBERTa token ids int32 ``[B, L]``: ``<s>``=0 at position 0, body uniform in
  ``[3, 50264]``, ``</s>``=2 at ``len-1``, pad id 1 (mask 0) after.
* CLIP token ids int32 ``[B, 77]``: BOS 49406 at 0, body uniform in ``[0, 49405]``,
  EOS 49407 at ``len-1``, padded with 49407 (mask 0).  With these ids both HF EOS-pooling
  rules (``argmax`` / first ``eos_token_id``) pick ``len-1``.
* Images uint8 ``[B, 224, 224, 3]`` (HWC, RGB) uniform 0..255.
* Truth-Vault ``[N, 512]`` fp32 N(0,1) rows (the reference normalises rows itself,
  misinfo_forensics.py:443-445).
* FusionJudge inputs ``[B, 5]`` (config 1).

Tokenisation and JPEG decode are outside the timed path.
"""
from __future__ import annotations

import numpy as np

from .weights import CLIP_TEXT

ROBERTA_MAX_BODY = 50264


def _rng(seed: int, tag: str) -> np.random.Generator:
    import zlib
    return np.random.Generator(np.random.PCG64((int(seed) * 1000003 ^ zlib.crc32(tag.encode())) & 0xFFFFFFFFFFFF))


def roberta_ids(batch: int, seq_len: int = 128, seed: int = 1234, lengths=None):
    g = _rng(seed, "roberta_ids")
    ids = np.full((batch, seq_len), 1, dtype=np.int32)
    mask = np.zeros((batch, seq_len), dtype=np.int32)
    if lengths is None:
        lengths = [seq_len] * batch
    for i in range(batch):
        n = int(min(max(lengths[i % len(lengths)], 2), seq_len))
        ids[i, 0] = 0
        ids[i, 1:n - 1] = g.integers(3, ROBERTA_MAX_BODY + 1, size=n - 2)
        ids[i, n - 1] = 2
        mask[i, :n] = 1
    return ids, mask


def clip_ids(batch: int, seq_len: int = 77, seed: int = 1234, lengths=None):
    g = _rng(seed, "clip_ids")
    eos, bos = CLIP_TEXT["eos_id"], CLIP_TEXT["bos_id"]
    ids = np.full((batch, seq_len), eos, dtype=np.int32)
    mask = np.zeros((batch, seq_len), dtype=np.int32)
    if lengths is None:
        lengths = [seq_len] * batch
    for i in range(batch):
        n = int(min(max(lengths[i % len(lengths)], 2), seq_len))
        ids[i, 0] = bos
        ids[i, 1:n - 1] = g.integers(0, bos, size=n - 2)
        ids[i, n - 1] = eos
        mask[i, :n] = 1
    return ids, mask


def images(batch: int, seed: int = 1234, size: int = 224, structured: bool = True) -> np.ndarray:
    """uint8 [B, size, size, 3].  ``structured`` images (per-image colour, gradient, sinusoid
    and noise level) give random-init encoders input-dependent outputs; uniform noise images
    all share the same global statistics and collapse to nearly one embedding."""
    g = _rng(seed, "images")
    if not structured:
        return g.integers(0, 256, size=(batch, size, size, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32) / float(size - 1)
    out = np.empty((batch, size, size, 3), np.uint8)
    for i in range(batch):
        base = g.uniform(0, 255, 3).astype(np.float32)
        gx, gy = g.uniform(-120, 120, 3).astype(np.float32), g.uniform(-120, 120, 3).astype(np.float32)
        fr, amp = np.float32(g.uniform(2, 12)), np.float32(g.uniform(0, 80))
        ph = g.uniform(0, 6.28, 3).astype(np.float32)
        img = base + gx * xx[..., None] + gy * yy[..., None] \
            + amp * np.sin(fr * (xx + yy)[..., None] * np.float32(3.14159) + ph)
        img += g.normal(0, g.uniform(5, 60), (size, size, 3)).astype(np.float32)
        out[i] = np.clip(img, 0, 255).astype(np.uint8)
    return out


def vault(n: int = 2170, dim: int = 512, seed: int = 77) -> np.ndarray:
    g = _rng(seed, "vault")
    return g.standard_normal((n, dim), dtype=np.float32)


def fusion_inputs(batch: int = 1024, seed: int = 1234) -> np.ndarray:
    """Config 1 inputs: ai/misinfo/deepfake ~U[0,1], clip_sim ~U[-0.2,0.5], vault in {0} U U[0.86,1]."""
    g = _rng(seed, "fusion")
    x = np.empty((batch, 5), dtype=np.float32)
    x[:, 0:3] = g.uniform(0, 1, (batch, 3))
    x[:, 3] = g.uniform(-0.2, 0.5, batch)
    hit = g.uniform(0, 1, batch) < 0.25
    x[:, 4] = np.where(hit, g.uniform(0.86, 1.0, batch), 0.0)
    return x
