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


class IdTableTokenizer:
    """Tokenizer-call interface over a {text: token-id list} table (the vocab files are absent):
    RoBERTa's call of misinfo_forensics.py:327-333 (``max_length`` truncation) and the CLIP
    processor's text call of :386-391 / :473-478 (``truncation`` at 77); right padding with
    ``pad_id``.  Used by the per-sample bench lines, which time the API around a tokenizer."""

    def __init__(self, table, pad_id: int, clip: bool = False):
        self.table, self.pad_id, self.clip = table, pad_id, clip

    def __call__(self, text=None, images=None, return_tensors="pt", max_length=512, truncation=False,
                 padding=True):
        import torch
        texts = [text] if isinstance(text, str) else list(text)
        cap = 77 if self.clip else max_length
        seqs = [list(self.table[s])[:cap] if truncation else list(self.table[s]) for s in texts]
        L = max(len(s) for s in seqs)
        ids = torch.full((len(seqs), L), self.pad_id, dtype=torch.long)
        mask = torch.zeros((len(seqs), L), dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.tensor(s)
            mask[i, :len(s)] = 1
        return {"input_ids": ids, "attention_mask": mask}


def text_tables(n: int, seed: int = 1234, rob_len: int = 128, clip_len: int = 77):
    """n texts "pair i" -> (RoBERTa ids of ``rob_len`` tokens, CLIP ids of ``clip_len`` tokens),
    the same ids the batched bench uses for the same seed."""
    rid, _ = roberta_ids(n, rob_len, seed)
    cid, _ = clip_ids(n, clip_len, seed)
    texts = [f"pair {i}" for i in range(n)]
    rob = {t: rid[i].tolist() for i, t in enumerate(texts)}
    clp = {t: cid[i].tolist() for i, t in enumerate(texts)}
    return texts, IdTableTokenizer(rob, 1), IdTableTokenizer(clp, CLIP_TEXT["eos_id"], clip=True)
