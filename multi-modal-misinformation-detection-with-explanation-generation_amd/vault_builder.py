"""Truth-Vault index builder: ``generate_embeddings_database`` (train_clip_detective.py:457-607)
on the HIP CLIP towers, sharded over ranks.

The reference walks the article list one article at a time (processor -> CLIPDetective forward
under fp16 autocast -> L2-normalise both embeddings, train_clip_detective.py:533-566) and pickles
the schema of lines 515-527.  Here:

* every rank takes a contiguous shard of the articles (``sharding.shard_range``), loads its
  images / tokenises its texts on the host and encodes them in batches of ``batch`` through the
  HIP CLIP image and text towers (unit-norm fp32 rows, the l2norm kernel);
* ONE all-gather (``sharding.gather_rows``: RCCL over xGMI when the process group is ``nccl``,
  gloo in the CPU tests) assembles the [N, 512] image / text embedding tables and the per-article
  success flags on every rank -- the only place on this project's path where a collective is
  meaningful (every rank ends with the replicated vault it will search);
* rank 0 writes the reference's pickle schema and ``*_summary.json``; articles whose image or
  text fails to load are skipped with the reference's message, as the reference does.

The encoder is pluggable (``encode``) so the host logic and the collective are testable on CPU
with the oracle as the encoder; the product path passes the HIP engine.
"""
from __future__ import annotations

import json
import os
import pickle
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import io_utils
from .sharding import gather_rows, shard_range

Encoder = Callable[[np.ndarray, np.ndarray, np.ndarray], Tuple[torch.Tensor, torch.Tensor]]


def load_clip_detective_checkpoint(model_path: str) -> Tuple[Dict[str, np.ndarray], Dict]:
    """``torch.load(model_path)['model_state_dict']`` of a CLIPDetective (train_clip_detective.py:
    76-127: the CLIPModel lives under ``clip.``) -> CLIPModel state dict + checkpoint metadata.
    Loaded with ``weights_only=True`` (the reference uses weights_only=False, line 495)."""
    ck = torch.load(model_path, map_location="cpu", weights_only=True)
    sd = ck["model_state_dict"]
    clip_sd = {k[len("clip."):]: v.float().numpy() for k, v in sd.items() if k.startswith("clip.")}
    return clip_sd, {"epoch": ck.get("epoch"), "val_accuracy": ck.get("val_accuracy")}


def engine_encoder(engine) -> Encoder:
    """The HIP CLIP towers of an ``Engine``: uint8 [b,224,224,3] + ids/mask [b,77] -> unit rows."""
    def enc(imgs, ids, mask):
        return engine.clip_image(imgs), engine.clip_text(ids, mask)
    return enc


def _prepare(articles: List[Dict], processor, eos_id: int):
    """Host side of one shard: PIL load + CLIP geometry, tokenisation (truncation=True,
    max_length=77 as train_clip_detective.py:540-547).  Returns pixels, ids, mask, ok flags."""
    n = len(articles)
    px = np.zeros((n, 224, 224, 3), np.uint8)
    seqs, ok = [], np.zeros(n, np.int32)
    for i, a in enumerate(articles):
        try:
            img = io_utils.to_pil(a["image_local_path"])
            seq = io_utils.tokenize_clip(processor, [a["text_content"]], truncation=True)[0][:77]
            px[i] = io_utils.clip_pixels(img)
            seqs.append(seq)
            ok[i] = 1
        except Exception as e:  # noqa: BLE001  (the reference skips the article, lines 568-570)
            print(f"\nError processing {a.get('article_id')}: {e}")
            seqs.append([eos_id])
    if not seqs:
        return px, np.zeros((0, 77), np.int32), np.zeros((0, 77), np.int32), ok
    ids, mask = io_utils.pad_ids(seqs, eos_id, 77)
    return px, ids, mask, ok


def encode_shard(articles: List[Dict], processor, encode: Encoder, eos_id: int = 49407, batch: int = 256,
                 device=None) -> Dict[str, torch.Tensor]:
    """Embeddings of one rank's articles: {"img": [n,512], "txt": [n,512], "ok": [n]}."""
    px, ids, mask, ok = _prepare(articles, processor, eos_id)
    n = len(articles)
    dev = device if device is not None else torch.device("cpu")
    img = torch.zeros((n, 512), dtype=torch.float32, device=dev)
    txt = torch.zeros((n, 512), dtype=torch.float32, device=dev)
    for s in range(0, n, batch):
        e = min(n, s + batch)
        ie, te = encode(px[s:e], ids[s:e], mask[s:e])
        img[s:e] = torch.as_tensor(ie).to(dev, torch.float32)
        txt[s:e] = torch.as_tensor(te).to(dev, torch.float32)
    return {"img": img, "txt": txt, "ok": torch.as_tensor(ok).to(dev)}


def generate_embeddings_database(model_path: str = "clip_detective_best.pth",
                                 json_file: str = "vector_db_seed.json",
                                 output_file: str = "guardian_embeddings.pkl", *,
                                 processor=None, encode: Optional[Encoder] = None, engine=None,
                                 val_accuracy=None, eos_token_id: int = 49407, batch: int = 256,
                                 rank: int = 0, world: int = 1, group=None, device=None) -> Optional[Dict]:
    """train_clip_detective.py:457-607 with the reference's signature and on-disk result.

    Without ``encode``/``engine``: loads ``model_path`` (CLIPDetective checkpoint) into a new HIP
    engine on this rank's device.  ``rank``/``world``/``group``: an initialised torch.distributed
    process group (one process per GPU); world = 1 runs single-process."""
    if processor is None:
        raise RuntimeError("a CLIP processor/tokenizer is required (pass processor=)")
    if not os.path.isabs(model_path):  # train_clip_detective.py:476-477 (stored in the metadata)
        model_path = os.path.join(os.getcwd(), model_path)
    if encode is None:
        if engine is None:
            from .engine import Engine
            if not os.path.exists(model_path):
                print(f"\n✗ Error: Model checkpoint not found at: {model_path}")
                return None
            clip_sd, meta = load_clip_detective_checkpoint(model_path)
            val_accuracy = meta.get("val_accuracy", val_accuracy)
            engine = Engine(torch.cuda.current_device(), None, clip_sd, eos_token_id=eos_token_id, max_batch=batch)
        encode = engine_encoder(engine)
        device = device if device is not None else engine.device
    with open(json_file, "r", encoding="utf-8") as f:
        articles = json.load(f)
    N = len(articles)
    s, e = shard_range(N, rank, world)
    local = encode_shard(articles[s:e], processor, encode, eos_token_id, batch, device)
    full = gather_rows(local, N, group) if world > 1 else local
    ok = full["ok"].cpu().numpy().astype(bool)
    img = full["img"].cpu().numpy()[ok]
    txt = full["txt"].cpu().numpy()[ok]
    # the reference normalises once more on the host (lines 558-560): unit rows stay unit
    if len(img):
        img = img / np.linalg.norm(img, axis=1, keepdims=True)
        txt = txt / np.linalg.norm(txt, axis=1, keepdims=True)
    kept = [a for a, k in zip(articles, ok) if k]
    db = {
        "article_ids": [a["article_id"] for a in kept],
        "text_contents": [a["text_content"] for a in kept],
        "image_paths": [a["image_local_path"] for a in kept],
        "image_embeddings": img.astype(np.float32),
        "text_embeddings": txt.astype(np.float32),
        "metadata": {"model_path": model_path, "total_articles": N,
                     "embedding_dim": int(img.shape[1]) if len(img) else None,
                     "val_accuracy": val_accuracy},
    }
    if rank == 0:
        with open(output_file, "wb") as f:
            pickle.dump(db, f)
        summary = {"total_articles": len(db["article_ids"]), "embedding_dimension": db["metadata"]["embedding_dim"],
                   "model_val_accuracy": val_accuracy, "database_size_mb": os.path.getsize(output_file) / 1e6,
                   "sample_articles": db["article_ids"][:5]}
        with open(output_file.replace(".pkl", "_summary.json"), "w", encoding="utf-8") as f:
            json.dump(summary, f, indent=2)
    return db
