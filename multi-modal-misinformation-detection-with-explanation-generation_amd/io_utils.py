"""Host-side input handling for the drop-in API: image loading/geometry, tokenisation calls and the
Truth-Vault file format.  Arithmetic (normalisation, every model) stays on the GPU: images cross
the boundary as uint8 HWC pixels, text as int32 token ids.
"""
from __future__ import annotations

import io
import os
import pickle
from typing import List, Optional, Tuple, Union

import numpy as np

try:
    from PIL import Image
except Exception:  # noqa: BLE001
    Image = None


def to_pil(image_or_path):
    """misinfo_forensics.py:255-258 (_to_pil_image)."""
    if Image is not None and isinstance(image_or_path, Image.Image):
        return image_or_path.convert("RGB")
    return Image.open(str(image_or_path)).convert("RGB")


def effnet_pixels(img) -> np.ndarray:
    """EfficientNet geometry (misinfo_forensics.py:249-253): Resize((224, 224)) bilinear on the PIL
    image (torchvision's PIL path); ToTensor/Normalize happen in the stem kernel."""
    if img.size != (224, 224):
        img = img.resize((224, 224), Image.BILINEAR)
    return np.asarray(img, dtype=np.uint8)


def clip_pixels(img) -> np.ndarray:
    """CLIPImageProcessor geometry: shortest edge -> 224 (bicubic), centre crop 224x224.  Rescale and
    the OpenAI mean/std normalisation happen in the patch-embedding kernel."""
    w, h = img.size
    if (w, h) != (224, 224):
        short, long_ = (w, h) if w <= h else (h, w)
        new_long = int(224 * long_ / short)
        nw, nh = (224, new_long) if w <= h else (new_long, 224)
        img = img.resize((nw, nh), Image.BICUBIC)
        top, left = (nh - 224) // 2, (nw - 224) // 2
        img = img.crop((left, top, left + 224, top + 224))
    return np.asarray(img, dtype=np.uint8)


def _open(item):
    return to_pil(Image.open(io.BytesIO(item)) if isinstance(item, (bytes, bytearray)) else item)


def _decode_one(args):
    i, item, eff, clp = args
    pil = _open(item)
    eff[i] = effnet_pixels(pil)
    clp[i] = clip_pixels(pil)


def _rgbx_view(pil):
    """Pillow keeps RGB pixels as 4 bytes (RGBX); its Arrow export (Pillow >= 11.2) hands that
    memory over without a copy, which np.asarray (a GIL-held tobytes copy) does not."""
    try:
        import pyarrow as pa
        buf = pa.array(pil).buffers()[-1]
        w, h = pil.size
        if buf is not None and buf.size == w * h * 4:
            return np.frombuffer(buf, np.uint8).reshape(h, w, 4)
    except Exception:  # noqa: BLE001 - no pyarrow / no Arrow export: the copying path below
        pass
    return None


def decode_rgb(images, workers: Optional[int] = None) -> List[np.ndarray]:
    """Decode only (threaded) -> uint8 HxWx4 RGBX views of Pillow's own pixel memory when the
    Arrow export is available (else HxWx3 RGB copies); the resampling to both towers' windows then
    runs on the device (Engine.resize_images, Pillow-exact).  All arrays returned are of one kind."""
    if workers is None:
        workers = min(len(images), len(os.sched_getaffinity(0)), 16)

    def one(item):
        pil = _open(item)
        pil.load()
        v = _rgbx_view(pil)
        return (v, pil) if v is not None else (np.asarray(pil, dtype=np.uint8), pil)
    if workers <= 1 or len(images) <= 1:
        res = [one(x) for x in images]
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=workers) as ex:
            res = list(ex.map(one, images))
    if len({a.shape[2] for a, _ in res}) > 1:  # mixed kinds: fall back to RGB copies for all
        return [np.asarray(p, dtype=np.uint8) for _, p in res]
    return [a for a, _ in res]


def decode_batch(images, workers: Optional[int] = None, out: Optional[Tuple[np.ndarray, np.ndarray]] = None):
    """Host input stage of a batch: each image (path, PIL image or encoded bytes) is
    decoded once and resampled to both towers' geometries -- EfficientNet's squash-resize and CLIP's
    shortest-edge resize + centre crop -- straight into uint8 [B,224,224,3] arrays (e.g. pinned
    staging buffers passed as `out`).  Pillow's decoders and resamplers release the GIL, so a thread
    pool scales over the host cores; results equal the serial per-image path bit for bit."""
    n = len(images)
    eff, clp = out if out is not None else (np.empty((n, 224, 224, 3), np.uint8), np.empty((n, 224, 224, 3), np.uint8))
    if workers is None:
        workers = min(n, len(os.sched_getaffinity(0)), 16)
    jobs = [(i, im, eff, clp) for i, im in enumerate(images)]
    if workers <= 1 or n <= 1:
        for j in jobs:
            _decode_one(j)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=workers) as ex:
            list(ex.map(_decode_one, jobs))
    return eff, clp


def pad_ids(seqs: List[List[int]], pad_id: int, length: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    L = length or max(len(s) for s in seqs)
    ids = np.full((len(seqs), L), pad_id, dtype=np.int32)
    mask = np.zeros((len(seqs), L), dtype=np.int32)
    for i, s in enumerate(seqs):
        n = min(len(s), L)
        ids[i, :n] = s[:n]
        mask[i, :n] = 1
    return ids, mask


def _to_list(x):
    if hasattr(x, "tolist"):
        x = x.tolist()
    return [int(v) for v in x]


def tokenize_roberta(tok, text: str) -> List[int]:
    """analyze_text tokenisation (misinfo_forensics.py:327-333)."""
    enc = tok(text, return_tensors="pt", max_length=512, truncation=True, padding=True)
    ids = enc["input_ids"]
    if (hasattr(ids, "dim") and ids.dim() == 2) or (isinstance(ids, (list, tuple)) and isinstance(ids[0], (list, tuple))):
        ids = ids[0]
    return _to_list(ids)


def tokenize_roberta_batch(tok, texts: List[str]) -> List[List[int]]:
    """tokenize_roberta for many texts in one tokenizer call (fast tokenizers encode the batch in
    parallel); each text is encoded independently and right padding only appends, so stripping
    by the attention mask returns exactly the per-text ids."""
    try:
        enc = tok(list(texts), return_tensors="pt", max_length=512, truncation=True, padding=True)
    except (TypeError, KeyError, ValueError):  # a tokenizer object that only takes single strings
        return [tokenize_roberta(tok, t) for t in texts]
    return _strip_padded(enc["input_ids"], enc["attention_mask"], len(texts))


def _strip_padded(ids, mask, n: int) -> List[List[int]]:
    """Per-row unpadded id lists of a right-padded batch encoding (one vectorised length count
    instead of a Python sum per row)."""
    try:
        a, m = np.asarray(ids).reshape(n, -1), np.asarray(mask).reshape(n, -1)
    except ValueError:  # ragged lists (a tokenizer that ignores padding=True): row by row
        return [_to_list(ids[i])[:int(sum(_to_list(mask[i])))] for i in range(n)]
    lens = m.sum(axis=1).tolist()
    rows = a.tolist()
    return [[int(v) for v in rows[i][:lens[i]]] for i in range(n)]


def tokenize_clip(proc, texts: List[str], truncation: bool = False) -> List[List[int]]:
    """CLIPProcessor text tokenisation (misinfo_forensics.py:386-391, 473-478); returns the unpadded
    id lists (padding ids never influence the causal EOS-pooled embedding)."""
    kw = dict(text=list(texts), return_tensors="pt", padding=True)
    if truncation:
        kw["truncation"] = True
    enc = proc(**kw)
    return _strip_padded(enc["input_ids"], enc["attention_mask"], len(texts))


# ---------------------------------------------------------------------------------------------
# Truth-Vault file (train_clip_detective.py:515-581 writes it; misinfo_forensics.py:214-246 reads)
# ---------------------------------------------------------------------------------------------
class _SafeUnpickler(pickle.Unpickler):
    """Only numpy arrays and plain containers: a vault file cannot execute code on load."""
    _ALLOWED = {
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "dict"), ("builtins", "list"),
        ("collections", "OrderedDict"), ("numpy", "float32"), ("numpy", "float64"), ("numpy", "int64"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"vault file references {module}.{name}; only numpy arrays and "
                                     "plain containers are accepted")


def load_vault(path: str):
    """Returns (embeddings [N, D] in the stored dtype, metadata list of {title, url, date}) or (None, None)
    for an unknown format, following misinfo_forensics.py:222-246.  Accepts the reference's
    pickle (restricted unpickler), .npz, or .json."""
    if path.endswith(".npz"):
        d = dict(np.load(path, allow_pickle=False))
    elif path.endswith(".json"):
        import json
        with open(path) as f:
            d = json.load(f)
    else:
        with open(path, "rb") as f:
            d = _SafeUnpickler(io.BytesIO(f.read())).load()
    if "embeddings" in d:
        emb, meta = d["embeddings"], d["metadata"]
        meta = [dict(m) for m in meta]
    elif "image_embeddings" in d:
        emb = d["image_embeddings"]
        texts = list(d.get("text_contents", []))
        paths = list(d.get("image_paths", []))
        meta = [{"title": texts[i] if i < len(texts) else "Unknown",
                 "url": paths[i] if i < len(paths) else "N/A", "date": "N/A"} for i in range(len(texts))]
    else:
        return None, None
    return np.ascontiguousarray(np.asarray(emb)), meta  # stored dtype kept (search renormalises in it)


def vault_unit_rows(emb) -> np.ndarray:
    """misinfo_forensics.py:443-445 as written: ``V / np.linalg.norm(V, axis=1, keepdims=True)`` in
    the vault's own dtype (a float16 vault renormalises in float16; a zero row becomes NaN, which
    the device ranking then places first, as numpy's argsort does).  The reference recomputes this
    on every search call; it is done once, when the vault is set."""
    v = np.asarray(emb)
    with np.errstate(invalid="ignore", divide="ignore"):
        return v / np.linalg.norm(v, axis=1, keepdims=True)
