"""ORACLE (test infrastructure only) — CPU restatement of the orchestration around the models:
Truth-Vault search, FusionJudge, verdict fallbacks, rule-based explanation and the
``analyze()`` result dict.  Each function cites the reference lines it restates.
Never imported by the product path.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import models as M


def vault_normalise(vault: np.ndarray) -> np.ndarray:
    """misinfo_forensics.py:443-445 (recomputed on every call in the reference)."""
    return vault / np.linalg.norm(vault, axis=1, keepdims=True)


def vault_search(vault: np.ndarray, query_unit: np.ndarray, top_k: int = 5):
    """misinfo_forensics.py:443-464 for one query: GEMV, argsort top-k descending, threshold.
    Returns (top_indices, top_similarities, vault_discrepancy, max_similarity)."""
    sims = vault_normalise(vault) @ query_unit
    top = np.argsort(sims)[-top_k:][::-1]
    top_s = sims[top]
    max_s = float(top_s[0])
    return top, top_s, (max_s if max_s > 0.85 else 0.0), max_s


def fusion_logits(sd, x5: torch.Tensor) -> torch.Tensor:
    """misinfo_forensics.py:83-90, 106-108: Linear(5,64) ReLU Dropout(inert) Linear(64,32) ReLU
    Linear(32,2)."""
    h = F.relu(M._lin(sd, "fusion_layer.0", x5))
    h = F.relu(M._lin(sd, "fusion_layer.3", h))
    return M._lin(sd, "fusion_layer.5", h)


def fusion_verdict(sd, scores: Dict[str, float]) -> Dict:
    """misinfo_forensics.py:575-615."""
    x = torch.tensor([[scores.get("ai_score", 0.0), scores.get("misinfo_score", 0.0),
                       scores.get("deepfake_score", 0.0), scores.get("clip_similarity", 0.0),
                       scores.get("vault_discrepancy", 0.0)]], dtype=torch.float32)
    probs = torch.softmax(fusion_logits(sd, x), dim=1)
    real_prob, fake_prob = probs[0, 0].item(), probs[0, 1].item()
    label = 1 if fake_prob > 0.5 else 0
    return {"verdict": label, "confidence": fake_prob if label == 1 else real_prob,
            "fake_probability": fake_prob, "real_probability": real_prob}


def fallback_verdict(text_present: bool, image_present: bool, all_scores: Dict) -> Dict:
    """misinfo_forensics.py:882-899 (no fusion when a modality is missing)."""
    if text_present and not image_present:
        fake = float(all_scores.get("misinfo_score", 0.0))
    elif image_present and not text_present:
        fake = float(max(all_scores.get("deepfake_score", 0.0), all_scores.get("vault_discrepancy", 0.0)))
    else:
        fake = 0.5
    fake = max(0.0, min(1.0, fake))
    real = 1.0 - fake
    label = 1 if fake > 0.5 else 0
    return {"verdict": label, "confidence": fake if label == 1 else real,
            "fake_probability": fake, "real_probability": real}


def explanation(all_scores: Dict, vault_matches: list) -> str:
    """misinfo_forensics.py:742-765 rule cascade (Gemini unavailable, 707-709)."""
    v = "FAKE" if all_scores["verdict"] == 1 else "REAL"
    if all_scores["vault_discrepancy"] > 0.7:
        return (f"This content is classified as {v}. "
                f"Our database found this image was previously published in a different context "
                f"(\"{vault_matches[0]['title']}\"), suggesting potential misuse.")
    if all_scores["deepfake_score"] > 0.7:
        return (f"This content is classified as {v}. "
                f"The image shows strong signs of digital manipulation (deepfake probability: "
                f"{all_scores['deepfake_score']:.1%}).")
    if all_scores["ai_score"] > 0.7:
        return (f"This content is classified as {v}. "
                f"The text exhibits characteristics typical of AI-generated content.")
    if all_scores["misinfo_score"] > 0.7:
        return (f"This content is classified as {v}. "
                f"The text uses language patterns commonly associated with misinformation.")
    if all_scores["clip_similarity"] < 0.3:
        return (f"This content is classified as {v}. "
                f"The image and caption show poor alignment, suggesting potential mismatching.")
    return (f"This content is classified as {v} with {all_scores['confidence']:.1%} confidence. "
            f"Multiple signals from text analysis, image forensics, and database checks support this assessment.")


class OracleForensics:
    """Per-sample restatement of ``MisinfoForensics.analyze`` (misinfo_forensics.py:767-927)
    over pre-tokenised inputs: ``text`` is a pair (roberta_ids, clip_ids) of 1-D int arrays
    (unpadded, as the reference tokenises a single string), ``image`` a uint8 [224,224,3]."""

    def __init__(self, det_sd, clip_sd, vault: Optional[np.ndarray] = None,
                 vault_meta: Optional[List[dict]] = None, title_clip_ids: Optional[list] = None,
                 eos_token_id: int = 49407):
        self.sd = M.to_torch(det_sd)
        self.csd = M.to_torch(clip_sd)
        self.vault = vault
        self.vault_meta = vault_meta
        self.title_ids = title_clip_ids
        self.eos = eos_token_id

    # misinfo_forensics.py:319-352
    def analyze_text(self, rob_ids):
        ids = torch.as_tensor(np.asarray(rob_ids)[None])
        h = M.roberta_forward(self.sd, ids, torch.ones_like(ids))
        ai, mi = M.text_heads(self.sd, h[:, 0, :])
        return {"ai_score": torch.softmax(ai, 1)[0, 1].item(),
                "misinfo_score": torch.softmax(mi, 1)[0, 1].item()}

    # misinfo_forensics.py:354-373
    def analyze_image(self, img):
        x = M.effnet_preprocess(torch.as_tensor(np.asarray(img)[None]))
        return {"deepfake_score": torch.softmax(M.effnet_forward(self.sd, x), 1)[0, 1].item()}

    def _text_emb(self, clip_ids):
        ids = torch.as_tensor(np.asarray(clip_ids)[None])
        return M.clip_text_features(self.csd, ids, torch.ones_like(ids), self.eos)

    def _image_emb(self, img):
        return M.clip_image_features(self.csd, M.clip_preprocess(torch.as_tensor(np.asarray(img)[None])))

    # misinfo_forensics.py:375-408
    def analyze_consistency(self, clip_ids, img):
        t = M.l2n(M.l2n(self._text_emb(clip_ids)))
        i = M.l2n(M.l2n(self._image_emb(img)))
        return {"clip_similarity": (t @ i.T).item()}

    # misinfo_forensics.py:410-491
    def search_vault(self, img, caption_clip_ids=None, top_k: int = 5):
        if self.vault is None:
            return {"vault_discrepancy": 0.0, "matches": [], "vault_available": False, "text_similarity": 0.0}
        q = M.l2n(self._image_emb(img)).numpy()[0]
        top, top_s, disc, max_s = vault_search(self.vault, q, top_k)
        matches = [{"similarity": float(s), "title": self.vault_meta[int(i)]["title"],
                    "url": self.vault_meta[int(i)].get("url", "N/A"),
                    "date": self.vault_meta[int(i)].get("date", "N/A")} for i, s in zip(top, top_s)]
        text_sim = 0.0
        if caption_clip_ids is not None and max_s > 0.85 and matches:
            a = M.l2n(self._text_emb(caption_clip_ids))
            b = M.l2n(self._text_emb(self.title_ids[int(top[0])]))
            text_sim = float((a[0] @ b[0]).item())
        return {"vault_discrepancy": disc, "matches": matches, "vault_available": True,
                "text_similarity": text_sim, "top_indices": [int(i) for i in top]}

    def analyze(self, text=None, image=None) -> Dict:
        if text is None and image is None:
            raise ValueError("Provide at least one of: text, image_path, or video_path")
        text_scores = {"ai_score": 0.0, "misinfo_score": 0.0}
        if text is not None:
            text_scores = self.analyze_text(text[0])
        image_scores = {"deepfake_score": 0.0}
        cons = {"clip_similarity": 0.0}
        vault_res = {"vault_discrepancy": 0.0, "matches": [], "vault_available": self.vault is not None,
                     "text_similarity": 0.0}
        if image is not None:
            image_scores = self.analyze_image(image)
            if text is not None:
                cons = self.analyze_consistency(text[1], image)
            vault_res = self.search_vault(image, text[1] if text is not None else None)
        all_scores = {**text_scores, **image_scores, **cons,
                      "vault_discrepancy": vault_res["vault_discrepancy"],
                      "text_similarity": vault_res.get("text_similarity", 0.0)}
        if text is not None and image is not None:
            vr = fusion_verdict(self.sd, all_scores)
        else:
            vr = fallback_verdict(text is not None, image is not None, all_scores)
        all_scores.update(vr)
        return {"verdict": vr["verdict"], "verdict_text": "FAKE" if vr["verdict"] == 1 else "REAL",
                "confidence": vr["confidence"], "scores": all_scores,
                "vault_matches": vault_res["matches"],
                "explanation": explanation(all_scores, vault_res["matches"])}


def batched_scores(det_sd, clip_sd, rob_ids, rob_mask, clip_ids, clip_mask, imgs_u8,
                   vault: Optional[np.ndarray], eos_token_id: int = 49407, title_emb_unit=None,
                   top_k: int = 5):
    """Batched fp32 restatement of the five signals + fusion for text+image pairs (the bench
    workload; ViT computed once per pair).  Returns a dict of numpy arrays."""
    sd, csd = M.to_torch(det_sd), M.to_torch(clip_sd)
    rid, rm = torch.as_tensor(rob_ids), torch.as_tensor(rob_mask)
    h = M.roberta_forward(sd, rid, rm)
    ai, mi = M.text_heads(sd, h[:, 0, :])
    imgs = torch.as_tensor(imgs_u8)
    eff = M.effnet_forward(sd, M.effnet_preprocess(imgs))
    img_e = M.l2n(M.clip_image_features(csd, M.clip_preprocess(imgs)))
    txt_e = M.l2n(M.clip_text_features(csd, torch.as_tensor(clip_ids), torch.as_tensor(clip_mask), eos_token_id))
    clip_sim = (img_e * txt_e).sum(-1)
    B = rid.shape[0]
    disc = torch.zeros(B)
    tsim = torch.zeros(B)
    top_idx = np.zeros((B, top_k), dtype=np.int64)
    top_sim = np.zeros((B, top_k), dtype=np.float32)
    if vault is not None:
        vn = vault_normalise(vault)
        sims = img_e.numpy() @ vn.T
        for b in range(B):
            t = np.argsort(sims[b])[-top_k:][::-1]
            top_idx[b], top_sim[b] = t, sims[b, t]
            m = float(sims[b, t[0]])
            disc[b] = m if m > 0.85 else 0.0
            if m > 0.85 and title_emb_unit is not None:
                tsim[b] = float(txt_e[b] @ torch.as_tensor(title_emb_unit[t[0]]))
    x5 = torch.stack([torch.softmax(ai, 1)[:, 1], torch.softmax(mi, 1)[:, 1],
                      torch.softmax(eff, 1)[:, 1], clip_sim, disc], dim=1)
    probs = torch.softmax(fusion_logits(sd, x5), 1)
    return {"scores": x5.numpy(), "probs": probs.numpy(), "text_similarity": tsim.numpy(),
            "top_idx": top_idx, "top_sim": top_sim, "ai_logits": ai.numpy(), "misinfo_logits": mi.numpy(),
            "effnet_logits": eff.numpy(), "image_emb": img_e.numpy(), "text_emb": txt_e.numpy(),
            "cls": h[:, 0, :].numpy()}
