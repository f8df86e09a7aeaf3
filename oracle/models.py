"""ORACLE (test infrastructure only) — fp32 CPU restatement of the hot path's model math.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline: the product path never calls it.

Every function restates the arithmetic of the library call the reference makes, as
functional PyTorch fp32 on CPU over a plain ``{state-dict name: tensor}`` mapping:

* RoBERTa-base: HF transformers 5.15.0 ``RobertaModel`` (TF:models/roberta/modeling_roberta.py
  56-155 embeddings, 158-251 self-attention, 329-399 layer, 401-465 encoder), called from
  ``MultiModalMisinfoDetector.forward_text`` (misinfo_forensics.py:92-100).
* Dual heads: misinfo_forensics.py:57-69, 97-98, softmax[:,1] 342-347.
* EfficientNet-B0: torchvision ``efficientnet_b0`` (proxy-pinned, see "Parity status" below;
  torchvision is not installed — SURVEY.md §8c) with the 2-class classifier of
  misinfo_forensics.py:72-76, preprocessing misinfo_forensics.py:249-253.
* CLIP ViT-B/32: HF ``CLIPModel`` (TF:models/clip/modeling_clip.py 138-219 embeddings,
  280-385 attention/MLP/layer, 494-590 text tower incl. EOS pooling 561-582, 594-657 vision
  tower, 683-751 get_*_features).

Parity status: pinned against fixtures produced by the reference code itself
(tests/golden/make_golden.py) for RoBERTa/heads/CLIP/vault/fusion/analyze.  torchvision (the
reference's EfficientNet) is not installed, so the EfficientNet restatement is proxy-pinned: against
the independent EfficientNet of transformers 5.15 configured as B0 with the torchvision-layout
weights mapped onto it (tests/test_oracle_effnet_hf.py: features, logits and scores measured
bit-identical in this container; the test's bound is 1e-4 x the feature scale so other BLAS builds
pass), plus the structural checks (5,288,548 parameters at 1000 classes, 360 state-dict keys).
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def to_torch(sd) -> SD:
    return {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(v)) for k, v in sd.items()}


def _lin(sd: SD, name: str, x: Tensor, bias: bool = True) -> Tensor:
    w = sd[name + ".weight"]
    return F.linear(x, w, sd[name + ".bias"] if bias else None)


def _ln(sd: SD, name: str, x: Tensor, eps: float = 1e-5) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], eps)


def _attention(q: Tensor, k: Tensor, v: Tensor, heads: int, allow: Tensor) -> Tensor:
    """softmax(QK^T * d^-0.5 masked) V, fp32 softmax (TF roberta eager_attention_forward /
    TF clip:280-333).  ``allow`` is bool [B, Lq, Lk] (True = attend)."""
    B, L, D = q.shape
    d = D // heads
    q = q.view(B, L, heads, d).transpose(1, 2)
    k = k.view(B, L, heads, d).transpose(1, 2)
    v = v.view(B, L, heads, d).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) * (d ** -0.5)
    s = s.masked_fill(~allow[:, None], torch.finfo(torch.float32).min)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v)
    return o.transpose(1, 2).reshape(B, L, D)


# ------------------------------------------------------------------------------------------
# RoBERTa-base (post-LN encoder)
# ------------------------------------------------------------------------------------------
def roberta_position_ids(ids: Tensor, padding_idx: int = 1) -> Tensor:
    """TF roberta:142-155 create_position_ids_from_input_ids: cumsum(ids != pad) * mask + pad."""
    mask = ids.ne(padding_idx).int()
    return (torch.cumsum(mask, dim=1).type_as(mask) * mask).long() + padding_idx


def roberta_forward(sd: SD, ids: Tensor, mask: Tensor, prefix: str = "roberta.",
                    layers: int = 12, heads: int = 12) -> Tensor:
    """Last hidden state [B, L, 768] (TF roberta:75-121 embeddings; 329-399 layers)."""
    p = prefix
    ids = ids.long()
    pos = roberta_position_ids(ids)
    x = (sd[p + "embeddings.word_embeddings.weight"][ids]
         + sd[p + "embeddings.token_type_embeddings.weight"][torch.zeros_like(ids)]
         + sd[p + "embeddings.position_embeddings.weight"][pos])
    x = _ln(sd, p + "embeddings.LayerNorm", x)
    allow = mask.bool()[:, None, :].expand(-1, ids.shape[1], -1)
    for i in range(layers):
        lp = f"{p}encoder.layer.{i}."
        q = _lin(sd, lp + "attention.self.query", x)
        k = _lin(sd, lp + "attention.self.key", x)
        v = _lin(sd, lp + "attention.self.value", x)
        a = _attention(q, k, v, heads, allow)
        x = _ln(sd, lp + "attention.output.LayerNorm", _lin(sd, lp + "attention.output.dense", a) + x)
        h = F.gelu(_lin(sd, lp + "intermediate.dense", x))  # GELU-erf (TF activations.py)
        x = _ln(sd, lp + "output.LayerNorm", _lin(sd, lp + "output.dense", h) + x)
    return x


def text_heads(sd: SD, cls: Tensor):
    """misinfo_forensics.py:57-69, 97-98: Linear(768,256) ReLU Dropout(inert) Linear(256,2)."""
    ai = _lin(sd, "ai_head.3", F.relu(_lin(sd, "ai_head.0", cls)))
    mi = _lin(sd, "misinfo_head.3", F.relu(_lin(sd, "misinfo_head.0", cls)))
    return ai, mi


# ------------------------------------------------------------------------------------------
# EfficientNet-B0 (torchvision spec, eval mode)
# ------------------------------------------------------------------------------------------
def effnet_preprocess(img_u8_hwc: Tensor) -> Tensor:
    """misinfo_forensics.py:249-253: Resize((224,224)) (identity at 224^2), ToTensor (/255,
    CHW), Normalize(ImageNet)."""
    x = img_u8_hwc.permute(0, 3, 1, 2).float().div(255.0)
    m = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    s = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    return (x - m) / s


def _bn(sd: SD, name: str, x: Tensor, eps: float = 1e-5) -> Tensor:
    return F.batch_norm(x, sd[name + ".running_mean"], sd[name + ".running_var"],
                        sd[name + ".weight"], sd[name + ".bias"], False, 0.0, eps)


# torchvision efficientnet_b0 inverted-residual setting (expand, kernel, stride, cin, cout, n)
_EFFNET_B0 = [(1, 3, 1, 32, 16, 1), (6, 3, 2, 16, 24, 2), (6, 5, 2, 24, 40, 2), (6, 3, 2, 40, 80, 3),
              (6, 5, 1, 80, 112, 3), (6, 5, 2, 112, 192, 4), (6, 3, 1, 192, 320, 1)]


def _effnet_blocks():
    for si, (e, k, s, cin, cout, n) in enumerate(_EFFNET_B0):
        for j in range(n):
            inp = cin if j == 0 else cout
            st = s if j == 0 else 1
            yield dict(prefix=f"features.{si + 1}.{j}.block", expand=e, k=k, stride=st,
                       cexp=inp * e, residual=(st == 1 and inp == cout))


def effnet_forward(sd: SD, x: Tensor, prefix: str = "efficientnet.", return_features: bool = False):
    """torchvision EfficientNet-B0 features -> avgpool -> classifier (Dropout inert, Linear)."""
    p = prefix
    h = F.silu(_bn(sd, p + "features.0.1", F.conv2d(x, sd[p + "features.0.0.weight"], stride=2, padding=1)))
    for b in _effnet_blocks():
        bp = p + b["prefix"]
        inp = h
        i = 0
        if b["expand"] != 1:
            h = F.silu(_bn(sd, f"{bp}.{i}.1", F.conv2d(h, sd[f"{bp}.{i}.0.weight"])))
            i += 1
        h = F.silu(_bn(sd, f"{bp}.{i}.1", F.conv2d(h, sd[f"{bp}.{i}.0.weight"], stride=b["stride"],
                                                    padding=(b["k"] - 1) // 2, groups=b["cexp"])))
        i += 1
        s = F.adaptive_avg_pool2d(h, 1)
        s = F.silu(F.conv2d(s, sd[f"{bp}.{i}.fc1.weight"], sd[f"{bp}.{i}.fc1.bias"]))
        s = torch.sigmoid(F.conv2d(s, sd[f"{bp}.{i}.fc2.weight"], sd[f"{bp}.{i}.fc2.bias"]))
        h = h * s
        i += 1
        h = _bn(sd, f"{bp}.{i}.1", F.conv2d(h, sd[f"{bp}.{i}.0.weight"]))
        if b["residual"]:
            h = h + inp  # StochasticDepth is identity in eval
    h = F.silu(_bn(sd, p + "features.8.1", F.conv2d(h, sd[p + "features.8.0.weight"])))
    feat = torch.flatten(F.adaptive_avg_pool2d(h, 1), 1)
    logits = _lin(sd, p + "classifier.1", feat)
    return (logits, feat) if return_features else logits


# ------------------------------------------------------------------------------------------
# CLIP ViT-B/32
# ------------------------------------------------------------------------------------------
def clip_preprocess(img_u8_hwc: Tensor) -> Tensor:
    """CLIPImageProcessor at 224x224 input: shortest-edge resize and centre crop are identity,
    rescale 1/255, normalise with the OpenAI mean/std."""
    x = img_u8_hwc.permute(0, 3, 1, 2).float() * (1.0 / 255.0)
    m = torch.tensor(CLIP_MEAN).view(1, 3, 1, 1)
    s = torch.tensor(CLIP_STD).view(1, 3, 1, 1)
    return (x - m) / s


def _clip_layer(sd: SD, lp: str, x: Tensor, heads: int, allow: Tensor) -> Tensor:
    """TF clip:343-385 CLIPEncoderLayer (pre-LN, quick_gelu MLP)."""
    h = _ln(sd, lp + "layer_norm1", x)
    a = _attention(_lin(sd, lp + "self_attn.q_proj", h), _lin(sd, lp + "self_attn.k_proj", h),
                   _lin(sd, lp + "self_attn.v_proj", h), heads, allow)
    x = x + _lin(sd, lp + "self_attn.out_proj", a)
    h = _ln(sd, lp + "layer_norm2", x)
    h = _lin(sd, lp + "mlp.fc1", h)
    h = h * torch.sigmoid(1.702 * h)  # quick_gelu
    return x + _lin(sd, lp + "mlp.fc2", h)


def clip_image_features(sd: SD, pixels: Tensor, layers: int = 12, heads: int = 12) -> Tensor:
    """``get_image_features`` (TF clip:138-219, 594-657, 719-751): unnormalised [B, 512]."""
    B = pixels.shape[0]
    p = "vision_model."
    patches = F.conv2d(pixels, sd[p + "embeddings.patch_embedding.weight"], stride=32)
    patches = patches.flatten(2).transpose(1, 2)
    cls = sd[p + "embeddings.class_embedding"].expand(B, 1, -1)
    x = torch.cat([cls, patches], dim=1) + sd[p + "embeddings.position_embedding.weight"][None]
    x = _ln(sd, p + "pre_layrnorm", x)
    allow = torch.ones(B, x.shape[1], x.shape[1], dtype=torch.bool)
    for i in range(layers):
        x = _clip_layer(sd, f"{p}encoder.layers.{i}.", x, heads, allow)
    pooled = _ln(sd, p + "post_layernorm", x[:, 0, :])
    return F.linear(pooled, sd["visual_projection.weight"])


def clip_eos_index(ids: Tensor, eos_token_id: int = 49407) -> Tensor:
    """TF clip:561-582: legacy configs (eos_token_id == 2) take argmax(ids); otherwise the
    first position equal to eos_token_id."""
    ids = ids.to(torch.int)
    if eos_token_id == 2:
        return ids.argmax(dim=-1)
    return (ids == eos_token_id).int().argmax(dim=-1)


def clip_text_features(sd: SD, ids: Tensor, mask: Tensor, eos_token_id: int = 49407,
                       layers: int = 12, heads: int = 8) -> Tensor:
    """``get_text_features`` (TF clip:221-257, 494-590, 683-717): unnormalised [B, 512]."""
    p = "text_model."
    ids = ids.long()
    B, L = ids.shape
    x = sd[p + "embeddings.token_embedding.weight"][ids] + sd[p + "embeddings.position_embedding.weight"][:L][None]
    causal = torch.tril(torch.ones(L, L, dtype=torch.bool))
    allow = causal[None] & mask.bool()[:, None, :]
    for i in range(layers):
        x = _clip_layer(sd, f"{p}encoder.layers.{i}.", x, heads, allow)
    x = _ln(sd, p + "final_layer_norm", x)
    pooled = x[torch.arange(B), clip_eos_index(ids, eos_token_id)]
    return F.linear(pooled, sd["text_projection.weight"])


def l2n(x: Tensor) -> Tensor:
    return x / x.norm(dim=-1, keepdim=True)
