"""CPU probe: how far do the HIP path's storage precisions move the 5 scores?

Emulates, in fp32 torch on the CPU, the roundings the device path applies (bf16 GEMM operands,
bf16 attention probabilities / context, bf16 FFN activations) with two residual-stream
policies, and prints the max |score - fp32 score| for the text heads and the CLIP cosine:

  fp32res : residual stream and pre-LN sums kept in fp32 (the round-1 device layout)
  ydelta16: residual stream fp32, the GEMM outputs added to it (out-proj, FFN-2) stored bf16
  bf16res : pre-LN sums and LN outputs stored in bf16 only (half the residual HBM traffic)

    python tools/numerics_probe.py [--batch 32]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmf_amd.synthetic as syn  # noqa: E402
import mmf_amd.weights as W  # noqa: E402
from oracle import models as M  # noqa: E402


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def lin(sd, name, x, rnd, bias=True):
    w = sd[name + ".weight"]
    return F.linear(bf(x) if rnd else x, bf(w) if rnd else w, sd[name + ".bias"] if bias else None)


def attn(q, k, v, heads, allow, rnd):
    B, L, D = q.shape
    d = D // heads
    q, k, v = (t.view(B, L, heads, d).transpose(1, 2) for t in (q, k, v))
    if rnd:
        q, k, v = bf(q), bf(k), bf(v)
    s = torch.matmul(q, k.transpose(-1, -2)) * (d ** -0.5)
    s = s.masked_fill(~allow[:, None], torch.finfo(torch.float32).min)
    p = torch.softmax(s, -1)
    if rnd:
        p = bf(p)
    o = torch.matmul(p, v).transpose(1, 2).reshape(B, L, D)
    return bf(o) if rnd else o


def roberta(sd, ids, mask, mode):
    rnd = mode != "fp32"
    res16 = mode == "bf16res"
    p = "roberta."
    ids = ids.long()
    pos = M.roberta_position_ids(ids)
    x = (sd[p + "embeddings.word_embeddings.weight"][ids] + sd[p + "embeddings.token_type_embeddings.weight"][0]
         + sd[p + "embeddings.position_embeddings.weight"][pos])
    x = M._ln(sd, p + "embeddings.LayerNorm", x)
    if res16:
        x = bf(x)
    allow = mask.bool()[:, None, :].expand(-1, ids.shape[1], -1)
    for i in range(12):
        lp = f"{p}encoder.layer.{i}."
        q = lin(sd, lp + "attention.self.query", x, rnd)
        k = lin(sd, lp + "attention.self.key", x, rnd)
        v = lin(sd, lp + "attention.self.value", x, rnd)
        a = attn(q, k, v, 12, allow, rnd)
        y = lin(sd, lp + "attention.output.dense", a, rnd)
        s = (bf(y) if mode == "ydelta16" else y) + x
        if res16:
            s = bf(s)
        x = M._ln(sd, lp + "attention.output.LayerNorm", s)
        if res16:
            x = bf(x)
        h = F.gelu(lin(sd, lp + "intermediate.dense", x, rnd))
        y = lin(sd, lp + "output.dense", bf(h) if rnd else h, rnd)
        s = (bf(y) if mode == "ydelta16" else y) + x
        if res16:
            s = bf(s)
        x = M._ln(sd, lp + "output.LayerNorm", s)
        if res16:
            x = bf(x)
    return x


def clip_text(sd, ids, mask, mode):
    rnd = mode != "fp32"
    res16 = mode == "bf16res"
    p = "text_model."
    ids = ids.long()
    B, L = ids.shape
    x = sd[p + "embeddings.token_embedding.weight"][ids] + sd[p + "embeddings.position_embedding.weight"][:L][None]
    if res16:
        x = bf(x)
    allow = torch.tril(torch.ones(L, L, dtype=torch.bool))[None] & mask.bool()[:, None, :]
    for i in range(12):
        lp = f"{p}encoder.layers.{i}."
        h = M._ln(sd, lp + "layer_norm1", x)
        a = attn(lin(sd, lp + "self_attn.q_proj", h, rnd), lin(sd, lp + "self_attn.k_proj", h, rnd),
                 lin(sd, lp + "self_attn.v_proj", h, rnd), 8, allow, rnd)
        y = lin(sd, lp + "self_attn.out_proj", a, rnd)
        x = x + (bf(y) if mode == "ydelta16" else y)
        if res16:
            x = bf(x)
        h = M._ln(sd, lp + "layer_norm2", x)
        h = lin(sd, lp + "mlp.fc1", h, rnd)
        h = h * torch.sigmoid(1.702 * h)
        y = lin(sd, lp + "mlp.fc2", bf(h) if rnd else h, rnd)
        x = x + (bf(y) if mode == "ydelta16" else y)
        if res16:
            x = bf(x)
    x = M._ln(sd, p + "final_layer_norm", x)
    pooled = x[torch.arange(B), M.clip_eos_index(ids, 49407)]
    return M.l2n(F.linear(pooled, sd["text_projection.weight"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    torch.set_num_threads(8)
    det = M.to_torch(W.synthetic_detector_state(0))
    clip = M.to_torch(W.synthetic_clip_state(0))
    B = a.batch
    rid, rm = syn.roberta_ids(B, 128, 11)
    cid, cm = syn.clip_ids(B, 77, 11)
    rid, rm, cid, cm = map(torch.from_numpy, (rid, rm, cid, cm))
    out = {}
    with torch.no_grad():
        for mode in ("fp32", "fp32res", "ydelta16", "bf16res"):
            x = roberta(det, rid, rm, mode)[:, 0]
            ai, mi = M.text_heads(det, x)
            out[mode] = (torch.softmax(ai, 1)[:, 1], torch.softmax(mi, 1)[:, 1], clip_text(clip, cid, cm, mode))
    for mode in ("fp32res", "ydelta16", "bf16res"):
        e_ai = (out[mode][0] - out["fp32"][0]).abs().max().item()
        e_mi = (out[mode][1] - out["fp32"][1]).abs().max().item()
        e_ct = (1 - (out[mode][2] * out["fp32"][2]).sum(1)).abs().max().item()
        print(f"{mode}: max|d ai_score| {e_ai:.2e}  max|d misinfo_score| {e_mi:.2e}  max(1-cos text emb) {e_ct:.2e}")


if __name__ == "__main__":
    main()
