"""CPU probe: numerics of the "lazy LayerNorm" encoder layout before building it on the device.

Emulates in fp32 torch with fp16 roundings where the device stores fp16:

  cur : the current device layout -- fp16 GEMM operands, fp16 residual streams, LN materialised by
        add+LN kernels (RoBERTa stream = fp16(LN(s)), CLIP stream = fp16(s), GEMM operand fp16(LN(s)))
  fold: LN never materialised -- the producer GEMM (out-proj / FFN-2) stores the raw sum s in fp16
        plus per-row (mean, rstd); the consumer GEMM (QKV / FFN-1) reads fp16(s) as its A operand
        against W' = fp16(W * gamma) and finishes with r * (acc - mean * u) + c, u = rowsum(W'),
        c = b + W . beta; RoBERTa's post-LN residual LN(s) is formed elementwise in the next
        producer's epilogue

and prints max |score - fp32| for the two text heads and 1 - cos of the CLIP text embedding.

    python tools/lnfold_probe.py [--batch 16]
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

EPS = 1e-5


def h(x):
    return x.half().float()


def stats(s):
    mu = s.mean(-1, keepdim=True)
    r = torch.rsqrt(((s - mu) ** 2).mean(-1, keepdim=True) + EPS)
    return mu, r


def ln_apply(s, mu, r, g, b):
    return (s - mu) * r * g + b


def lin16(sd, name, x):
    return F.linear(h(x), h(sd[name + ".weight"]), sd[name + ".bias"])


def lin_fold(sd, name, s, ln, mode):
    """LN(s) . W^T + b: materialised (cur) or folded (fold)."""
    g, b = sd[ln + ".weight"], sd[ln + ".bias"]
    w, bias = sd[name + ".weight"], sd[name + ".bias"]
    mu, r = stats(s)
    if mode == "cur":
        return F.linear(h(ln_apply(s, mu, r, g, b)), h(w), bias)
    wf = h(w * g[None, :])
    u = wf.sum(1)
    c = bias + w @ b
    return r * (F.linear(h(s), wf) - mu * u) + c


def attn(q, k, v, heads, allow):
    B, L, D = q.shape
    d = D // heads
    q, k, v = (h(t).view(B, L, heads, d).transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(q, k.transpose(-1, -2)) * (d ** -0.5)
    s = s.masked_fill(~allow[:, None], torch.finfo(torch.float32).min)
    p = torch.softmax(s, -1)
    return h(torch.matmul(h(p), v).transpose(1, 2).reshape(B, L, D))


def roberta(sd, ids, mask, mode):
    p = "roberta."
    ids = ids.long()
    pos = M.roberta_position_ids(ids)
    e = (sd[p + "embeddings.word_embeddings.weight"][ids] + sd[p + "embeddings.token_type_embeddings.weight"][0]
         + sd[p + "embeddings.position_embeddings.weight"][pos])
    allow = mask.bool()[:, None, :].expand(-1, ids.shape[1], -1)
    # stream: (s, ln name) -- the layer input is LN_ln(s)
    s, ln = h(e), p + "embeddings.LayerNorm"
    if mode == "cur":
        s, ln = h(M._ln(sd, ln, e)), None
    for i in range(12):
        lp = f"{p}encoder.layer.{i}."

        def inp_lin(name):
            if ln is None:
                return lin16(sd, name, s)
            return lin_fold(sd, name, s, ln, mode)

        def residual():
            if ln is None:
                return s
            mu, r = stats(s)
            return ln_apply(s, mu, r, sd[ln + ".weight"], sd[ln + ".bias"])

        q, k, v = (inp_lin(lp + "attention.self." + n) for n in ("query", "key", "value"))
        a = attn(q, k, v, 12, allow)
        y = lin16(sd, lp + "attention.output.dense", a)
        if mode == "cur":
            s1 = h(y) + s
            s, ln = h(M._ln(sd, lp + "attention.output.LayerNorm", s1)), None
        else:
            s, ln = h(y + residual()), lp + "attention.output.LayerNorm"
        hid = F.gelu(inp_lin(lp + "intermediate.dense"))
        y = lin16(sd, lp + "output.dense", h(hid))
        if mode == "cur":
            s2 = h(y) + s
            s, ln = h(M._ln(sd, lp + "output.LayerNorm", s2)), None
        else:
            s, ln = h(y + residual()), lp + "output.LayerNorm"
    if ln is None:
        return s
    mu, r = stats(s)
    return ln_apply(s, mu, r, sd[ln + ".weight"], sd[ln + ".bias"])


def clip_text(sd, ids, mask, mode):
    p = "text_model."
    ids = ids.long()
    B, L = ids.shape
    x = h(sd[p + "embeddings.token_embedding.weight"][ids] + sd[p + "embeddings.position_embedding.weight"][:L][None])
    allow = torch.tril(torch.ones(L, L, dtype=torch.bool))[None] & mask.bool()[:, None, :]
    for i in range(12):
        lp = f"{p}encoder.layers.{i}."
        q, k, v = (lin_fold(sd, lp + "self_attn." + n, x, lp + "layer_norm1", mode) for n in ("q_proj", "k_proj", "v_proj"))
        a = attn(q, k, v, 8, allow)
        y = lin16(sd, lp + "self_attn.out_proj", a)
        x = h(x + (h(y) if mode == "cur" else y))
        hid = lin_fold(sd, lp + "mlp.fc1", x, lp + "layer_norm2", mode)
        hid = hid * torch.sigmoid(1.702 * hid)
        y = lin16(sd, lp + "mlp.fc2", h(hid))
        x = h(x + (h(y) if mode == "cur" else y))
    x = M._ln(sd, p + "final_layer_norm", x)
    pooled = x[torch.arange(B), M.clip_eos_index(ids, 49407)]
    return M.l2n(F.linear(pooled, sd["text_projection.weight"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    torch.set_num_threads(8)
    det = M.to_torch(W.synthetic_detector_state(a.seed))
    clip = M.to_torch(W.synthetic_clip_state(a.seed))
    B = a.batch
    rid, rm = syn.roberta_ids(B, 128, 11)
    cid, cm = syn.clip_ids(B, 77, 11)
    rid, rm, cid, cm = map(torch.from_numpy, (rid, rm, cid, cm))
    with torch.no_grad():
        x = M.roberta_forward(det, rid.long(), rm.long())[:, 0]
        ai, mi = M.text_heads(det, x)
        ref = (torch.softmax(ai, 1)[:, 1], torch.softmax(mi, 1)[:, 1])
        import numerics_probe as NP
        ref_t = NP.clip_text(clip, cid, cm, "fp32")  # same eos rule as the emulation
        for mode in ("cur", "fold"):
            x = roberta(det, rid, rm, mode)[:, 0]
            ai, mi = M.text_heads(det, x)
            sc = (torch.softmax(ai, 1)[:, 1], torch.softmax(mi, 1)[:, 1])
            t = clip_text(clip, cid, cm, mode)
            print(f"{mode}: max|d ai| {(sc[0] - ref[0]).abs().max():.2e}  max|d misinfo| {(sc[1] - ref[1]).abs().max():.2e}"
                  f"  max(1-cos clip text) {(1 - (t * ref_t).sum(1)).abs().max():.2e}", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
