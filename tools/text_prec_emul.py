"""CPU emulation of the RoBERTa tower's fp16 rounding points (text_hilo = 1, the split hi + lo
stream) on the gamma-7 dominating-channel draw (tests/test_gpu_outliers.py), to find which rounding
points carry the error that the precise mode removes.  Each flag removes one rounding point (that
value kept in fp32); prints max |score - fp64 reference| per variant.  Not a parity tool: the
device kernels' accumulation orders are not modelled, only where values are rounded to fp16.

    python tools/text_prec_emul.py [--rows 32] [--gamma 7]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import mmf_amd.synthetic as syn  # noqa: E402
import mmf_amd.weights as W  # noqa: E402
from oracle import models as M  # noqa: E402
from test_gpu_outliers import DOM_CH, dominating_gamma_state  # noqa: E402


def h(x):
    return x.half().float()


def split_corr(x, S):
    """fp16 hi of x, with the channels S kept exact (the hi + lo correction columns)"""
    y = h(x)
    if S is not None:
        y[..., S] = x[..., S]
    return y


def forward(sd, ids, mask, cfg, S):
    """cfg: set of rounding points kept in fp32; S: channels of the LN outputs whose GEMM operand
    (and weight columns) carry the hi + lo correction"""
    f = lambda name: name in cfg  # noqa: E731
    p = "roberta."
    B, L = ids.shape
    pos = M.roberta_position_ids(ids)
    x = (sd[p + "embeddings.word_embeddings.weight"][ids] + sd[p + "embeddings.token_type_embeddings.weight"][0]
         + sd[p + "embeddings.position_embeddings.weight"][pos])
    x = M._ln(sd, p + "embeddings.LayerNorm", x)
    allow = mask.bool()[:, None, None, :]

    def wq(name, cols_exact=None):
        w = sd[name + ".weight"]
        wh = h(w)
        if cols_exact is not None:
            wh[:, cols_exact] = w[:, cols_exact]
        return wh, sd[name + ".bias"]

    for i in range(12):
        lp = f"{p}encoder.layer.{i}."
        a = x if f("qkv_a") else split_corr(x, S)
        outs = []
        for n in ("query", "key", "value"):
            w, b = wq(lp + "attention.self." + n, S if (S is not None and f("w_corr")) else None)
            if f("w_exact"):
                w = sd[lp + "attention.self." + n + ".weight"]
            o = F.linear(a, w, b)
            outs.append(o if f("qkv_out") else h(o))
        q, k, v = outs
        d = 64
        qh = q.view(B, L, 12, d).transpose(1, 2)
        kh = k.view(B, L, 12, d).transpose(1, 2)
        vh = v.view(B, L, 12, d).transpose(1, 2)
        s = torch.matmul(qh, kh.transpose(-1, -2)) * 0.125
        s = s.masked_fill(~allow, float("-inf"))
        pr = torch.softmax(s, -1)
        if not f("probs"):
            pr = h(pr)
        ctx = torch.matmul(pr, vh).transpose(1, 2).reshape(B, L, 768)
        if not f("ctx"):
            ctx = h(ctx)
        w, b = wq(lp + "attention.output.dense")
        if f("w_exact"):
            w = sd[lp + "attention.output.dense.weight"]
        y = F.linear(ctx, w, b)
        if not f("y"):
            y = h(y)
        x = M._ln(sd, lp + "attention.output.LayerNorm", y + x)
        a = x if f("fc1_a") else split_corr(x, S)
        w, b = wq(lp + "intermediate.dense", S if (S is not None and f("w_corr")) else None)
        if f("w_exact"):
            w = sd[lp + "intermediate.dense.weight"]
        hid = F.gelu(F.linear(a, w, b))
        if not f("hidden"):
            hid = h(hid)
        w, b = wq(lp + "output.dense")
        if f("w_exact"):
            w = sd[lp + "output.dense.weight"]
        y = F.linear(hid, w, b)
        if not f("y"):
            y = h(y)
        x = M._ln(sd, lp + "output.LayerNorm", y + x)
    return x


def scores(sd, cls):
    ai, mi = M.text_heads(sd, cls)
    return torch.stack([torch.softmax(ai, 1)[:, 1], torch.softmax(mi, 1)[:, 1]], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--gamma", type=float, default=7.0)
    a = ap.parse_args()
    det = dominating_gamma_state(W.synthetic_detector_state(0), a.gamma, kappa=a.gamma)
    rid, rm = syn.roberta_ids(a.rows, 128, 99, [128, 100, 60, 17])
    ids, mask = torch.as_tensor(rid).long(), torch.as_tensor(rm).long()
    sd64 = {k: torch.as_tensor(v).double() for k, v in det.items()}
    sd32 = {k: torch.as_tensor(v).float() for k, v in det.items()}
    torch.set_num_threads(8)
    with torch.no_grad():
        ref = scores(sd64, M.roberta_forward(sd64, ids, mask)[:, 0]).numpy()
        gam = np.abs(det["roberta.encoder.layer.0.output.LayerNorm.weight"])
        top = [int(c) for c in np.argsort(-gam)[:32]]
        variants = [
            ("split (all rounding points)", set(), None),
            ("fp32 everywhere", {"qkv_a", "fc1_a", "qkv_out", "probs", "ctx", "y", "hidden", "w_exact"}, None),
            ("exact weights", {"w_exact"}, None),
            ("exact QKV / FC1 operands", {"qkv_a", "fc1_a"}, None),
            ("corr. channel S={dom}", {"w_corr"}, [DOM_CH]),
            ("corr. 32 top-|gamma| channels", {"w_corr"}, top),
            ("fp32 QKV outputs", {"qkv_out"}, None),
            ("fp32 probs", {"probs"}, None),
            ("fp32 ctx", {"ctx"}, None),
            ("fp32 branch outputs y", {"y"}, None),
            ("fp32 hidden", {"hidden"}, None),
            ("corr S + fp32 y", {"w_corr", "y"}, [DOM_CH]),
            ("corr S + fp32 y + qkv_out", {"w_corr", "y", "qkv_out"}, [DOM_CH]),
            ("corr S + fp32 y + ctx", {"w_corr", "y", "ctx"}, [DOM_CH]),
            ("corr S + y + ctx + qkv_out + probs", {"w_corr", "y", "ctx", "qkv_out", "probs"}, [DOM_CH]),
            ("corr S + y + ctx + hidden", {"w_corr", "y", "ctx", "hidden"}, [DOM_CH]),
            ("all but weights", {"qkv_a", "fc1_a", "qkv_out", "probs", "ctx", "y", "hidden"}, None),
        ]
        for name, cfg, S in variants:
            out = scores(sd32, forward(sd32, ids, mask, cfg, S)[:, 0]).double().numpy()
            print(json.dumps({"variant": name.replace("{dom}", str(DOM_CH)),
                              "max_err": round(float(np.abs(out - ref).max()), 7)}), flush=True)


if __name__ == "__main__":
    main()
