"""Pins the oracle's EfficientNet-B0 (oracle/models.py:effnet_forward) against an independent
public implementation of the same architecture.

The reference builds `torchvision.models.efficientnet_b0` (misinfo_forensics.py:73-79,
classifier[1] -> Linear(1280, 2)); torchvision is not installed here, so the oracle's restatement
cannot be run against it.  transformers (5.x, installed) ships its own EfficientNet
(models/efficientnet/modeling_efficientnet.py).  Configured as B0 (width = depth = 1.0,
hidden_dim 1280, BatchNorm eps 1e-5 as torchvision's default nn.BatchNorm2d) with symmetric
depthwise padding on every block (`depthwise_padding` = all blocks: correct_pad(k, adjust=False)
= k//2 on each side, torchvision's `(k - 1) // 2`) and the stem's TF-style (0, 1, 0, 1) zero pad
swapped for torchvision's padding=1, it computes the same function as torchvision's B0: same
MBConv order (expand 1x1 + BN + SiLU, depthwise + BN + SiLU, SE on the block-input width / 4
with SiLU / sigmoid, project 1x1 + BN, identity residual when stride 1 and cin == cout), same
head (1x1 -> 1280 + BN + SiLU, global mean).  Mapping the torchvision-layout weights onto it and
comparing features and logits pins the oracle's block structure, BN placement, SE width and
residual rule (parity test infrastructure only; CPU)."""
import numpy as np
import pytest
import torch

from oracle import models as M

transformers = pytest.importorskip("transformers")


def _hf_b0():
    from transformers import EfficientNetConfig, EfficientNetModel
    cfg = EfficientNetConfig(width_coefficient=1.0, depth_coefficient=1.0, hidden_dim=1280,
                             depthwise_padding=list(range(64)), batch_norm_eps=1e-5)
    m = EfficientNetModel(cfg).eval()
    m.embeddings.padding = torch.nn.ZeroPad2d(1)  # torchvision stem: Conv2d(3, 32, 3, 2, padding=1)
    return m


def _tv_to_hf(sd):
    """torchvision efficientnet_b0 keys (prefix "efficientnet.") -> transformers EfficientNetModel."""
    out = {}

    def bn(src, dst):
        for s in ("weight", "bias", "running_mean", "running_var"):
            out[f"{dst}.{s}"] = sd[f"{src}.{s}"]

    p = "efficientnet.features."
    out["embeddings.convolution.weight"] = sd[p + "0.0.weight"]
    bn(p + "0.1", "embeddings.batchnorm")
    b = 0
    for si, (e, k, s, cin, cout, n) in enumerate(M._EFFNET_B0):
        for j in range(n):
            tp, hp = f"{p}{si + 1}.{j}.block", f"encoder.blocks.{b}"
            i = 0
            if e != 1:
                out[f"{hp}.expansion.expand_conv.weight"] = sd[f"{tp}.0.0.weight"]
                bn(f"{tp}.0.1", f"{hp}.expansion.expand_bn")
                i = 1
            out[f"{hp}.depthwise_conv.depthwise_conv.weight"] = sd[f"{tp}.{i}.0.weight"]
            bn(f"{tp}.{i}.1", f"{hp}.depthwise_conv.depthwise_norm")
            for a, c in (("fc1", "reduce"), ("fc2", "expand")):
                out[f"{hp}.squeeze_excite.{c}.weight"] = sd[f"{tp}.{i + 1}.{a}.weight"]
                out[f"{hp}.squeeze_excite.{c}.bias"] = sd[f"{tp}.{i + 1}.{a}.bias"]
            out[f"{hp}.projection.project_conv.weight"] = sd[f"{tp}.{i + 2}.0.weight"]
            bn(f"{tp}.{i + 2}.1", f"{hp}.projection.project_bn")
            b += 1
    out["encoder.top_conv.weight"] = sd[p + "8.0.weight"]
    bn(p + "8.1", "encoder.top_bn")
    return out


def test_oracle_effnet_matches_transformers_b0(det_sd, golden_inputs):
    sd = M.to_torch(det_sd)
    hf = _hf_b0()
    mapped = _tv_to_hf(sd)
    missing, unexpected = hf.load_state_dict(mapped, strict=False)
    # the only keys left unset are BatchNorm step counters, unused in eval
    assert all(k.endswith("num_batches_tracked") for k in missing), missing
    assert not unexpected, unexpected
    assert len(hf.encoder.blocks) == 16 and sum(p.numel() for p in hf.parameters()) == 4_007_548

    x = M.effnet_preprocess(torch.as_tensor(golden_inputs["imgs"][:4]))
    with torch.no_grad():
        logits, feat = M.effnet_forward(sd, x, return_features=True)
        o = hf(pixel_values=x)
        hf_feat = o.last_hidden_state.mean(dim=(2, 3))
        hf_logits = torch.nn.functional.linear(hf_feat, sd["efficientnet.classifier.1.weight"],
                                               sd["efficientnet.classifier.1.bias"])
    assert torch.allclose(o.pooler_output.flatten(1), hf_feat, atol=1e-5)
    scale = float(feat.abs().max())
    np.testing.assert_allclose(feat.numpy(), hf_feat.numpy(), atol=1e-4 * scale, rtol=0)
    np.testing.assert_allclose(logits.numpy(), hf_logits.numpy(), atol=1e-4 * max(1.0, float(logits.abs().max())),
                               rtol=0)
    # and the score the pipeline reports (softmax(.)[:, 1], misinfo_forensics.py:366-371)
    np.testing.assert_allclose(torch.softmax(logits, 1)[:, 1].numpy(), torch.softmax(hf_logits, 1)[:, 1].numpy(),
                               atol=1e-5)
