"""fp16 residual streams under trained-model-like outlier features.

Trained RoBERTa / CLIP carry a few hidden channels whose residual-stream values are orders of
magnitude above the rest (the "outlier features" of transformer LMs); the synthetic N(0, 0.02)
draws have none.  The device path stores the CLIP residual streams in fp16 (``clip_res16 = 1``),
RoBERTa's in fp16 unless its LayerNorm parameters bound the stream above 64 (``text_hilo = -1``:
then fp16 hi + lo), and every GEMM operand / activation in fp16; this draw drives them near their
range:

* RoBERTa (post-LN): in 2 channels every LayerNorm's beta = 900, so the stream -- the LN output,
  stored in fp16 -- holds ~900 there in every layer and every next LayerNorm's mean / variance is
  dominated by them; the weight columns reading those channels (QKV, FFN-1, the heads' first layer)
  are scaled by 0.01 as in trained models, where outlier channels are near no-ops for attention,
  and 3 FFN-1 rows per layer are scaled x8;
* CLIP towers (pre-LN): in 2 channels every FFN-2 adds a bias of 80, so the fp16 stream
  accumulates to ~1e3 by the last layer (the lazy-LN statistics are dominated by them); 3 FFN-1
  rows per layer x8.

The bar is the north-star one: the 5 scores and fusion probabilities within 1e-3 of the fp32
oracle, no inf / NaN, at the full bench batch (B = 256, L = 128, 77-token captions).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROB_CH, VIS_CH, TXT_CH = (77, 588), (13, 400), (50, 300)
OUT = 900.0  # RoBERTa outlier level
STEP = 80.0  # CLIP: per-layer FFN-2 bias in the outlier channels


def outlier_states(det, clip):
    """The draw.  LayerNorm statistics are dominated by the outlier channels (sigma ~ 46 for two
    channels at 900 among 768), so, as in trained models, the normal channels' gamma carries the
    compensating scale and the outlier channels' gamma is small (their LN outputs are near no-ops):
    the normal channels keep O(1) values and input-dependent signal."""
    det = {k: np.array(v, copy=True) for k, v in det.items()}
    clip = {k: np.array(v, copy=True) for k, v in clip.items()}
    ch = list(ROB_CH)
    normal = np.ones(768, bool)
    normal[ch] = False
    sig = OUT * np.sqrt(len(ch) / 768.0)
    det["roberta.embeddings.LayerNorm.bias"][ch] = OUT
    det["roberta.embeddings.LayerNorm.weight"][ch] = 0.5
    for i in range(12):
        p = f"roberta.encoder.layer.{i}."
        for ln in ("attention.output.LayerNorm", "output.LayerNorm"):
            det[p + ln + ".weight"][normal] *= sig
            det[p + ln + ".weight"][ch] = 0.5
            det[p + ln + ".bias"][ch] = OUT
        for w in ("attention.self.query", "attention.self.key", "attention.self.value", "intermediate.dense"):
            det[p + w + ".weight"][:, ch] *= 0.01
        det[p + "intermediate.dense.weight"][[11, 1500, 2900]] *= 8.0
    for h in ("ai_head", "misinfo_head"):
        det[f"{h}.0.weight"][:, ch] *= 0.01
    for tower, chs, H in (("vision_model", VIS_CH, 768), ("text_model", TXT_CH, 512)):
        c = list(chs)
        nm = np.ones(H, bool)
        nm[c] = False
        for i in range(12):
            p = f"{tower}.encoder.layers.{i}."
            clip[p + "mlp.fc2.bias"][c] += STEP
            g = max(1.0, STEP * i * np.sqrt(len(c) / H))  # the stream's outlier level entering layer i
            for ln in ("layer_norm1", "layer_norm2"):
                clip[p + ln + ".weight"][nm] *= g
                clip[p + ln + ".weight"][c] = 0.05
            clip[p + "mlp.fc1.weight"][[5, 900, 1800]] *= 8.0
        fin = "vision_model.post_layernorm" if tower == "vision_model" else "text_model.final_layer_norm"
        clip[fin + ".weight"][nm] *= STEP * 12 * np.sqrt(len(c) / H)
        clip[fin + ".weight"][c] = 0.05
    return det, clip


def test_outlier_streams_full_size_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    from oracle import models as M
    from oracle.pipeline import batched_scores
    det, clip = outlier_states(W.synthetic_detector_state(0), W.synthetic_clip_state(0))
    Bf = 256
    eng = Engine(0, det, clip, max_batch=Bf)
    # default options: CLIP streams fp16; RoBERTa's layout chosen at load time from the LayerNorm
    # parameters (|beta| + 4 |gamma| = 900+ here -> the split hi + lo stream)
    assert eng.get_option("text_hilo") == -1 and eng.get_option("clip_res16") == 1
    assert eng.get_option("text_hilo_effective") == 1
    rid, rm = syn.roberta_ids(Bf, 128, 1234)
    cid, cm = syn.clip_ids(Bf, 77, 1234)
    imgs = syn.images(Bf, 1234)
    vault = syn.vault(2170, 512, 77)
    emb = eng.clip_image(imgs).cpu().numpy()
    for i, r in enumerate(range(0, 2170, 70)[: Bf // 8]):
        vault[r] = emb[i * 8] * 2.0
    eng.set_vault(vault)
    out = eng.analyze_batch(rid, rm, cid, cm, imgs)
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    with torch.no_grad():
        ref = batched_scores(det, clip, rid, rm, cid, cm, imgs, vault)
        # the draw does what it claims: the last RoBERTa layer's CLS row carries O(1e3) values in
        # the outlier channels
        sd = M.to_torch(det)
        cls = M.roberta_forward(sd, torch.as_tensor(rid[:4]).long(), torch.as_tensor(rm[:4]).long())[:, 0]
    assert float(cls[:, list(ROB_CH)].abs().min()) > 500.0
    rest = cls[:, [c for c in range(768) if c not in ROB_CH]]
    assert float(rest.std()) > 0.3 and float((cls[0] - cls[1]).abs().max()) > 0.1  # normal channels alive
    assert np.isfinite(got["scores"]).all() and np.isfinite(got["probs"]).all()
    d = np.abs(got["scores"] - ref["scores"]).max(0)
    names = ("ai", "misinfo", "deepfake", "clip_sim", "vault_disc")
    print("outlier draw: max |d| " + ", ".join(f"{n} {v:.2e}" for n, v in zip(names, d)) +
          f"; probs {np.abs(got['probs'] - ref['probs']).max():.2e}")
    # the fp16-only RoBERTa stream on the same draw, for the record (what the load-time check avoids)
    eng.set_option("text_hilo", 0)
    o16 = eng.analyze_batch(rid, rm, cid, cm, imgs)["scores"].cpu().numpy()
    eng.set_option("text_hilo", -1)
    print(f"  fp16-only RoBERTa stream: max |d| ai {np.abs(o16[:, 0] - ref['scores'][:, 0]).max():.2e}, "
          f"misinfo {np.abs(o16[:, 1] - ref['scores'][:, 1]).max():.2e}")
    np.testing.assert_allclose(got["scores"], ref["scores"], atol=1e-3)
    np.testing.assert_allclose(got["probs"], ref["probs"], atol=1e-3)
    eng.close()


def test_plain_draw_keeps_the_fp16_stream(det_sd, clip_sd):
    """The load-time check leaves ordinary weights on the faster fp16-only stream."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mmf_amd.engine import Engine
    eng = Engine(0, det_sd, clip_sd, max_batch=8)
    assert eng.get_option("text_hilo_effective") == 0
    eng.close()
