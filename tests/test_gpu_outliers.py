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
    # default options: RoBERTa's layout chosen at load time from the LayerNorm parameters (|beta| +
    # sqrt(767) |gamma| = 900+ here -> the split hi + lo stream), or the precise mode when the
    # calibration sees the split stream move a score by > 5e-4; the CLIP streams by their load-time
    # calibration (any choice must meet the bar below)
    print(f"RoBERTa calibration on the outlier draw: {eng.text_check}")
    assert eng.text_check["fast_layout"] == "split"
    assert eng.get_option("text_hilo_effective") == (2 if eng.text_check["mode"] == "precise" else 1)
    print(f"CLIP stream check on the outlier draw: {eng.clip_stream_check}")
    assert eng.get_option("clip_res16") == int(eng.clip_stream_check["fp16_streams"])
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
    mode = eng.get_option("text_hilo")
    eng.set_option("text_hilo", 0)
    o16 = eng.analyze_batch(rid, rm, cid, cm, imgs)["scores"].cpu().numpy()
    eng.set_option("text_hilo", mode)
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


DOM_CH = 301  # the dominating RoBERTa channel of the gamma draw


def dominating_gamma_state(det, gamma_out=3.5, kappa=3.5, emb_scale=30.0, seed_level=60.0):
    """VERDICT r3 item 2's draw: beta ~ 0 in every LayerNorm and a large gamma (`gamma_out`) in ONE
    channel that dominates the LayerNorm statistics -- the case the round-3 bound (|beta| + 4 |gamma|)
    missed.  The word embeddings carry a constant `seed_level` in the channel (normal channels scaled
    to std 0.6), so the embedding LayerNorm's xhat there is near its sqrt(767) ceiling, and every
    later LayerNorm sees the channel dominating again: the post-LN stream settles at ~82 (gamma 3.5)
    / ~113 (gamma 5) / ~151 (gamma 7) in that channel in every layer (the test reads the level from
    the oracle).  As in trained models the normal channels' gamma carries the compensating scale (`kappa`,
    here equal to gamma_out, which keeps them alive: rows differ by O(1)) and the weight columns
    reading the channel are x0.01.  max |beta| + 4 |gamma| stays at 17 / 24 / 33, under the 64
    threshold: the round-3 guard picked the fp16-only stream for it."""
    det = {k: np.array(v, copy=True) for k, v in det.items()}
    c = DOM_CH
    nm = np.ones(768, bool)
    nm[c] = False
    det["roberta.embeddings.word_embeddings.weight"][:, nm] *= emb_scale
    det["roberta.embeddings.word_embeddings.weight"][:, c] += seed_level
    for ln in ["roberta.embeddings.LayerNorm"] + [f"roberta.encoder.layer.{i}.{n}" for i in range(12)
                                                  for n in ("attention.output.LayerNorm", "output.LayerNorm")]:
        det[ln + ".weight"][nm] *= kappa
        det[ln + ".weight"][c] = gamma_out
        det[ln + ".bias"][:] = np.clip(det[ln + ".bias"], -0.02, 0.02)  # beta ~ 0
    for i in range(12):
        p = f"roberta.encoder.layer.{i}."
        for w in ("attention.self.query", "attention.self.key", "attention.self.value", "intermediate.dense"):
            det[p + w + ".weight"][:, c] *= 0.01
    for h in ("ai_head", "misinfo_head"):
        det[f"{h}.0.weight"][:, c] *= 0.01
    return det


def _ln_bound(det, xhat):
    return max(float((np.abs(det[k[:-6] + "bias"]) + xhat * np.abs(v)).max())
               for k, v in det.items() if k.startswith("roberta") and k.endswith("LayerNorm.weight"))


@pytest.mark.parametrize("gamma_out,mode", [(3.5, "split"), (5.0, "precise")])
def test_dominating_gamma_channel_calibration(det_sd, clip_sd, gamma_out, mode):
    """The sound bound |beta| + sqrt(767) |gamma| selects the split hi + lo stream as the fast layout
    on a draw whose post-LN stream is ~82 / ~113 in one dominating channel with beta ~ 0 (the
    round-3 bound, 17 / 24, did not); the calibration then keeps it at gamma 3.5 (2.9e-4 from the
    precise mode) and selects the precise mode at gamma 5 (6.9e-4, round 5), and the full-size
    scores and probabilities stay within 1e-3 of the oracle (the exact mode is asserted).  (At
    gamma 7 -- stream ~151 -- the split stream measured 1.6e-3 / 1.1e-3 and fp16-only 2.7e-3 / 3.6e-3:
    that draw amplifies the fp16 rounding of the GEMM operands themselves -- the oracle with only its
    encoder weights rounded to fp16 moves by 5e-4 there, 3e-5 on the plain draw -- which no stream
    layout removes)"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle import models as M
    from oracle.pipeline import batched_scores
    det = dominating_gamma_state(det_sd, gamma_out, kappa=gamma_out)
    assert _ln_bound(det, 4.0) < 64.0 < _ln_bound(det, np.sqrt(767.0))
    Bf = 256
    eng = Engine(0, det, clip_sd, max_batch=Bf)
    print(f"RoBERTa calibration: {eng.text_check}")
    assert eng.text_check["fast_layout"] == "split"  # the bound alone already leaves the fp16-only stream
    assert eng.text_check["mode"] == mode
    assert eng.get_option("text_hilo_effective") == {"split": 1, "precise": 2}[mode]
    rid, rm = syn.roberta_ids(Bf, 128, 1234)
    cid, cm = syn.clip_ids(Bf, 77, 1234)
    imgs = syn.images(Bf, 1234)
    vault = syn.vault(2170, 512, 77)
    eng.set_vault(vault)
    out = eng.analyze_batch(rid, rm, cid, cm, imgs)
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    with torch.no_grad():
        ref = batched_scores(det, clip_sd, rid, rm, cid, cm, imgs, vault)
        sd = M.to_torch(det)
        cls = M.roberta_forward(sd, torch.as_tensor(rid[:4]).long(), torch.as_tensor(rm[:4]).long())[:, 0]
    lvl = float(cls[:, DOM_CH].abs().min())
    rest = cls[:, [c for c in range(768) if c != DOM_CH]]
    print(f"dominating channel draw (gamma {gamma_out}): stream level {lvl:.1f}, rest std {float(rest.std()):.2f}")
    assert 70.0 < lvl < 200.0 and lvl > 4.0 * gamma_out * 4  # the draw does what it claims
    assert float(rest.std()) > 0.3 and float((cls[0] - cls[1]).abs().max()) > 0.1
    d = np.abs(got["scores"] - ref["scores"]).max(0)
    mode = eng.get_option("text_hilo")
    eng.set_option("text_hilo", 0)
    o16 = eng.analyze_batch(rid, rm, cid, cm, imgs)["scores"].cpu().numpy()
    eng.set_option("text_hilo", mode)
    print(f"  selected ({eng.text_check['mode']}): ai {d[0]:.2e} misinfo {d[1]:.2e}; fp16-only stream: ai "
          f"{np.abs(o16[:, 0] - ref['scores'][:, 0]).max():.2e} misinfo {np.abs(o16[:, 1] - ref['scores'][:, 1]).max():.2e}")
    np.testing.assert_allclose(got["scores"], ref["scores"], atol=1e-3)
    np.testing.assert_allclose(got["probs"], ref["probs"], atol=1e-3)
    eng.close()


def overflow_clip_state(clip_sd, step=7000.0):
    """FFN-2 biases of +`step` per layer in 2 text-tower channels: the pre-LN stream passes fp16's
    range (~8e4) by the last layer."""
    clip = {k: np.array(v, copy=True) for k, v in clip_sd.items()}
    c, H = list(TXT_CH), 512
    nm = np.ones(H, bool)
    nm[c] = False
    for i in range(12):
        p = f"text_model.encoder.layers.{i}."
        clip[p + "mlp.fc2.bias"][c] += step
        g = max(1.0, step * i * np.sqrt(len(c) / H))
        for ln in ("layer_norm1", "layer_norm2"):
            clip[p + ln + ".weight"][nm] *= g
            clip[p + ln + ".weight"][c] = 0.05
    clip["text_model.final_layer_norm.weight"][nm] *= step * 12 * np.sqrt(len(c) / H)
    clip["text_model.final_layer_norm.weight"][c] = 0.05
    return clip


def test_clip_runtime_overflow_trap(det_sd, clip_sd):
    """the load-time CLIP calibration is a measurement on 8 inputs, not a bound.  If an
    input overflows the fp16 streams after it passed (simulated here by forcing clip_res16 = 1 on the
    overflow draw), the synchronous API paths see the non-finite CLIP output, switch the engine to
    fp32 streams and re-run: analyze_pairs / analyze_consistency return the fp32-stream values."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.api import MisinfoForensics
    clip = overflow_clip_state(clip_sd)
    n = 6
    texts, rob, clp = syn.text_tables(n, 91)
    from PIL import Image
    imgs = [Image.fromarray(a) for a in syn.images(n, 91)]

    def mk():
        return MisinfoForensics(fusion_weights="", faiss_index_path="", detector_state=det_sd, clip_state=clip,
                                roberta_tokenizer=rob, clip_processor=clp, max_batch=8, verbose=False)
    ref = mk()
    assert ref.engine.get_option("clip_res16") == 0  # the calibration catches this draw
    want = [d["scores"]["clip_similarity"] for d in ref.analyze_pairs(texts, imgs)]
    want1 = ref.analyze_consistency(texts[0], imgs[0])["clip_similarity"]
    ref.engine.close()
    mf = mk()
    mf.engine.set_option("clip_res16", 1)  # as if the calibration inputs had not overflowed
    got = [d["scores"]["clip_similarity"] for d in mf.analyze_pairs(texts, imgs)]
    print(f"runtime trap: {mf.engine.clip_stream_check}")
    assert mf.engine.get_option("clip_res16") == 0 and mf.engine.clip_stream_check["runtime_overflow"]
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, want, atol=1e-6)
    mf.engine.set_option("clip_res16", 1)
    got1 = mf.analyze_consistency(texts[0], imgs[0])["clip_similarity"]
    assert np.isfinite(got1) and abs(got1 - want1) < 1e-6 and mf.engine.get_option("clip_res16") == 0
    mf.engine.close()


def test_gamma7_draw_selects_precise_mode(det_sd, clip_sd):
    """the gamma = 7 dominating-channel draw (post-LN stream ~151 in the channel),
    where the split stream misses the bar (1.6e-3 / 1.1e-3: the fp16 rounding of the GEMM operands
    themselves is amplified by every LayerNorm).  Under DEFAULT options the load-time calibration
    must select the precise mode (~22-bit GEMM operands, fp32 stream / LayerNorm / attention), and
    the full-size scores and probabilities meet 1e-3 against the oracle at B = 256."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle.pipeline import batched_scores
    det = dominating_gamma_state(det_sd, 7.0, kappa=7.0)
    Bf = 256
    eng = Engine(0, det, clip_sd, max_batch=Bf)
    print(f"RoBERTa calibration (gamma 7): {eng.text_check}")
    assert eng.text_check["mode"] == "precise" and eng.get_option("text_hilo_effective") == 2
    # round 6: the calibration keeps only the GEMM kinds that need hi / lo operands (the rest read
    # fp16 operands; their precise weights are released)
    m = eng.text_check["prec_mask"]
    assert eng.get_option("text_prec_mask") == m and eng.get_option("text_precise_packed") == m & 15
    rid, rm = syn.roberta_ids(Bf, 128, 1234)
    cid, cm = syn.clip_ids(Bf, 77, 1234)
    imgs = syn.images(Bf, 1234)
    vault = syn.vault(2170, 512, 77)
    eng.set_vault(vault)
    got = {k: v.cpu().numpy() for k, v in eng.analyze_batch(rid, rm, cid, cm, imgs).items()}
    with torch.no_grad():
        ref = batched_scores(det, clip_sd, rid, rm, cid, cm, imgs, vault)
    d = np.abs(got["scores"] - ref["scores"]).max(0)
    eng.set_option("text_hilo", 1)
    o1 = eng.analyze_batch(rid, rm, cid, cm, imgs)["scores"].cpu().numpy()
    eng.set_option("text_hilo", 2)
    print(f"  precise mode: ai {d[0]:.2e} misinfo {d[1]:.2e}, probs {np.abs(got['probs'] - ref['probs']).max():.2e}; "
          f"split stream: ai {np.abs(o1[:, 0] - ref['scores'][:, 0]).max():.2e} "
          f"misinfo {np.abs(o1[:, 1] - ref['scores'][:, 1]).max():.2e}")
    np.testing.assert_allclose(got["scores"], ref["scores"], atol=1e-3)
    np.testing.assert_allclose(got["probs"], ref["probs"], atol=1e-3)
    eng.close()


def test_clip_stream_overflow_selects_fp32_streams(det_sd, clip_sd):
    """CLIP's pre-LN streams have no parameter bound, so the engine measures them at load
    (Engine.check_clip_streams).  A draw whose text-tower stream passes fp16's range (FFN-2 biases
    of +7000 per layer in 2 channels: ~8e4 by the last layer) must fall back to fp32 streams and
    match the oracle; the plain draw keeps the fp16 streams."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle.pipeline import batched_scores
    plain = Engine(0, det_sd, clip_sd, max_batch=8)
    chk = plain.clip_stream_check
    print(f"plain draw: {chk}")
    assert chk["fp16_streams"] and plain.get_option("clip_res16") == 1
    plain.close()
    clip = overflow_clip_state(clip_sd)
    Bf = 64
    eng = Engine(0, det_sd, clip, max_batch=Bf)
    chk = eng.clip_stream_check
    print(f"overflow draw: {chk}")
    assert not chk["fp16_streams"] and eng.get_option("clip_res16") == 0
    rid, rm = syn.roberta_ids(Bf, 128, 77)
    cid, cm = syn.clip_ids(Bf, 77, 77)
    imgs = syn.images(Bf, 77)
    vault = syn.vault(2170, 512, 77)
    eng.set_vault(vault)
    got = {k: v.cpu().numpy() for k, v in eng.analyze_batch(rid, rm, cid, cm, imgs).items()}
    with torch.no_grad():
        ref = batched_scores(det_sd, clip, rid, rm, cid, cm, imgs, vault)
    assert np.isfinite(got["scores"]).all()
    np.testing.assert_allclose(got["scores"], ref["scores"], atol=1e-3)
    np.testing.assert_allclose(got["probs"], ref["probs"], atol=1e-3)
    eng.close()
