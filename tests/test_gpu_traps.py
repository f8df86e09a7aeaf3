"""Run-time precision traps of the fast towers.

The load-time calibration (Engine.check_text_precision / check_effnet_precision) measures seeded
inputs; it bounds nothing for an input that drives an fp16 activation past 65504.  Each draw here is
"otherwise calibrated" -- the calibration keeps the fast tower -- but carries a channel that one
specific input overflows: a saturated colour on a high-gain EfficientNet stem channel, a rare token
on a RoBERTa FFN row.  In both draws the overflowing channel feeds the rest of the network through a
zero weight, so a finite value contributes exactly 0 and only inf (inf x 0 = NaN) changes the
output: the forced fast tower returns a NaN score for that input alone, and the synchronous API paths
must switch the tower (fp32 EfficientNet tower; RoBERTa precise mode with fp32 stream and branch
outputs) and return the values of that path to 1e-6.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

STEM_GAIN = 2640.0  # 2x2 checker taps: a 0/255 checkerboard gives 26.55 x 2640 = 70.1k > 65504
TOK, DIM, OUT_CH = 50000, 100, 200  # RoBERTa: the rare token, its embedding direction, the FFN-2 row


def overflow_effnet_state(det):
    """Stem channel 0 is a zero-sum 2x2 checker filter (+g, -g / -g, +g on every colour plane, gain
    STEM_GAIN, BN identity): smooth content and the synthetic images' noise stay below ~48k, a
    pixel-level 0/255 checkerboard reaches 70k.  The stage-1 depthwise weight of channel 0 is zero,
    so only an inf in that channel reaches the logits (inf x 0 = NaN)."""
    det = {k: np.array(v, copy=True) for k, v in det.items()}
    w = det["efficientnet.features.0.0.weight"]
    w[0] = 0.0
    w[0, :, 0, 0] = w[0, :, 1, 1] = STEM_GAIN
    w[0, :, 0, 1] = w[0, :, 1, 0] = -STEM_GAIN
    bn = "efficientnet.features.0.1."
    det[bn + "weight"][0], det[bn + "bias"][0] = 1.0, 0.0
    det[bn + "running_mean"][0], det[bn + "running_var"][0] = 0.0, 1.0
    det["efficientnet.features.1.0.block.0.0.weight"][0] = 0.0
    return det


def checkerboard():
    yy, xx = np.mgrid[0:224, 0:224]
    img = np.zeros((224, 224, 3), np.uint8)
    img[(yy + xx) % 2 == 0] = 255
    return img


def stem_ch0_max(det, imgs):
    """max |stem channel-0 pre-activation| over uint8 images [N,224,224,3] (fp32, CPU)."""
    from oracle import models as M
    x = M.effnet_preprocess(torch.as_tensor(imgs))
    w = torch.as_tensor(det["efficientnet.features.0.0.weight"][:1])
    return float(torch.nn.functional.conv2d(x, w, stride=2, padding=1).abs().max())


def overflow_text_state(det):
    """Token TOK's embedding points along DIM (LayerNorm: ~27.7 there); layer 0's FFN-1 rows 0..63
    read only DIM with bias -400 (every other token: GELU(<= -200) = 0 exactly; TOK: 708), and FFN-2
    row OUT_CH sums those 64 at weight 2: 90.6k for TOK -- finite in fp32, inf in an fp16 store."""
    det = {k: np.array(v, copy=True) for k, v in det.items()}
    det["roberta.embeddings.word_embeddings.weight"][TOK, DIM] = 30.0
    p = "roberta.encoder.layer.0."
    w1, b1 = det[p + "intermediate.dense.weight"], det[p + "intermediate.dense.bias"]
    w1[:64] = 0.0
    w1[:64, DIM] = 40.0
    b1[:64] = -400.0
    det[p + "output.dense.weight"][OUT_CH, :64] = 2.0
    return det


def _mk(det, clip_sd, texts=None, rob=None, clp=None):
    from mmf_amd.api import MisinfoForensics
    return MisinfoForensics(fusion_weights="", faiss_index_path="", detector_state=det, clip_state=clip_sd,
                            roberta_tokenizer=rob, clip_processor=clp, max_batch=8, verbose=False)


def test_effnet_runtime_overflow_trap(det_sd, clip_sd):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from PIL import Image
    det = overflow_effnet_state(det_sd)
    n = 4
    texts, rob, clp = syn.text_tables(n, 93)
    arrs = syn.images(n, 93)
    arrs[1] = checkerboard()  # the trigger image
    # the draw does what it claims: the calibration images and the other inputs stay in fp16's
    # range in the channel, the checkerboard leaves it
    cal_max = max(stem_ch0_max(det, syn.images(64, 5003)[i:i + 16]) for i in range(0, 64, 16))
    print(f"stem channel 0: calibration max {cal_max:.0f}, checkerboard {stem_ch0_max(det, arrs[1:2]):.0f}")
    assert cal_max < 60000.0 and stem_ch0_max(det, arrs[[0, 2, 3]]) < 60000.0
    assert stem_ch0_max(det, arrs[1:2]) > 66000.0
    imgs = [Image.fromarray(a) for a in arrs]
    mf = _mk(det, clip_sd, texts, rob, clp)
    print(f"calibration: {mf.engine.effnet_check}")
    assert mf.engine.effnet_check["tower"] == "fp16"  # an otherwise calibrated draw
    s16 = mf.engine.effnet_forward(arrs)[1].cpu().numpy()
    print(f"forced fp16 tower: {s16}")
    assert not np.isfinite(s16[1]) and np.isfinite(s16[[0, 2, 3]]).all()  # the overflow is input-driven
    # the fp32 tower's values (what the trap must return)
    mf.engine.set_option("effnet_fp32", 1)
    want = mf.engine.effnet_forward(arrs)[1].cpu().numpy()
    want_pairs = [d["scores"] for d in mf.analyze_pairs(texts, imgs)]
    mf.engine.set_option("effnet_fp32", 0)
    mf.engine._auto_set["effnet_fp32"] = 0  # (back to the calibrated state: not a user pin)
    got = mf.analyze_image(imgs[1])["deepfake_score"]
    assert mf.engine.get_option("effnet_fp32") == 1 and mf.engine.effnet_check["runtime_overflow"]
    assert np.isfinite(got) and abs(got - want[1]) < 1e-6
    mf.engine.set_option("effnet_fp32", 0)
    mf.engine._auto_set["effnet_fp32"] = 0
    got_pairs = [d["scores"] for d in mf.analyze_pairs(texts, imgs)]
    assert mf.engine.get_option("effnet_fp32") == 1
    for g, w in zip(got_pairs, want_pairs):
        for k in ("ai_score", "misinfo_score", "deepfake_score", "clip_similarity", "fake_probability"):
            assert np.isfinite(g[k]) and abs(g[k] - w[k]) < 1e-6, (k, g[k], w[k])
    mf.engine.close()


def test_text_runtime_overflow_trap(det_sd, clip_sd):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from PIL import Image
    det = overflow_text_state(det_sd)
    cal, _ = syn.roberta_ids(64, 128, 6007, [128, 64, 17, 5])
    assert not (cal == TOK).any()  # the calibration texts do not contain the token
    n = 4
    texts, rob, clp = syn.text_tables(n, 94)
    rid, _ = syn.roberta_ids(n, 128, 94)
    rid = rid.tolist()
    assert TOK not in sum(rid, [])
    rid[2][40] = TOK  # text 2 carries the rare token
    from mmf_amd.synthetic import IdTableTokenizer
    rob = IdTableTokenizer({t: rid[i] for i, t in enumerate(texts)}, 1)
    imgs = [Image.fromarray(a) for a in syn.images(n, 94)]
    mf = _mk(det, clip_sd, texts, rob, clp)
    chk = mf.engine.text_check
    print(f"calibration: {chk}")
    assert chk["mode"] in ("fp16", "split") and mf.engine.get_option("text_hilo_effective") < 2
    assert mf.engine.get_option("text_precise_packed") == 0  # released with the fast layout
    ids = np.array(rid, np.int32)
    fast = mf.engine.text_forward(ids, np.ones_like(ids))[2].cpu().numpy()
    print(f"forced fast layout: {fast}")
    assert not np.isfinite(fast[2]).all() and np.isfinite(fast[[0, 1, 3]]).all()
    # the precise mode on fp16 operands (text_prec_mask 0: what the trap selects once the calibration
    # released the hi / lo weights)
    mf.engine.set_option("text_prec_mask", 0)
    mf.engine.set_option("text_hilo", 2)
    want = mf.engine.text_forward(ids, np.ones_like(ids))[2].cpu().numpy()
    want_pairs = [d["scores"] for d in mf.analyze_pairs(texts, imgs)]
    mf.engine._auto_write("text_hilo", -1)
    got = mf.analyze_text(texts[2])
    assert mf.engine.get_option("text_hilo_effective") == 2 and mf.engine.text_check["runtime_overflow"]
    assert abs(got["ai_score"] - want[2, 0]) < 1e-6 and abs(got["misinfo_score"] - want[2, 1]) < 1e-6
    mf.engine._auto_write("text_hilo", -1)
    got_pairs = [d["scores"] for d in mf.analyze_pairs(texts, imgs)]
    assert mf.engine.get_option("text_hilo_effective") == 2
    for g, w in zip(got_pairs, want_pairs):
        for k in ("ai_score", "misinfo_score", "deepfake_score", "clip_similarity", "fake_probability"):
            assert np.isfinite(g[k]) and abs(g[k] - w[k]) < 1e-6, (k, g[k], w[k])
    mf.engine.close()
