"""Pin the CPU oracle against the fixtures the reference code itself produced
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

import mmf_amd.weights as W
from oracle import models as M
from oracle import pipeline as P

torch.set_num_threads(8)
TOL_F32 = 2e-4  # fp32 restatement vs HF/numpy reference: reduction-order noise only


def test_state_dict_structure():
    # torchvision EfficientNet-B0 published parameter count at 1000 classes
    assert W.param_count(W.effnet_spec(num_classes=1000)) == 5_288_548
    assert W.param_count(W.effnet_spec()) == 4_010_110
    assert len(W.effnet_spec()) == 360
    assert W.param_count(W.roberta_spec()) == 124_645_632
    assert W.param_count(W.clip_spec()) == 151_277_313


def test_roberta_cls_and_heads(golden, golden_inputs, det_sd):
    sd = M.to_torch(det_sd)
    ids = torch.as_tensor(golden["rob_ids"])
    mask = torch.as_tensor(golden["rob_mask"])
    h = M.roberta_forward(sd, ids, mask)           # batched + padded to 128
    cls = h[:, 0, :]
    np.testing.assert_allclose(cls.numpy(), golden["cls_hidden"], atol=TOL_F32, rtol=0)
    ai, mi = M.text_heads(sd, cls)
    np.testing.assert_allclose(ai.numpy(), golden["ai_logits"], atol=TOL_F32, rtol=0)
    np.testing.assert_allclose(mi.numpy(), golden["misinfo_logits"], atol=TOL_F32, rtol=0)


def test_effnet_vs_reference_run(golden, golden_inputs, det_sd):
    sd = M.to_torch(det_sd)
    x = M.effnet_preprocess(torch.as_tensor(golden_inputs["imgs"]))
    np.testing.assert_allclose(M.effnet_forward(sd, x).numpy(), golden["effnet_logits"], atol=1e-3, rtol=1e-4)


def test_clip_embeddings(golden, golden_inputs, clip_sd):
    csd = M.to_torch(clip_sd)
    img = M.clip_image_features(csd, M.clip_preprocess(torch.as_tensor(golden_inputs["imgs"])))
    np.testing.assert_allclose(img.numpy(), golden["clip_image_features_raw"], atol=TOL_F32, rtol=0)
    np.testing.assert_allclose(M.l2n(img).numpy(), golden["clip_image_embeds"], atol=TOL_F32, rtol=0)
    txt = M.clip_text_features(csd, torch.as_tensor(golden["clip_ids"]), torch.as_tensor(golden["clip_mask"]),
                               golden_inputs["eos"])
    np.testing.assert_allclose(M.l2n(txt).numpy(), golden["clip_text_embeds"], atol=TOL_F32, rtol=0)
    sim = (M.l2n(img) * M.l2n(txt)).sum(-1)
    np.testing.assert_allclose(sim.numpy(), golden["clip_similarity"], atol=TOL_F32, rtol=0)


def test_clip_eos_rules():
    ids = torch.tensor([[49406, 5, 7, 49407, 49407], [49406, 49407, 49407, 49407, 49407]])
    assert M.clip_eos_index(ids, 49407).tolist() == [3, 1]
    assert M.clip_eos_index(ids, 2).tolist() == [3, 1]   # argmax picks the first max


def test_batched_pipeline(golden, golden_inputs, det_sd, clip_sd):
    gi = golden_inputs
    csd = M.to_torch(clip_sd)
    tid = np.zeros((2170, 77), np.int32) + 49407
    tmask = np.zeros((2170, 77), np.int32)
    for j, t in enumerate(gi["title_ids"]):
        tid[j, :len(t)] = t
        tmask[j, :len(t)] = 1
    # title embeddings only for the rows that can be a top-1 hit (keeps the CPU test fast)
    rows = sorted(set(golden["vault_top_idx"][:, 0].tolist()))
    temb = np.zeros((2170, 512), np.float32)
    temb[rows] = M.l2n(M.clip_text_features(csd, torch.as_tensor(tid[rows]), torch.as_tensor(tmask[rows]),
                                            gi["eos"])).numpy()
    out = P.batched_scores(det_sd, clip_sd, golden["rob_ids"], golden["rob_mask"], golden["clip_ids"],
                           golden["clip_mask"], gi["imgs"], gi["vault"], gi["eos"], temb)
    np.testing.assert_array_equal(out["top_idx"], golden["vault_top_idx"])
    np.testing.assert_allclose(out["top_sim"], golden["vault_top_sim"], atol=TOL_F32)
    np.testing.assert_allclose(out["text_similarity"], golden["text_similarity"], atol=TOL_F32)
    np.testing.assert_allclose(out["scores"], golden["scores"], atol=1e-4)
    np.testing.assert_allclose(out["probs"], golden["fusion_probs"], atol=1e-4)


def test_fusion_config1(golden, det_sd):
    sd = M.to_torch(det_sd)
    p = torch.softmax(P.fusion_logits(sd, torch.as_tensor(golden["fusion_c1_inputs"])), 1)
    np.testing.assert_allclose(p.numpy(), golden["fusion_c1_probs"], atol=1e-6)


def test_fusion_verdict_dicts(golden, golden_json, det_sd):
    sd = M.to_torch(det_sd)
    keys = ("ai_score", "misinfo_score", "deepfake_score", "clip_similarity", "vault_discrepancy")
    for i, ref in enumerate(golden_json["fusion_verdicts"]):
        got = P.fusion_verdict(sd, dict(zip(keys, map(float, golden["fusion_c1_inputs"][i]))))
        assert got["verdict"] == ref["verdict"]
        for k in ("confidence", "fake_probability", "real_probability"):
            assert abs(got[k] - ref[k]) < 1e-6


def test_explanations_exact(golden_json):
    for case in golden_json["explanations"]:
        assert P.explanation(case["scores"], [{"title": "Planted title"}]) == case["text"]


@pytest.fixture(scope="module")
def oracle_forensics(golden, golden_inputs, det_sd, clip_sd):
    gi = golden_inputs
    return P.OracleForensics(det_sd, clip_sd, gi["vault"], gi["meta"], gi["title_ids"], gi["eos"])


def _text(golden, gi, i):
    return (golden["rob_ids"][i, :gi["rob_lens"][i]], golden["clip_ids"][i, :gi["clip_lens"][i]])


def _check_dict(got, ref, tol=2e-4):
    assert got["verdict"] == ref["verdict"] and got["verdict_text"] == ref["verdict_text"]
    assert abs(got["confidence"] - ref["confidence"]) < tol
    for k, v in ref["scores"].items():
        assert abs(got["scores"][k] - v) < tol, (k, got["scores"][k], v)
    assert [m["title"] for m in got["vault_matches"]] == [m["title"] for m in ref["vault_matches"]]
    for a, b in zip(got["vault_matches"], ref["vault_matches"]):
        assert abs(a["similarity"] - b["similarity"]) < tol and a["url"] == b["url"] and a["date"] == b["date"]
    assert got["explanation"] == ref["explanation"]


@pytest.mark.parametrize("i", [0, 1, 3])
def test_analyze_dict_pairs(i, golden, golden_json, golden_inputs, oracle_forensics):
    got = oracle_forensics.analyze(text=_text(golden, golden_inputs, i), image=golden_inputs["imgs"][i])
    _check_dict(got, golden_json["analyze"][i])


def test_analyze_single_modality(golden, golden_json, golden_inputs, oracle_forensics):
    for n, i in enumerate((0, 1)):
        _check_dict(oracle_forensics.analyze(text=_text(golden, golden_inputs, i)), golden_json["analyze_text_only"][n])
    for n, i in enumerate((2, 3)):
        _check_dict(oracle_forensics.analyze(image=golden_inputs["imgs"][i]), golden_json["analyze_image_only"][n])
    with pytest.raises(ValueError) as e:
        oracle_forensics.analyze()
    assert str(e.value) == golden_json["analyze_no_input_error"]
