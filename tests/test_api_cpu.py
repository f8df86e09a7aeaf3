"""CPU checks of the drop-in API's host logic (no GPU): state-dict contract, fusion-training
compatibility, explanation strings, vault file formats, image geometry, loud failure without HIP."""
import io
import os
import pickle

import numpy as np
import pytest
import torch

import mmf_amd.weights as W
from mmf_amd import explain, io_utils


def test_detector_state_dict_contract():
    from misinfo_forensics import MultiModalMisinfoDetector
    det = MultiModalMisinfoDetector()
    sd = det.state_dict()
    spec = W.detector_spec()
    assert list(sd.keys()) == list(spec.keys()) or set(sd.keys()) == set(spec.keys())
    for k, (shape, _) in spec.items():
        assert tuple(sd[k].shape) == tuple(shape), k
    # reference-style strict load of a synthetic full_model_state_dict
    det.load_state_dict({k: torch.as_tensor(v) for k, v in W.synthetic_detector_state(0).items()}, strict=True)


def test_fusion_training_path(golden):
    """train_fusion_judge.py:141-227: freeze all but fusion_layer, AdamW on forward_fusion."""
    from misinfo_forensics import MultiModalMisinfoDetector
    det = MultiModalMisinfoDetector()
    det.load_state_dict({k: torch.as_tensor(v) for k, v in W.synthetic_detector_state(0).items()})
    x = torch.as_tensor(golden["fusion_c1_inputs"][:64])
    det.eval()  # Dropout(0.2) inert, as in the reference's inference path
    with torch.no_grad():
        p = torch.softmax(det.forward_fusion(x), 1)
    np.testing.assert_allclose(p.numpy(), golden["fusion_c1_probs"][:64], atol=1e-6)
    for name, prm in det.named_parameters():
        prm.requires_grad = "fusion_layer" in name
    opt = torch.optim.AdamW([q for q in det.fusion_layer.parameters()], lr=1e-2)
    y = torch.randint(0, 2, (64,))
    before = det.fusion_layer[0].weight.clone()
    loss = torch.nn.functional.cross_entropy(det.forward_fusion(x), y)
    loss.backward()
    opt.step()
    assert not torch.equal(before, det.fusion_layer[0].weight)
    assert dict(det.named_parameters())["roberta.encoder.layer.0.attention.self.query.weight"].grad is None


def test_explanations_match_reference(golden_json):
    for case in golden_json["explanations"]:
        assert explain.fallback_explanation(case["scores"], [{"title": "Planted title"}]) == case["text"]
    for c in golden_json["clip_engine_explanations"]:
        assert explain.clip_engine_explanation(c["similarity"], c["label"]) == c["text"]
    for r in golden_json["analyze"]:
        rule = explain.explanation_rule(r["scores"])
        assert explain.fallback_explanation(r["scores"], r["vault_matches"], rule) == r["explanation"]


def test_gemini_prompt_mentions_scores(golden_json):
    r = golden_json["analyze"][0]
    p = explain.gemini_prompt(r["scores"], r["vault_matches"])
    assert "FORENSIC ANALYSIS SCORES" in p and r["vault_matches"][0]["title"] in p


def test_vault_formats(tmp_path):
    emb = np.random.default_rng(0).standard_normal((5, 512)).astype(np.float32)
    a = {"article_ids": list(range(5)), "text_contents": [f"t{i}" for i in range(5)],
         "image_paths": [f"p{i}.jpg" for i in range(5)], "image_embeddings": emb, "text_embeddings": emb,
         "metadata": {"model": "clip"}}
    pa = tmp_path / "a.pkl"
    pa.write_bytes(pickle.dumps(a))
    e, m = io_utils.load_vault(str(pa))
    np.testing.assert_array_equal(e, emb)
    assert m[3] == {"title": "t3", "url": "p3.jpg", "date": "N/A"}
    b = {"embeddings": emb, "metadata": [{"title": f"x{i}", "url": "u", "date": "d"} for i in range(5)]}
    pb = tmp_path / "b.pkl"
    pb.write_bytes(pickle.dumps(b))
    e, m = io_utils.load_vault(str(pb))
    assert m[1]["title"] == "x1"
    pc = tmp_path / "c.pkl"
    pc.write_bytes(pickle.dumps({"foo": 1}))
    assert io_utils.load_vault(str(pc)) == (None, None)


def test_vault_loader_executes_nothing(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps({"embeddings": Evil(), "metadata": []}))
    with pytest.raises(pickle.UnpicklingError):
        io_utils.load_vault(str(p))


def test_image_geometry_matches_hf_processor():
    from PIL import Image
    from transformers import CLIPImageProcessor
    from oracle import models as M
    rng = np.random.default_rng(1)
    for (w, h) in ((224, 224), (300, 200), (180, 260)):
        img = Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
        ref = CLIPImageProcessor()(images=img, return_tensors="pt")["pixel_values"]
        got = M.clip_preprocess(torch.as_tensor(io_utils.clip_pixels(img)[None]))
        assert got.shape == ref.shape
        np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=1e-5)
        assert io_utils.effnet_pixels(img).shape == (224, 224, 3)


def test_api_fails_loudly_without_hip():
    from misinfo_forensics import MisinfoForensics
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    with pytest.raises(RuntimeError, match="HIP device"):
        MisinfoForensics(synthetic_seed=0, device="cpu", verbose=False)


def test_video_frame_sampling_matches_reference():
    """sample_video_frames (misinfo_forensics.py:501-548 sampling) against the frames the reference
    itself consumed in tests/golden/golden_video.json (best frame + errors), cv2 replaced by the
    frame-replay stub; and the reference's error without OpenCV."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import cv2_stub
    import video_fixture as VF
    import mmf_amd.synthetic as syn
    from mmf_amd.api import sample_video_frames
    saved = sys.modules.pop("cv2", None)
    try:
        with pytest.raises(RuntimeError) as e:
            sample_video_frames("v_stride.mp4")
        assert "opencv-python is required for video analysis" in str(e.value)
        imgs = syn.images(8, 1234)
        cv2_stub.install(VF.bgr_videos(imgs))
        with open(os.path.join(os.path.dirname(__file__), "golden", "golden_video.json")) as f:
            gv = json.load(f)
        for c in gv["calls"]:
            frames = sample_video_frames(c["video"], c["max_frames"], c["stride_seconds"])
            fps = VF.VIDEOS[c["video"]]["fps"] or 25.0
            stride = max(1, int(round(fps * max(0.1, c["stride_seconds"]))))
            want = VF.VIDEOS[c["video"]]["frames"][::stride][:c["max_frames"]]
            assert len(frames) == len(want)
            for fr, s in zip(frames, want):
                assert np.array_equal(np.asarray(fr), imgs[s])
            assert c["result"]["best_frame_sample"] in want
        assert sample_video_frames("v_empty.mp4") == []
        with pytest.raises(RuntimeError) as e:
            sample_video_frames("missing.mp4")
        assert str(e.value) == gv["errors"]["missing.mp4"]
    finally:
        sys.modules.pop("cv2", None)
        if saved is not None:
            sys.modules["cv2"] = saved


def test_fingerprint_sees_dtype_round_trip():
    """.half() then .float() re-creates every tensor without bumping a version counter
    and could land on the packed state's old addresses.  The detector holds the storages of its
    last packed state, so the round trip always reads as stale (-> re-packed before the next call)."""
    from mmf_amd.api import MultiModalMisinfoDetector, ALL_COMPONENTS
    det = MultiModalMisinfoDetector()
    for c in ALL_COMPONENTS:  # what sync() records after packing a component
        det._synced[c] = det._fingerprint(c)
        det._held[c] = [t.untyped_storage() for t in det._tensors[c]]
    assert det.stale_components() == []
    det.fusion_layer.half()
    det.fusion_layer.float()
    assert det.stale_components() == ["fusion"]
    with torch.no_grad():
        det.ai_head[0].bias.add_(1.0)  # in place: version counter
    assert det.stale_components() == ["text", "fusion"]


def test_clip_eos_token_id_from_config(tmp_path, monkeypatch):
    """The EOS id the CLIP text tower pools at comes from text_config.eos_token_id of the CLIP
    config in clip_model_dir; env override first, 49407 without a config."""
    from transformers import CLIPConfig
    from mmf_amd.api import clip_eos_token_id
    monkeypatch.delenv("MMF_CLIP_EOS_TOKEN_ID", raising=False)
    CLIPConfig(text_config={"eos_token_id": 2}).save_pretrained(tmp_path)
    assert clip_eos_token_id(str(tmp_path)) == 2
    assert clip_eos_token_id(str(tmp_path / "missing")) == 49407
    assert clip_eos_token_id(None) == 49407
    monkeypatch.setenv("MMF_CLIP_EOS_TOKEN_ID", "123")
    assert clip_eos_token_id(str(tmp_path)) == 123
