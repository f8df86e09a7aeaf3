"""The drop-in API on the MI355X against the reference's own analyze() / CLIPSimilarityEngine
outputs (tests/golden/golden.json, produced by running /root/reference code).  Same inputs: the
reference's text strings (through the same id tables), PIL images, vault rows and titles."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _tables(golden, gi):
    rob, clp = {}, {}
    for i in range(golden["rob_ids"].shape[0]):
        t = f"sample text {i}"
        rob[t] = golden["rob_ids"][i, :gi["rob_lens"][i]].tolist()
        clp[t] = golden["clip_ids"][i, :gi["clip_lens"][i]].tolist()
    for j, ids in enumerate(gi["title_ids"]):
        clp[f"Guardian article {j}"] = ids.tolist()
    return rob, clp


@pytest.fixture(scope="module")
def forensics(golden, golden_inputs, det_sd, clip_sd, tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from tables import TableClipProcessor, TableRobertaTokenizer
    from misinfo_forensics import MisinfoForensics
    rob, clp = _tables(golden, golden_inputs)
    mf = MisinfoForensics(fusion_weights="/nonexistent", faiss_index_path="/nonexistent",
                          roberta_tokenizer=TableRobertaTokenizer(rob), clip_processor=TableClipProcessor(clp),
                          detector_state=det_sd, clip_state=clip_sd, max_batch=64, verbose=False)
    mf.set_vault(golden_inputs["vault"], golden_inputs["meta"])
    return mf


def _pil(gi, i):
    from PIL import Image
    return Image.fromarray(gi["imgs"][i])


def _check(got, ref, tol=TOL):
    for k, v in ref["scores"].items():  # scores first: their message names the signal that moved
        assert abs(got["scores"][k] - v) < tol, (k, got["scores"][k], v)
    assert got["verdict"] == ref["verdict"] and got["verdict_text"] == ref["verdict_text"]
    assert abs(got["confidence"] - ref["confidence"]) < tol
    assert [m["title"] for m in got["vault_matches"]] == [m["title"] for m in ref["vault_matches"]]
    for a, b in zip(got["vault_matches"], ref["vault_matches"]):
        assert abs(a["similarity"] - b["similarity"]) < tol and a["url"] == b["url"] and a["date"] == b["date"]
    assert got["explanation"] == ref["explanation"]


def test_analyze_pairs_match_reference(forensics, golden_json, golden_inputs):
    for i, ref in enumerate(golden_json["analyze"]):
        _check(forensics.analyze(text=f"sample text {i}", image_path=_pil(golden_inputs, i), verbose=False), ref)


def test_no_vault_loaded(golden, golden_json, golden_inputs, det_sd, clip_sd):
    """Truth-Vault not loaded (misinfo_forensics.py:422-428): search_vault returns the reference's
    unloaded dict, analyze() and analyze_pairs() run the other four signals with
    vault_discrepancy = 0 and no matches, and agree with the oracle's analyze without a vault."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from tables import TableClipProcessor, TableRobertaTokenizer
    from misinfo_forensics import MisinfoForensics
    from oracle.pipeline import OracleForensics
    rob, clp = _tables(golden, golden_inputs)
    mf = MisinfoForensics(fusion_weights="/nonexistent", faiss_index_path="/nonexistent",
                          roberta_tokenizer=TableRobertaTokenizer(rob), clip_processor=TableClipProcessor(clp),
                          detector_state=det_sd, clip_state=clip_sd, max_batch=8, verbose=False)
    assert not mf.vault_loaded
    assert mf.search_vault(_pil(golden_inputs, 0), "sample text 0") == golden_json["search_vault_unloaded"]
    orc = OracleForensics(det_sd, clip_sd, eos_token_id=golden_inputs["eos"])
    texts = [f"sample text {i}" for i in range(4)]
    batch = mf.analyze_pairs(texts, [_pil(golden_inputs, i) for i in range(4)])
    for i in range(4):
        t = (golden["rob_ids"][i, :golden_inputs["rob_lens"][i]], golden["clip_ids"][i, :golden_inputs["clip_lens"][i]])
        ref = orc.analyze(text=t, image=golden_inputs["imgs"][i])
        assert ref["scores"]["vault_discrepancy"] == 0.0 and ref["vault_matches"] == []
        for got in (mf.analyze(text=texts[i], image_path=_pil(golden_inputs, i), verbose=False), batch[i]):
            _check(got, ref)
    mf.engine.close()


def test_long_text_analyze_text(forensics, det_sd, clip_sd):
    """A 400-token article (past the 128 reserved by default; the reference truncates at 512):
    the workspaces grow and analyze_text matches the oracle's single-text forward."""
    import mmf_amd.synthetic as syn
    from oracle.pipeline import OracleForensics
    ids, _ = syn.roberta_ids(1, 400, 91)
    forensics.roberta_tokenizer.table["long article"] = ids[0].tolist()
    got = forensics.analyze_text("long article")
    assert forensics.engine.max_text_len == 512
    ref = OracleForensics(det_sd, clip_sd).analyze_text(ids[0])
    for k in ("ai_score", "misinfo_score"):
        assert abs(got[k] - ref[k]) < TOL, (k, got[k], ref[k])


def test_analyze_single_modalities(forensics, golden_json, golden_inputs):
    for n, i in enumerate((0, 1)):
        _check(forensics.analyze(text=f"sample text {i}", verbose=False), golden_json["analyze_text_only"][n])
    for n, i in enumerate((2, 3)):
        _check(forensics.analyze(image_path=_pil(golden_inputs, i), verbose=False),
               golden_json["analyze_image_only"][n])
    with pytest.raises(ValueError) as e:
        forensics.analyze(verbose=False)
    assert str(e.value) == golden_json["analyze_no_input_error"]


def test_batched_dicts_equal_single(forensics, golden_inputs):
    texts = [f"sample text {i}" for i in range(8)]
    batch = forensics.analyze_pairs(texts, [_pil(golden_inputs, i) for i in range(8)])
    for i in (0, 5):
        one = forensics.analyze(text=texts[i], image_path=_pil(golden_inputs, i), verbose=False)
        assert one["verdict"] == batch[i]["verdict"] and one["explanation"] == batch[i]["explanation"]


def test_analyze_pairs_chunks_past_capacity(forensics, golden_inputs):
    """More pairs than the reserved batch: analyze_pairs runs max_batch-sized chunks and returns
    one dict per pair, in order, equal to the single-launch result."""
    texts = [f"sample text {i % 8}" for i in range(10)]
    imgs = [_pil(golden_inputs, i % 8) for i in range(10)]
    full = forensics.analyze_pairs(texts, imgs)
    e = forensics.engine
    keep = (e.max_batch, e.max_text_len, e.max_clip_len)
    e.reserve(4, keep[1], keep[2])
    try:
        chunked = forensics.analyze_pairs(texts, imgs)
    finally:
        e.reserve(*keep)
    assert len(chunked) == 10
    for a, b in zip(chunked, full):
        _check(a, b)


def test_detector_forward_methods(forensics, golden, golden_inputs):
    from oracle import models as M
    x = M.effnet_preprocess(torch.as_tensor(golden_inputs["imgs"]))
    lg = forensics.detector.forward_image(x.cuda()).cpu()
    np.testing.assert_allclose(torch.softmax(lg, 1)[:, 1].numpy(),
                               torch.softmax(torch.as_tensor(golden["effnet_logits"]), 1)[:, 1].numpy(), atol=TOL)
    ai, mi = forensics.detector.forward_text(torch.as_tensor(golden["rob_ids"]).cuda(),
                                             torch.as_tensor(golden["rob_mask"]).cuda())
    np.testing.assert_allclose(torch.softmax(ai.cpu(), 1)[:, 1].numpy(),
                               torch.softmax(torch.as_tensor(golden["ai_logits"]), 1)[:, 1].numpy(), atol=TOL)


def test_retrained_fusion_layer_reaches_the_kernel(forensics):
    det = forensics.detector
    saved = {k: v.clone() for k, v in det.fusion_layer.state_dict().items()}
    with torch.no_grad():
        det.fusion_layer[5].bias.add_(torch.tensor([0.3, -0.3], device=forensics.device))
    s = {"ai_score": 0.4, "misinfo_score": 0.6, "deepfake_score": 0.2, "clip_similarity": 0.1,
         "vault_discrepancy": 0.0}
    got = forensics.fusion_verdict(s)
    det.eval()
    with torch.no_grad():
        p = torch.softmax(det.forward_fusion(torch.tensor([[0.4, 0.6, 0.2, 0.1, 0.0]], device=forensics.device)), 1)[0]
    assert abs(got["fake_probability"] - p[1].item()) < 1e-5
    det.fusion_layer.load_state_dict(saved)
    forensics.detector.sync_fusion(force=True)


def test_clip_similarity_engine(golden, golden_json, golden_inputs, clip_sd, tmp_path):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from tables import TableClipProcessor
    from clip_similarity_engine import CLIPSimilarityEngine
    _, clp = _tables(golden, golden_inputs)
    eng = CLIPSimilarityEngine(threshold=0.25, processor=TableClipProcessor(clp), clip_state=clip_sd)
    for rec in golden_json["clip_engine"]:
        i = rec["sample"]
        p = str(tmp_path / f"img{i}.png")
        _pil(golden_inputs, i).save(p)
        sim, label = eng.calculate_similarity(p, f"sample text {i}")
        assert abs(sim - rec["similarity"]) < TOL and label == rec["label"]
        r = eng.analyze_with_explanation(p, f"sample text {i}")
        assert r["label"] == rec["with_explanation"]["label"]
        assert abs(r["similarity_score"] - rec["with_explanation"]["similarity_score"]) <= 1e-3 + 1e-9
    errs = golden_json["clip_engine_errors"]
    with pytest.raises(FileNotFoundError) as e:
        eng.calculate_similarity("missing.png", "x")
    assert str(e.value) == errs[0]["msg"]
    with pytest.raises(ValueError) as e:
        eng.calculate_similarity(str(tmp_path / "img0.png"), "")
    assert str(e.value) == errs[1]["msg"]


def test_analyze_video_matches_reference(forensics, golden, golden_json, golden_inputs):
    """analyze_video / analyze(video_path=...) (misinfo_forensics.py:493-573, 812-829) against the
    reference's own results (tests/golden/golden_video.json; OpenCV replaced by the frame-replay
    stub on both sides).  All frames of a video go through one batched EfficientNet / CLIP /
    vault pass here; the reference ran 3 single-image passes per frame."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import cv2_stub
    import video_fixture as VF
    import mmf_amd.synthetic as syn
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_video.json")) as f:
        gv = json.load(f)
    imgs = golden_inputs["imgs"]
    cv2_stub.install(VF.bgr_videos(imgs))
    seeds = golden_json["meta"]["seeds"]
    forensics.set_vault(VF.video_vault(syn.vault(2170, 512, seeds[2]), golden["clip_image_features_raw"]),
                        golden_inputs["meta"])
    try:
        for c in gv["calls"]:
            ref = c["result"]
            got = forensics.analyze_video(c["video"], text=f"sample text {c['text']}" if c["text"] is not None else None,
                                          max_frames=c["max_frames"], stride_seconds=c["stride_seconds"])
            for k in ("deepfake_score", "clip_similarity", "vault_discrepancy"):
                assert abs(got[k] - ref[k]) < TOL, (c, k, got[k], ref[k])
            assert abs(got["text_similarity"] - ref["text_similarity"]) < TOL
            assert [m["title"] for m in got["vault_matches"]] == [m["title"] for m in ref["vault_matches"]]
            for a, b in zip(got["vault_matches"], ref["vault_matches"]):
                assert abs(a["similarity"] - b["similarity"]) < TOL
            assert np.array_equal(np.asarray(got["best_frame"]), imgs[ref["best_frame_sample"]])
        for a in gv["analyze"]:
            got = forensics.analyze(text=f"sample text {a['text']}" if a["text"] is not None else None,
                                    video_path=a["video"], verbose=False)
            _check(got, a["result"])
        for vid, msg in gv["errors"].items():
            with pytest.raises(RuntimeError) as e:
                forensics.analyze_video(vid)
            assert str(e.value) == msg
    finally:
        sys.modules.pop("cv2", None)
        forensics.set_vault(golden_inputs["vault"], golden_inputs["meta"])


def test_vault_builder_on_hip(clip_sd, tmp_path):
    """generate_embeddings_database (train_clip_detective.py:457-607) with the HIP CLIP towers,
    weights loaded from a CLIPDetective-format checkpoint ('model_state_dict' with 'clip.' keys),
    against the CPU oracle's normalised embeddings."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from tables import TableClipProcessor
    from PIL import Image
    import mmf_amd.synthetic as syn
    from mmf_amd import io_utils
    from mmf_amd.vault_builder import generate_embeddings_database
    from oracle import models as M
    n = 40
    imgs = syn.images(n, 91)
    lens = [(7 * i) % 76 + 2 for i in range(n)]
    ids, _ = syn.clip_ids(n, 77, 92, lens)
    table, arts = {}, []
    for i in range(n):
        p = str(tmp_path / f"a{i}.png")
        Image.fromarray(imgs[i]).save(p)
        table[f"t{i}"] = ids[i, :lens[i]].tolist()
        arts.append({"article_id": i, "text_content": f"t{i}", "image_local_path": p})
    (tmp_path / "seed.json").write_text(json.dumps(arts))
    ck = str(tmp_path / "clip_detective_best.pth")
    torch.save({"model_state_dict": {"clip." + k: torch.as_tensor(v) for k, v in clip_sd.items()},
                "epoch": 3, "val_accuracy": 0.9}, ck)
    db = generate_embeddings_database(ck, str(tmp_path / "seed.json"), str(tmp_path / "vault.pkl"),
                                      processor=TableClipProcessor(table), batch=16)
    assert db["article_ids"] == list(range(n)) and db["metadata"]["val_accuracy"] == 0.9
    sd = M.to_torch(clip_sd)
    with torch.no_grad():
        px = np.stack([io_utils.clip_pixels(Image.fromarray(imgs[i])) for i in range(n)])
        ie = M.l2n(M.clip_image_features(sd, M.clip_preprocess(torch.as_tensor(px)))).numpy()
        msk = (np.arange(77)[None] < np.asarray(lens)[:, None]).astype(np.int32)
        te = M.l2n(M.clip_text_features(sd, torch.as_tensor(ids), torch.as_tensor(msk))).numpy()
    assert (db["image_embeddings"] * ie).sum(1).min() > 1 - 1e-4
    assert (db["text_embeddings"] * te).sum(1).min() > 1 - 1e-4
    emb, meta = io_utils.load_vault(str(tmp_path / "vault.pkl"))
    assert emb.shape == (n, 512) and meta[3]["title"] == "t3"
