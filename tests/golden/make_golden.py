"""Generate the golden fixtures by running the REFERENCE code itself (build container only).

    python tests/golden/make_golden.py            # writes tests/golden/golden.npz + golden.json
    python tests/golden/make_golden.py --video    # writes tests/golden/golden_video.json
    python tests/golden/make_golden.py --vault-edge  # writes tests/golden/golden_vault_edge.json

What runs: ``/root/reference/misinfo_forensics.py`` and ``clip_similarity_engine.py`` are
imported unmodified.  Because the build container has no network, weights or tokenizer
vocabularies, the harness:

* registers stub ``dotenv`` / ``torchvision`` modules (tv_stub.py) *after* importing
  transformers, so ``misinfo_forensics`` imports;
* builds ``MultiModalMisinfoDetector`` from a local ``save_pretrained`` directory of a
  roberta-base-shaped ``RobertaModel`` and loads the seeded synthetic detector state dict
  (mmf_amd.weights) strictly; builds ``CLIPModel(CLIPConfig())`` with the seeded CLIP weights;
* bypasses ``MisinfoForensics.__init__`` (it fetches models by NAME) with ``object.__new__``
  and sets the attributes ``__init__`` would set;
* supplies table-driven tokenizers (text string -> pre-generated token ids) and a CLIP
  processor = real ``CLIPImageProcessor`` (PIL backend) + the id table;
* wraps ``clip_model.get_image_features/get_text_features`` to return tensors (the
  transformers-4.x semantics the reference was written for, misinfo_forensics.py:438-439,
  480-481; quirk Q5).

Everything stored is DATA: inputs (token ids), outputs of the reference (scores, logits,
embeddings, vault matches, verdicts, explanation strings).  Images and the base vault are
regenerated from seeds on the test side (synthetic.py) and checked by CRC32 here.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import transformers  # noqa: E402  (must precede the stubs)
from transformers import BatchEncoding, CLIPConfig, CLIPImageProcessor, CLIPModel, RobertaConfig, RobertaModel  # noqa: E402

import tv_stub  # noqa: E402
import mmf_amd.synthetic as syn  # noqa: E402
import mmf_amd.weights as W  # noqa: E402

REF = "/root/reference"

B = 8
ROB_LENS = [128, 97, 40, 5, 128, 64, 17, 3]
CLIP_LENS = [77, 30, 9, 3, 77, 50, 12, 2]
PLANT = {0: 100, 3: 1000, 5: 2000}       # sample -> vault row holding a copy of its image embedding
N_VAULT = 2170
SEED_W, SEED_IN, SEED_VAULT = 0, 1234, 77


from tables import TableClipProcessor, TableRobertaTokenizer  # noqa: E402


def crc(a: np.ndarray) -> int:
    return zlib.crc32(np.ascontiguousarray(a).tobytes())


def setup():
    """The reference objects and inputs shared by every fixture section."""
    torch.manual_seed(0)
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    tv_stub.install()
    sys.path.insert(0, REF)
    import misinfo_forensics as ref
    import clip_similarity_engine as ref_cse
    from PIL import Image

    det_sd = W.synthetic_detector_state(SEED_W)
    clip_sd = W.synthetic_clip_state(SEED_W)

    # ---- reference detector from a local save_pretrained dir (no network) -------------------
    tmp = tempfile.mkdtemp()
    rcfg = RobertaConfig(vocab_size=50265, max_position_embeddings=514, type_vocab_size=1, layer_norm_eps=1e-5)
    RobertaModel(rcfg, add_pooling_layer=True).save_pretrained(os.path.join(tmp, "roberta"))
    det = ref.MultiModalMisinfoDetector(os.path.join(tmp, "roberta"))
    missing, unexpected = det.load_state_dict({k: torch.from_numpy(v) for k, v in det_sd.items()}, strict=True)
    det.eval()
    clip = CLIPModel(CLIPConfig())
    clip.load_state_dict({k: torch.from_numpy(v) for k, v in clip_sd.items()}, strict=True)
    clip.eval()
    eos_id = clip.config.text_config.eos_token_id

    # Q5 shim: transformers 5.x returns BaseModelOutputWithPooling from get_*_features
    class ClipQ5:  # proxy handed to the reference; the real CLIPModel.forward is untouched
        def __init__(self, m):
            self.m = m

        def __call__(self, **kw):
            return self.m(**kw)

        def get_image_features(self, **kw):
            return self.m.get_image_features(**kw).pooler_output

        def get_text_features(self, **kw):
            return self.m.get_text_features(**kw).pooler_output

    clipq = ClipQ5(clip)

    # ---- inputs ------------------------------------------------------------------------------
    rob_ids, rob_mask = syn.roberta_ids(B, 128, SEED_IN, ROB_LENS)
    clip_ids, clip_mask = syn.clip_ids(B, 77, SEED_IN, CLIP_LENS)
    imgs = syn.images(B, SEED_IN)
    texts = [f"sample text {i}" for i in range(B)]
    rob_table = {t: rob_ids[i, :ROB_LENS[i]].tolist() for i, t in enumerate(texts)}
    clip_table = {t: clip_ids[i, :CLIP_LENS[i]].tolist() for i, t in enumerate(texts)}
    # vault titles and their CLIP ids
    g = np.random.Generator(np.random.PCG64(4242))
    titles = [f"Guardian article {j}" for j in range(N_VAULT)]
    t_lens = g.integers(3, 78, N_VAULT)
    t_ids, _ = syn.clip_ids(N_VAULT, 77, 99, t_lens.tolist())
    for j, t in enumerate(titles):
        clip_table[t] = t_ids[j, :t_lens[j]].tolist()
    proc = TableClipProcessor(clip_table)
    pil = [Image.fromarray(imgs[i]) for i in range(B)]

    # ---- planted vault -----------------------------------------------------------------------
    with torch.no_grad():
        raw_img_emb = torch.cat([clipq.get_image_features(**proc(images=p, return_tensors="pt")) for p in pil]).numpy()
    vault = syn.vault(N_VAULT, 512, SEED_VAULT)
    vault_base_crc = crc(vault)
    for s, row in PLANT.items():
        vault[row] = raw_img_emb[s] * np.float32(3.0)
    meta = [{"title": titles[j], "url": f"https://example.org/a/{j}", "date": "N/A"} for j in range(N_VAULT)]

    # ---- reference MisinfoForensics without __init__ ----------------------------------------
    mf = object.__new__(ref.MisinfoForensics)
    mf.device = torch.device("cpu")
    mf.gemini_available = False
    mf.roberta_tokenizer = TableRobertaTokenizer(rob_table)
    mf.detector = det
    mf.clip_processor = proc
    mf.clip_model = clipq
    mf.vault_loaded = True
    mf.vault_embeddings = vault
    mf.vault_metadata = meta
    mf.efficientnet_transform = tv_stub.Compose([
        tv_stub.Resize((224, 224)), tv_stub.ToTensor(),
        tv_stub.Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])])
    return dict(ref=ref, ref_cse=ref_cse, det=det, clip=clip, clipq=clipq, eos_id=eos_id, proc=proc, pil=pil,
                texts=texts, imgs=imgs, mf=mf, rob_table=rob_table, clip_table=clip_table, rob_ids=rob_ids,
                rob_mask=rob_mask, clip_ids=clip_ids, clip_mask=clip_mask, t_ids=t_ids, t_lens=t_lens,
                raw_img_emb=raw_img_emb, vault_base_crc=vault_base_crc)


def video_fixtures(S) -> dict:
    """analyze_video / analyze(video_path=...) (misinfo_forensics.py:493-573, 812-829) run by the
    reference against cv2_stub (OpenCV is absent) on the video_fixture.py inputs."""
    import cv2_stub
    from video_fixture import ANALYZE_CALLS, VIDEO_CALLS, VIDEOS, bgr_videos, video_vault
    cv2_stub.install(bgr_videos(S["imgs"]))
    mf, texts = S["mf"], S["texts"]
    saved = mf.vault_embeddings
    mf.vault_embeddings = video_vault(syn.vault(N_VAULT, 512, SEED_VAULT), S["raw_img_emb"])
    js = {"calls": [], "analyze": [], "errors": {}}
    for vid, ti, mx, st in VIDEO_CALLS:
        r = mf.analyze_video(vid, text=texts[ti] if ti is not None else None, max_frames=mx, stride_seconds=st)
        bf = r.pop("best_frame")
        r["best_frame_sample"] = (None if bf is None else
                                  next(i for i in VIDEOS[vid]["frames"] if np.array_equal(np.asarray(bf), S["imgs"][i])))
        js["calls"].append({"video": vid, "text": ti, "max_frames": mx, "stride_seconds": st, "result": r})
    for vid, ti in ANALYZE_CALLS:
        r = mf.analyze(text=texts[ti] if ti is not None else None, video_path=vid, verbose=False)
        js["analyze"].append({"video": vid, "text": ti, "result": r})
    for vid in ("v_empty.mp4", "missing.mp4"):
        try:
            mf.analyze_video(vid)
        except RuntimeError as e:
            js["errors"][vid] = str(e)
    mf.vault_embeddings = saved
    return js


def vault_edge_fixtures(S) -> dict:
    """The reference's search_vault (misinfo_forensics.py:410-491) on the vault_edge.py cases.  The
    query image features are planted through the CLIP proxy (get_image_features returns the case's
    raw query; the reference normalises it itself), so only the vault arithmetic and ranking run."""
    import vault_edge as VE
    mf = S["mf"]
    saved = (mf.vault_embeddings, mf.vault_metadata, mf.clip_model)
    meta = [{"title": f"Guardian article {j}", "url": f"https://example.org/a/{j}", "date": "N/A"}
            for j in range(VE.N)]
    out = {"numpy": np.__version__, "cases": {}}

    class PlantedQuery:
        q = None

        def get_image_features(self, **kw):
            return torch.as_tensor(self.q)[None]

    proxy = PlantedQuery()
    try:
        mf.clip_model, mf.vault_metadata = proxy, meta
        for name in VE.CASES:
            vault, q = VE.case(name)
            mf.vault_embeddings = vault
            res = []
            for i in range(VE.NQ):
                proxy.q = q[i]
                for top_k in (5, 12):
                    r = mf.search_vault(S["pil"][0], top_k=top_k)
                    res.append({"query": i, "top_k": top_k, "vault_discrepancy": r["vault_discrepancy"],
                                "text_similarity": r["text_similarity"],
                                "idx": [int(m["title"].split()[-1]) for m in r["matches"]],
                                "sims": [m["similarity"] for m in r["matches"]]})
            out["cases"][name] = {"dtype": str(vault.dtype), "vault_crc": crc(vault), "results": res}
    finally:
        mf.vault_embeddings, mf.vault_metadata, mf.clip_model = saved
    return out


def main_vault_edge():
    S = setup()
    js = vault_edge_fixtures(S)
    with open(os.path.join(HERE, "golden_vault_edge.json"), "w") as f:
        json.dump(js, f, indent=1)
    print("wrote", os.path.join(HERE, "golden_vault_edge.json"))


def main_video():
    S = setup()
    js = video_fixtures(S)
    with open(os.path.join(HERE, "golden_video.json"), "w") as f:
        json.dump(js, f, indent=1, default=float)
    print("wrote", os.path.join(HERE, "golden_video.json"))


def main():
    S = setup()
    globals().update(S)
    ref, ref_cse, det, clip, clipq, eos_id, proc, pil, texts, imgs, mf = (
        S["ref"], S["ref_cse"], S["det"], S["clip"], S["clipq"], S["eos_id"], S["proc"], S["pil"], S["texts"],
        S["imgs"], S["mf"])
    rob_table, clip_table, rob_ids, rob_mask, clip_ids, clip_mask = (
        S["rob_table"], S["clip_table"], S["rob_ids"], S["rob_mask"], S["clip_ids"], S["clip_mask"])
    t_ids, t_lens, raw_img_emb, vault_base_crc = S["t_ids"], S["t_lens"], S["raw_img_emb"], S["vault_base_crc"]

    out = {}
    js = {"analyze": [], "analyze_text_only": [], "analyze_image_only": [], "clip_engine": [],
          "meta": {"B": B, "rob_lens": ROB_LENS, "clip_lens": CLIP_LENS, "plant": PLANT,
                   "seeds": [SEED_W, SEED_IN, SEED_VAULT], "eos_token_id": eos_id,
                   "images_crc": crc(imgs), "vault_base_crc": vault_base_crc,
                   "transformers": transformers.__version__}}
    cls, ai_l, mi_l, eff_l, ie, te, csim = [], [], [], [], [], [], []
    with torch.no_grad():
        for i in range(B):
            ids = torch.tensor([rob_table[texts[i]]])
            h = det.roberta(input_ids=ids, attention_mask=torch.ones_like(ids)).last_hidden_state
            cls.append(h[0, 0].numpy())
            a, m = det.forward_text(ids, torch.ones_like(ids))
            ai_l.append(a[0].numpy()); mi_l.append(m[0].numpy())
            x = mf.efficientnet_transform(pil[i]).unsqueeze(0)
            eff_l.append(det.forward_image(x)[0].numpy())
            o = clip(**proc(text=[texts[i]], images=pil[i], return_tensors="pt", padding=True))
            ie.append(o.image_embeds[0].numpy()); te.append(o.text_embeds[0].numpy())
            csim.append(mf.analyze_consistency(texts[i], pil[i])["clip_similarity"])
    out.update(cls_hidden=np.stack(cls), ai_logits=np.stack(ai_l), misinfo_logits=np.stack(mi_l),
               effnet_logits=np.stack(eff_l), clip_image_embeds=np.stack(ie),
               clip_text_embeds=np.stack(te), clip_similarity=np.array(csim, np.float32),
               clip_image_features_raw=raw_img_emb, rob_ids=rob_ids, rob_mask=rob_mask,
               clip_ids=clip_ids, clip_mask=clip_mask, title_clip_ids=t_ids,
               title_lens=t_lens.astype(np.int32))

    top_idx, top_sim, disc, tsim = [], [], [], []
    for i in range(B):
        r = mf.analyze(text=texts[i], image_path=pil[i], verbose=False)
        js["analyze"].append(r)
        v = mf.search_vault(pil[i], user_caption=texts[i])
        ti = [int(m["title"].split()[-1]) for m in v["matches"]]
        top_idx.append(ti); top_sim.append([m["similarity"] for m in v["matches"]])
        disc.append(v["vault_discrepancy"]); tsim.append(v["text_similarity"])
    out.update(vault_top_idx=np.array(top_idx, np.int64), vault_top_sim=np.array(top_sim, np.float32),
               vault_discrepancy=np.array(disc, np.float32), text_similarity=np.array(tsim, np.float32),
               scores=np.array([[r["scores"][k] for k in ("ai_score", "misinfo_score", "deepfake_score",
                                                          "clip_similarity", "vault_discrepancy")]
                                for r in js["analyze"]], np.float32),
               fusion_probs=np.array([[r["scores"]["real_probability"], r["scores"]["fake_probability"]]
                                      for r in js["analyze"]], np.float32))
    for i in (0, 1):
        js["analyze_text_only"].append(mf.analyze(text=texts[i], verbose=False))
    for i in (2, 3):
        js["analyze_image_only"].append(mf.analyze(image_path=pil[i], verbose=False))
    try:
        mf.analyze(verbose=False)
    except ValueError as e:
        js["analyze_no_input_error"] = str(e)
    # no vault loaded
    mf.vault_loaded = False
    js["search_vault_unloaded"] = mf.search_vault(pil[0], user_caption=texts[0])
    mf.vault_loaded = True

    # ---- fusion judge, config 1 -----------------------------------------------------------
    x5 = syn.fusion_inputs(1024, SEED_IN)
    with torch.no_grad():
        out["fusion_c1_inputs"] = x5
        out["fusion_c1_probs"] = torch.softmax(det.forward_fusion(torch.from_numpy(x5)), 1).numpy()
        js["fusion_verdicts"] = [mf.fusion_verdict(dict(zip(
            ("ai_score", "misinfo_score", "deepfake_score", "clip_similarity", "vault_discrepancy"),
            map(float, x5[i])))) for i in range(16)]

    # ---- fallback explanation cascade on crafted score dicts ----------------------------
    cases = []
    base = dict(ai_score=0.1, misinfo_score=0.1, deepfake_score=0.1, clip_similarity=0.5,
                vault_discrepancy=0.0, verdict=0, confidence=0.8123)
    for upd in ({}, {"vault_discrepancy": 0.93, "verdict": 1}, {"deepfake_score": 0.8765},
                {"ai_score": 0.75}, {"misinfo_score": 0.71, "verdict": 1}, {"clip_similarity": 0.1},
                {"clip_similarity": 0.3}, {"deepfake_score": 0.7}):
        s = dict(base, **upd)
        cases.append({"scores": s, "text": mf._generate_fallback_explanation(s, [{"title": "Planted title"}])})
    js["explanations"] = cases

    # ---- CLIPSimilarityEngine -----------------------------------------------------------
    eng = object.__new__(ref_cse.CLIPSimilarityEngine)
    eng.model, eng.processor, eng.threshold, eng.device = clip, proc, 0.25, "cpu"
    d = tempfile.mkdtemp()
    for i in range(4):
        path = os.path.join(d, f"img{i}.png")
        pil[i].save(path)
        sim, label = eng.calculate_similarity(path, texts[i])
        r = eng.analyze_with_explanation(path, texts[i])
        r["image_path"] = f"img{i}.png"
        js["clip_engine"].append({"sample": i, "similarity": sim, "label": label, "with_explanation": r})
    js["clip_engine_explanations"] = [
        {"similarity": s, "label": lab, "text": eng._generate_explanation(s, lab)}
        for s, lab in ((0.8, "Match"), (0.55, "Match"), (0.3, "Match"), (0.05, "Mismatch"), (0.2, "Mismatch"))]
    for bad in (("missing.png", texts[0]), (os.path.join(d, "img0.png"), "")):
        try:
            eng.calculate_similarity(*bad)
        except Exception as e:  # noqa: BLE001
            js.setdefault("clip_engine_errors", []).append({"type": type(e).__name__,
                                                            "msg": str(e).replace(d, "<tmp>")})

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(js, f, indent=1, default=float)
    print("wrote", os.path.join(HERE, "golden.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    if "--video" in sys.argv:
        main_video()
    elif "--vault-edge" in sys.argv:
        main_vault_edge()
    else:
        main()
