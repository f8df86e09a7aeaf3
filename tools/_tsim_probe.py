"""Diagnostic: max |got - reference| per score key over the golden analyze() dicts (drop-in API)."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import conftest
from tables import TableClipProcessor, TableRobertaTokenizer
from misinfo_forensics import MisinfoForensics
from PIL import Image
G = os.path.join(os.path.dirname(conftest.__file__), "golden")
golden = dict(np.load(os.path.join(G, "golden.npz")))
gj = json.load(open(os.path.join(G, "golden.json")))
gi = conftest.golden_inputs.__wrapped__(golden, gj)
import mmf_amd.weights as W
rob, clp = {}, {}
for i in range(golden["rob_ids"].shape[0]):
    t = f"sample text {i}"
    rob[t] = golden["rob_ids"][i, :gi["rob_lens"][i]].tolist()
    clp[t] = golden["clip_ids"][i, :gi["clip_lens"][i]].tolist()
for j, ids in enumerate(gi["title_ids"]):
    clp[f"Guardian article {j}"] = ids.tolist()
for mb in (64, 1):
    mf = MisinfoForensics(fusion_weights="/x", faiss_index_path="/x", roberta_tokenizer=TableRobertaTokenizer(rob),
                          clip_processor=TableClipProcessor(clp), detector_state=W.synthetic_detector_state(0),
                          clip_state=W.synthetic_clip_state(0), max_batch=max(mb, 8), verbose=False)
    mf.set_vault(gi["vault"], gi["meta"])
    d = {}
    texts = [f"sample text {i}" for i in range(len(gj["analyze"]))]
    pils = [Image.fromarray(gi["imgs"][i]) for i in range(len(texts))]
    outs = mf.analyze_pairs(texts, pils) if mb > 1 else [mf.analyze(text=t, image_path=p) for t, p in zip(texts, pils)]
    for got, ref in zip(outs, gj["analyze"]):
        for k, v in ref["scores"].items():
            d[k] = max(d.get(k, 0.0), abs(got["scores"][k] - v))
    print(f"batch {'pairs' if mb > 1 else 'single analyze()'}:", {k: f"{v:.2e}" for k, v in d.items()})
    mf.engine.close()
