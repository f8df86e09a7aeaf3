"""Where the per-pair analyze(text, image) latency goes (B = 1, the dashboard path,
forensics_dashboard.py:180-185).

    python tools/b1_latency.py [--n 100]

Prints one JSON object: p50 wall times of the whole call and of its stages -- tokenise + decode
(host), device resample, the 5-signal batch with its inputs already on the device (wall incl. one
sync, and device time by events), and result dicts."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def p50(xs):
    return round(float(np.percentile(np.asarray(xs) * 1e3, 50)), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    from PIL import Image
    import mmf_amd.synthetic as syn
    from mmf_amd import io_utils
    from mmf_amd.api import MisinfoForensics
    n = a.n + 10
    texts, rob, clp = syn.text_tables(n, 77)
    pils = [Image.fromarray(x) for x in syn.images(n, 77)]
    tid, tm = syn.clip_ids(2170, 77, 99, np.random.default_rng(5).integers(3, 78, 2170).tolist())
    meta = []
    for j in range(2170):
        clp.table[f"title {j}"] = tid[j, :int(tm[j].sum())].tolist()
        meta.append({"title": f"title {j}", "url": "N/A", "date": "N/A"})
    mf = MisinfoForensics(fusion_weights="", faiss_index_path="", synthetic_seed=0, roberta_tokenizer=rob,
                          clip_processor=clp, verbose=False)
    mf.set_vault(syn.vault(2170, 512, 77), meta)
    eng = mf.engine
    for i in range(10):
        mf.analyze(text=texts[i], image_path=pils[i], verbose=False)
    torch.cuda.synchronize()
    res = {k: [] for k in ("analyze", "host_stage", "resize", "batch_wall", "batch_device", "dicts", "sync_check")}
    for i in range(10, n):
        t0 = time.perf_counter()
        mf.analyze(text=texts[i], image_path=pils[i], verbose=False)
        res["analyze"].append(time.perf_counter() - t0)
        # the stages of analyze_pairs, one at a time
        t0 = time.perf_counter()
        rids = io_utils.tokenize_roberta_batch(rob, [texts[i]])
        rid, rm = io_utils.pad_ids(rids, 1)
        cid, cm = mf._clip_ids([texts[i]])
        rgb = io_utils.decode_rgb([pils[i]])
        res["host_stage"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        eff, cl = mf._resize(rgb)
        torch.cuda.synchronize()
        res["resize"].append(time.perf_counter() - t0)
        d = {k: torch.as_tensor(v).cuda() for k, v in (("rid", rid), ("rm", rm), ("cid", cid), ("cm", cm))}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mf.detector.sync()
        res["sync_check"].append(time.perf_counter() - t0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = eng.analyze_batch(d["rid"], d["rm"], d["cid"], d["cm"], eff, cl)
        e1.record()
        torch.cuda.synchronize()
        res["batch_wall"].append(time.perf_counter() - t0)
        res["batch_device"].append(e0.elapsed_time(e1) / 1e3)
        t0 = time.perf_counter()
        mf.batch_to_dicts(out)
        res["dicts"].append(time.perf_counter() - t0)
    print(json.dumps({k: p50(v) for k, v in res.items()} | {"unit": "ms (p50)", "calls": a.n}))
    eng.close()


if __name__ == "__main__":
    main()
