"""cProfile of the B = 1 analyze() path, or of FusionTrainingDataset's per-row calls ("rows"), with
bench.py per_sample_lines' setup: where the host time of one call goes besides the device work.
    python tools/analyze_b1_profile.py [calls] [rows]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    from PIL import Image
    import mmf_amd.benchrun as benchrun
    import mmf_amd.synthetic as syn
    from mmf_amd.api import MisinfoForensics
    seed = benchrun.input_seed(0) + 200
    texts, rob, clp = syn.text_tables(n + 10, seed)
    pils = [Image.fromarray(a) for a in syn.images(n + 10, seed)]
    tid, tm = syn.clip_ids(2170, 77, 99, np.random.default_rng(5).integers(3, 78, 2170).tolist())
    meta = []
    for j in range(2170):
        clp.table[f"title {j}"] = tid[j, :int(tm[j].sum())].tolist()
        meta.append({"title": f"title {j}", "url": "N/A", "date": "N/A"})
    mf = MisinfoForensics(fusion_weights="", faiss_index_path="", synthetic_seed=0, roberta_tokenizer=rob,
                          clip_processor=clp, verbose=False)
    mf.set_vault(syn.vault(2170, 512, 77), meta)
    rows = len(sys.argv) > 2 and sys.argv[2] == "rows"

    def call(i):
        if not rows:  # the dashboard path
            return mf.analyze(text=texts[i], image_path=pils[i], verbose=False)
        # FusionTrainingDataset.__getitem__'s four calls (train_fusion_judge.py:72-86)
        return (mf.analyze_text(texts[i]), mf.analyze_image(pils[i]), mf.analyze_consistency(texts[i], pils[i]),
                mf.search_vault(pils[i]))
    for i in range(10):
        call(i)
    t0 = time.perf_counter()
    for i in range(10, 10 + n):
        call(i)
    print(f"plain: {(time.perf_counter() - t0) / n * 1e3:.3f} ms / call ({'rows' if rows else 'analyze'})")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(10, 10 + n):
        call(i)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)
    mf.engine.close()


if __name__ == "__main__":
    main()
