"""Which tower / option breaks row batch-invariance (rows 40:48 of a B=256 batch vs the same rows
run as a batch of 8)?  Prints max |diff| of the CLIP image / text embeddings per option setting.

    python tools/batch_invariance_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=256)
    B = 256
    cid, cm = syn.clip_ids(B, 77, 5)
    imgs = syn.images(B, 5)
    settings = [{}, {"lazy_ln": 0}, {"gemm_config": 10}, {"gemm_config": 11}, {"gemm_splitk": 0}]
    for st in settings:
        old = {k: eng.get_option(k) for k in st}
        for k, v in st.items():
            eng.set_option(k, v)
        fi = eng.clip_image(imgs).cpu().numpy()
        pi = eng.clip_image(imgs[40:48]).cpu().numpy()
        ft = eng.clip_text(cid, cm).cpu().numpy()
        pt = eng.clip_text(cid[40:48], cm[40:48]).cpu().numpy()
        torch.cuda.synchronize()
        print(f"{st}: image max|d| {np.abs(fi[40:48] - pi).max():.3e}  text max|d| {np.abs(ft[40:48] - pt).max():.3e}",
              flush=True)
        for k, v in old.items():
            eng.set_option(k, v)


if __name__ == "__main__":
    main()
