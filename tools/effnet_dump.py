"""EfficientNet logits of a fixed synthetic batch -> .npy (compare builds bit for bit:
MMF_HIP_LIB=a.so python tools/effnet_dump.py a.npy [opt=v ...]; python tools/effnet_dump.py b.npy; cmp)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    eng = Engine(0, W.synthetic_detector_state(0), None, max_batch=256)
    for kv in sys.argv[2:]:  # run-time options k=v (e.g. effnet_chunks=1)
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    lg, sc = eng.effnet_forward(syn.images(256, 41))
    torch.cuda.synchronize()
    np.save(sys.argv[1], lg.cpu().numpy())


if __name__ == "__main__":
    main()
