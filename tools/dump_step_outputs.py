"""Every output of the bench's analyze_batch step (B = 256, bench inputs incl. the planted vault) ->
.npz, to compare two builds bit for bit:

    MMF_HIP_LIB=variants/x/libmmf_hip.so python tools/dump_step_outputs.py a.npz
    python tools/dump_step_outputs.py b.npz
    python tools/dump_step_outputs.py --cmp a.npz b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "--cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for k in a.files:
            x, y = a[k], b[k]
            same = x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8))
            d = "" if same else f" max |d| {np.nanmax(np.abs(x.astype(np.float64) - y.astype(np.float64))):.3e}"
            print(f"{k:16s} {'bit-identical' if same else 'DIFFERS'}{d}")
        return
    import torch
    import bench
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=256)
    t = bench.build_inputs(eng, 256, 0)
    out = eng.analyze_batch(t["rid"], t["rm"], t["cid"], t["cm"], t["img"])
    torch.cuda.synchronize()
    np.savez(sys.argv[1], **{k: v.cpu().numpy() for k, v in out.items()})


if __name__ == "__main__":
    main()
