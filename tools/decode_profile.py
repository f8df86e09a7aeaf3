"""Where the host time of analyze_pairs' image stage goes (decode / array copy / pack / H2D / device
resample) for N synthetic 640x480 JPEGs on this host."""
import io
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from host_pipeline_bench import synth_jpegs  # noqa: E402


def main():
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image
    from mmf_amd import io_utils
    from mmf_amd.engine import Engine
    n = 256
    jp = synth_jpegs(n)
    eng = Engine(0, None, None, max_batch=n)
    ex = ThreadPoolExecutor(16)
    for rep in range(3):
        t0 = time.perf_counter()
        ims = [Image.open(io.BytesIO(j)) for j in jp]
        t1 = time.perf_counter()
        list(ex.map(lambda im: im.load(), ims))
        t2 = time.perf_counter()
        arrs = list(ex.map(lambda im: np.asarray(im), ims))
        t3 = time.perf_counter()
        eff, clp = eng.resize_images(arrs)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        rgb = io_utils.decode_rgb(jp)
        t5 = time.perf_counter()
        print(f"open {1e3*(t1-t0):.1f} ms, decode(16 thr) {1e3*(t2-t1):.1f}, asarray {1e3*(t3-t2):.1f}, "
              f"pack+H2D+resample {1e3*(t4-t3):.1f}, decode_rgb() {1e3*(t5-t4):.1f}", flush=True)


if __name__ == "__main__":
    main()
