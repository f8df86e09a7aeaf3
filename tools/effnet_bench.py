"""EfficientNet-B0 tower alone (B images, synthetic weights/inputs) for per-kernel profiling:

    python tools/effnet_bench.py [--batch 256 --iters 10] [--ab dw_cw32=0 dw_cw32=1 --rounds 5] [--opt effnet_chunks=1]
    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -- python tools/effnet_bench.py --iters 2
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ab", nargs="*", default=[], help="interleaved option variants 'opt=v[,opt2=v]'")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--opt", nargs="*", default=[], help="handle options set before the run 'opt=v'")
    ap.add_argument("--pinned", action="store_true",
                    help="fp16 towers pinned (no load-time calibration launches in a profile of the tower)")
    a = ap.parse_args()
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    pin = dict(effnet_precision="fp16", text_precision="fp16") if a.pinned else {}
    eng = Engine(0, W.synthetic_detector_state(0), None, max_batch=a.batch, **pin)
    for kv in a.opt:
        k, x = kv.split("=", 1)
        eng.set_option(k, int(x))
    img = torch.from_numpy(syn.images(a.batch, 3)).cuda()
    eng.effnet_forward(img)
    torch.cuda.synchronize()
    if a.ab:
        import statistics
        variants = [{k: int(x) for k, x in (kv.split("=", 1) for kv in v.split(","))} for v in a.ab]
        times = [[] for _ in variants]
        for _ in range(a.rounds):
            for vi, v in enumerate(variants):
                for k, x in v.items():
                    eng.set_option(k, x)
                eng.effnet_forward(img)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    eng.effnet_forward(img)
                torch.cuda.synchronize()
                times[vi].append((time.perf_counter() - t0) / a.iters)
        for v, t in zip(a.ab, times):
            print(f"{v}: median {statistics.median(t) * 1e3:.3f} ms / forward (B={a.batch}) "
                  f"[{', '.join(f'{x * 1e3:.3f}' for x in t)}]", flush=True)
        return
    t0 = time.perf_counter()
    for _ in range(a.iters):
        eng.effnet_forward(img)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(f"effnet B={a.batch}: {dt * 1e3:.3f} ms / forward, {a.batch / dt:.0f} img/s")


if __name__ == "__main__":
    main()
