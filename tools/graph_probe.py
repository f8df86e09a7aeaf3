"""Is the analyze step launch-gap bound?  Times the HBM-resident B=256 step eagerly and as a
replayed hipGraph (torch.cuda.CUDAGraph capture of mmf_analyze_batch, tower streams forked and
joined inside the capture), interleaved rounds, and checks that the replay's outputs are the eager
outputs bit for bit.

    python tools/graph_probe.py [--rounds 5 --iters 20 --batch 256]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import bench
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    B = a.batch
    eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=B)
    t = bench.build_inputs(eng, B, 0)
    out = eng.alloc_outputs(B)

    def step():
        eng.analyze_batch(t["rid"], t["rm"], t["cid"], t["cm"], t["img"], out=out)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in out.items()}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    for k in out:
        out[k].zero_()
    g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(out[k], ref[k]) for k in out)
    print(f"graph replay outputs identical to eager: {same}", flush=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.iters

    te, tg = [], []
    for _ in range(a.rounds):
        te.append(timed(step))
        tg.append(timed(g.replay))
    me, mg = statistics.median(te), statistics.median(tg)
    print(f"eager {me * 1e3:.3f} ms/step ({B / me:.0f} pairs/s)  graph {mg * 1e3:.3f} ms/step ({B / mg:.0f} pairs/s)"
          f"  [{', '.join(f'{x * 1e3:.2f}' for x in te)}] [{', '.join(f'{x * 1e3:.2f}' for x in tg)}]", flush=True)


if __name__ == "__main__":
    main()
