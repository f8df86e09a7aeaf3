"""Interleaved timing of the HBM-resident B=256 analyze step under handle-option variants (one
process, one box), median over rounds; outputs of every variant checked against the first.

    python tools/step_ab.py "concurrent=1" "stagger_text=5,stagger_vit=10" [--rounds 5 --iters 20]
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
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--what", choices=("step", "clip", "text"), default="step",
                    help="step: analyze_batch; clip: mmf_clip_consistency (configs[3]); text: configs[1]")
    ap.add_argument("--batch", type=int, default=256, help="pairs per step (the bench workload: 256)")
    a = ap.parse_args()
    import bench
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    B = a.batch
    eng = Engine(0, W.synthetic_detector_state(0), W.synthetic_clip_state(0), max_batch=B)
    t = bench.build_inputs(eng, B, 0)
    out = eng.alloc_outputs(B)
    variants = [{k: int(x) for k, x in (kv.split("=", 1) for kv in v.split(","))} for v in a.variants]
    names = sorted({k for v in variants for k in v})
    base = {k: eng.get_option(k) for k in names}

    def setv(v):
        for k in names:
            eng.set_option(k, v.get(k, base[k]))

    if a.what == "clip":
        out = {"img_emb": torch.empty(B, 512, device=eng.device), "txt_emb": torch.empty(B, 512, device=eng.device),
               "sim": torch.empty(B, device=eng.device)}

        def step():
            eng.clip_consistency(t["img"], t["cid"], t["cm"], out=out)
    elif a.what == "text":
        from mmf_amd.hip import check, ptr, stream_ptr
        out = {k: torch.empty(B, 2, device=eng.device) for k in ("ai", "mi", "sc")}

        def step():
            check(eng.lib.mmf_text_forward(eng.h, ptr(t["rid"]), ptr(t["rm"]), B, 128, ptr(out["ai"]),
                                           ptr(out["mi"]), ptr(out["sc"]), stream_ptr()))
    else:
        def step():
            eng.analyze_batch(t["rid"], t["rm"], t["cid"], t["cm"], t["img"], out=out)

    ref = None
    for v in variants:
        setv(v)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        o = {k: x.clone() for k, x in out.items()}
        if ref is None:
            ref = o
        else:
            same = all(torch.equal(o[k], ref[k]) for k in o)
            dmax = max(float((o[k].double() - ref[k].double()).abs().max()) for k in o)
            print(f"{v}: outputs identical to {variants[0]}: {same} (max |d| {dmax:.2e})", flush=True)
    times = [[] for _ in variants]
    for _ in range(a.rounds):
        for i, v in enumerate(variants):
            setv(v)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                step()
            torch.cuda.synchronize()
            times[i].append((time.perf_counter() - t0) / a.iters)
    for v, ts in zip(a.variants, times):
        m = statistics.median(ts)
        print(f"{v:40s} {m * 1e3:7.3f} ms/step {B / m:8.0f} pairs/s  [{', '.join(f'{x * 1e3:.2f}' for x in ts)}]",
              flush=True)


if __name__ == "__main__":
    main()
