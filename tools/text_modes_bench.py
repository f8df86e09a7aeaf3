"""RoBERTa tower time per text mode at B = 256, L = 128.

    python tools/text_modes_bench.py [--gamma 7] [--iters 10] [--rounds 3]

Modes: fp16 / split stream (text_hilo 0 / 1), the precise mode (text_hilo 2) at several operand masks
(text_prec_mask: bit k = GEMM kind k -- QKV, out-proj, FFN-1, FFN-2 -- on hi / lo activations, bit k + 4
= also on W_lo).  The engine is built with
text_precision = "precise" so that every kind's hi / lo weights stay packed.  --gamma g uses the
dominating-channel draw of tests/test_gpu_outliers.py (0: the plain synthetic draw).  Interleaved
rounds, median ms per forward (HIP events on the stream the tower is launched on).
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gamma", type=float, default=0.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--masks", default="0,15,5,95,245,253,255")
    a = ap.parse_args()
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    det = W.synthetic_detector_state(0)
    if a.gamma:
        from test_gpu_outliers import dominating_gamma_state
        det = dominating_gamma_state(det, a.gamma, kappa=a.gamma)
    eng = Engine(0, det, None, max_batch=256, text_precision="precise")
    ids, mask = syn.roberta_ids(256, 128, 1234)
    modes = [("fp16", 0, None), ("split", 1, None)] + [(f"precise_m{m}", 2, m) for m in map(int, a.masks.split(","))]

    def setm(hilo, m):
        if m is not None:
            eng.set_option("text_prec_mask", m)
        eng.set_option("text_hilo", hilo)

    ref = {}
    for name, hilo, m in modes:
        setm(hilo, m)
        ref[name] = eng.text_forward(ids, mask)[2].double().cpu()
    samples = {n: [] for n, _, _ in modes}
    for _ in range(a.rounds):
        for name, hilo, m in modes:
            setm(hilo, m)
            for _ in range(2):
                eng.text_forward(ids, mask)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                eng.text_forward(ids, mask)
            e1.record()
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) / a.iters)
    for name, _, m in modes:
        s = sorted(samples[name])
        d = float((ref[name] - ref["precise_m255"]).abs().max()) if "precise_m255" in ref else None
        print(json.dumps({"mode": name, "ms": round(s[len(s) // 2], 3), "min_ms": round(s[0], 3),
                          "max_dscore_vs_full_precise": d, "gamma": a.gamma}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
