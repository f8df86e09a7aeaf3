"""Tower A/B timings on one GPU (interleaved rounds, HIP-event / wall timing of whole calls):

* CLIP towers (BASELINE configs[3], B = 256): both towers on concurrent streams (the production
  mmf_clip_consistency), serialised on one stream (option concurrent = 0), and each tower alone --
  what the streams already overlap, the headroom a grouped ViT + text launch could take;
* RoBERTa (configs[1], B = 256, L = 128) in each stream / precision mode: text_hilo 0 (fp16 stream),
  1 (split stream), 2 (precise mode: K-concatenated ~22-bit GEMM operands, fp32 stream / LN /
  attention) -- the cost of the precision fallbacks;
* EfficientNet (configs[2], B = 512) fp16 and fp32 towers;
* the engine's construction (weight packing + load-time calibration).

    python tools/tower_ab.py [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, steps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--what", default="clip,text,effnet", help="comma list of clip, text, effnet, step")
    a = ap.parse_args()
    what = set(a.what.split(","))
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    det, clip = W.synthetic_detector_state(0), W.synthetic_clip_state(0)
    t0 = time.perf_counter()
    eng = Engine(0, det, clip, max_batch=256)
    build_s = time.perf_counter() - t0
    print(json.dumps({"engine_build_s": round(build_s, 2), "text_check": eng.text_check,
                      "effnet_check": eng.effnet_check, "clip_stream_check": eng.clip_stream_check}), flush=True)
    B = 256
    dev = eng.device
    rid, rm = (torch.from_numpy(x).to(dev) for x in syn.roberta_ids(B, 128, 1234))
    cid, cm = (torch.from_numpy(x).to(dev) for x in syn.clip_ids(B, 77, 1234))
    img = torch.from_numpy(syn.images(B, 1234)).to(dev)
    cons = {"img_emb": torch.empty(B, 512, device=dev), "txt_emb": torch.empty(B, 512, device=dev),
            "sim": torch.empty(B, device=dev)}
    res = {}

    def add(k, v):
        res.setdefault(k, []).append(round(v, 3))
    for r in range(a.rounds):
        if "clip" in what:
            eng.set_option("concurrent", 1)
            add("clip_concurrent_ms", timed(lambda: eng.clip_consistency(img, cid, cm, out=cons), a.steps))
            eng.set_option("concurrent", 0)
            add("clip_serial_ms", timed(lambda: eng.clip_consistency(img, cid, cm, out=cons), a.steps))
            eng.set_option("concurrent", 1)
            add("vit_alone_ms", timed(lambda: eng.clip_image(img), a.steps))
            add("clip_text_alone_ms", timed(lambda: eng.clip_text(cid, cm), a.steps))
        if "step" in what:
            ab_out = eng.alloc_outputs(B)
            add("analyze_b256_ms", timed(lambda: eng.analyze_batch(rid, rm, cid, cm, img, out=ab_out), a.steps))
        if "text" in what:
            for mode in (0, 1, 2):
                eng.set_option("text_hilo", mode)
                add(f"roberta_text_hilo{mode}_ms", timed(lambda: eng.text_forward(rid, rm), a.steps))
            eng.set_option("text_hilo", -1)
    if "effnet" not in what:
        print(json.dumps({k: {"rounds": v, "min": min(v), "median": sorted(v)[len(v) // 2]} for k, v in res.items()},
                         indent=1), flush=True)
        eng.close()
        return
    eng.reserve(512, 128, 77)
    img5 = torch.from_numpy(syn.images(512, 99)).to(dev)
    for r in range(a.rounds):
        for fp32 in (0, 1):
            eng.set_option("effnet_fp32", fp32)
            add(f"effnet_b512_fp32_{fp32}_ms", timed(lambda: eng.effnet_forward(img5), a.steps))
    eng.set_option("effnet_fp32", 0)
    out = {k: {"rounds": v, "min": min(v), "median": sorted(v)[len(v) // 2]} for k, v in res.items()}
    print(json.dumps(out, indent=1), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
