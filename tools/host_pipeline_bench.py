"""Host input-stage throughput: what the CPU side of a serving box can feed the GPU path.

    python tools/host_pipeline_bench.py [--n 256] [--json out.json]

* images: N synthetic 640x480 JPEGs (quality 90, smooth structured content) decoded once each and
  resampled to both towers' geometries by `io_utils.decode_batch` at 1, 4, 8 and all usable
  threads (images/s);
* text: a byte-level BPE tokenizer (the RoBERTa tokenizer's algorithm family, HF `tokenizers`),
  trained here on a synthetic corpus because the roberta-base / CLIP vocab files are absent (so
  the rate is representative of the algorithm, not parity-pinned), encoding N news-length texts
  (~90 words) with truncation at 128 tokens, serial and batched (texts/s).
Prints one JSON object; the GPU box numbers are committed as profiles/r02_host_pipeline.json (git history at 168304c).
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mmf_amd import benchrun, io_utils  # noqa: E402


def synth_jpegs(n, w=640, h=480, seed=3, progressive=False):
    from PIL import Image
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = []
    for i in range(n):
        f = g.uniform(0.005, 0.05, size=3)
        ph = g.uniform(0, 6.28, size=3)
        a = np.stack([127 + 100 * np.sin(xx * f[c] + yy * f[(c + 1) % 3] + ph[c]) for c in range(3)], -1)
        a += g.normal(0, 8, size=a.shape)
        b = io.BytesIO()
        Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(b, format="JPEG", quality=90, progressive=progressive)
        out.append(b.getvalue())
    return out


def synth_texts(n, seed=4, words=90):
    g = np.random.default_rng(seed)
    syll = ["ka", "to", "ri", "men", "sa", "lo", "ve", "dan", "ur", "po", "li", "tic", "al", "ne", "ws", "re", "port",
            "ed", "in", "on", "the", "gov", "ern", "ment", "claim", "ing", "sta", "te", "of", "fi", "cial"]
    vocab = ["".join(g.choice(syll, size=g.integers(1, 4))) for _ in range(5000)]
    return [" ".join(g.choice(vocab, size=words)) + "." for _ in range(n)], vocab


def rate(fn, n, reps=3):
    fn()  # warm
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return n / best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    cores = benchrun.usable_cpus()
    res = {"usable_cores": cores, "n": a.n}
    jpegs = synth_jpegs(a.n)
    res["jpeg_bytes_avg"] = int(np.mean([len(j) for j in jpegs]))
    img = {}
    for w in sorted({1, 4, 8, cores}):
        img[f"threads_{w}"] = round(rate(lambda: io_utils.decode_batch(jpegs, workers=w), a.n), 1)
    res["decode_resize_images_per_s"] = img

    from tokenizers import ByteLevelBPETokenizer
    texts, vocab = synth_texts(a.n)
    tok = ByteLevelBPETokenizer()
    tok.train_from_iterator(synth_texts(4000, seed=9)[0], vocab_size=8000, min_frequency=2, show_progress=False)
    tok.enable_truncation(128)
    res["tokenize_texts_per_s"] = {
        "serial": round(rate(lambda: [tok.encode(t) for t in texts], a.n), 1),
        "batched": round(rate(lambda: tok.encode_batch(texts), a.n), 1),
    }
    res["note"] = ("synthetic 640x480 JPEGs -> both 224x224 geometries (io_utils.decode_batch); byte-level BPE "
                   "trained on a synthetic corpus (vocab files absent: throughput of the algorithm, parity unpinned)")
    print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
