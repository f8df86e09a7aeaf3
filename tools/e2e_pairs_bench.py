"""Text+JPEG -> verdict throughput through the drop-in API (`MisinfoForensics.analyze_pairs`), i.e.
the reference's `analyze(text, image)` for a batch of real-format inputs, with the time split into
its host and device stages.

    python tools/e2e_pairs_bench.py [--n 256] [--reps 3] [--progressive] [--json out.json]

`bench_line()` is bench.py's `per_sample.text_jpeg_pairs` line (the same calls, fewer stage splits).

Inputs: synthetic 640x480 JPEGs (tools/host_pipeline_bench.py) and ~40-word texts; tokenizers are
byte-level BPEs trained on a synthetic corpus and wrapped with RoBERTa's / CLIP's special-token and
padding conventions (the vocab files are absent), weights are synthetic.  Prints one JSON object.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from host_pipeline_bench import synth_jpegs, synth_texts  # noqa: E402


class _BPE:
    """A byte-level BPE with a tokenizer-call interface: `prefix + bpe[:cap] + suffix`, right padded."""

    def __init__(self, bpe, prefix, suffix, pad, cap):
        self.bpe, self.prefix, self.suffix, self.pad, self.cap = bpe, prefix, suffix, pad, cap

    def _ids(self, encs, truncation, max_length):
        seqs = [self.prefix + e.ids[:self.cap] + self.suffix for e in encs]
        if truncation:
            seqs = [s[:max_length] for s in seqs]
        L = max(len(s) for s in seqs)
        ids = torch.full((len(seqs), L), self.pad, dtype=torch.long)
        mask = torch.zeros((len(seqs), L), dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.tensor(s)
            mask[i, :len(s)] = 1
        return {"input_ids": ids, "attention_mask": mask}


class RobertaLike(_BPE):
    def __call__(self, text, return_tensors="pt", max_length=512, truncation=True, padding=True):
        texts = [text] if isinstance(text, str) else list(text)
        return self._ids(self.bpe.encode_batch(texts), truncation, max_length)


class ClipLike(_BPE):
    def __call__(self, text=None, images=None, return_tensors="pt", padding=False, truncation=False):
        return self._ids(self.bpe.encode_batch(list(text)), truncation, 77)


def _forensics(n, progressive=False):
    from tokenizers import ByteLevelBPETokenizer
    from mmf_amd.api import MisinfoForensics
    bpe = ByteLevelBPETokenizer()
    bpe.train_from_iterator(synth_texts(4000, seed=9)[0], vocab_size=8000, min_frequency=2, show_progress=False)
    rob = RobertaLike(bpe, [0], [2], 1, 510)
    clp = ClipLike(bpe, [49406], [49407], 49407, 75)
    texts = synth_texts(n, seed=4, words=40)[0]
    jpegs = synth_jpegs(n, progressive=progressive)
    mf = MisinfoForensics(fusion_weights="", faiss_index_path="", synthetic_seed=0, roberta_tokenizer=rob,
                          clip_processor=clp, max_batch=n, verbose=False)
    g = np.random.default_rng(11)
    emb = g.standard_normal((2170, 512)).astype(np.float32)
    mf.set_vault(emb, [{"title": t, "url": "u", "date": "d"} for t in synth_texts(2170, seed=12, words=12)[0]])
    return mf, rob, texts, jpegs


def bench_line(n=256, reps=3):
    """bench.py's secondary line: analyze_pairs over n text + JPEG pairs (encoded bytes in host memory,
    the reference's real input format), one call and a 4-chunk call, device JPEG decode vs Pillow."""
    mf, _, texts, jpegs = _forensics(n)
    best = {}
    for chunks in (1, 4):
        t4, j4 = texts * chunks, jpegs * chunks
        for dj in (True, False):
            mf.device_jpeg = dj
            mf.analyze_pairs(t4, j4)  # warm
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                mf.analyze_pairs(t4, j4)
                ts.append(time.perf_counter() - t0)
            best[(chunks, dj)] = chunks * n / min(ts)
    mf.engine.close()
    return {"config": f"analyze_pairs over {n} text + JPEG pairs (synthetic 640x480 q90 4:2:0 JPEG bytes, "
                      "~40-word texts, synthetic BPE tokenizers): decode + tokenise + resample + 5 signals + "
                      "result dicts, host stages on the box's CPU share",
            "value": round(best[(1, True)], 1), "unit": "pairs/s",
            "pipelined_4_chunks": round(best[(4, True)], 1),
            "pillow_decode": {"value": round(best[(1, False)], 1), "pipelined_4_chunks": round(best[(4, False)], 1)},
            "note": "device JPEG path: host Huffman decoding into packed coefficients, IDCT / upsampling / colour "
                    "and both resamplings on the GPU, pixels bit-exact with Pillow (tests/test_gpu_jpeg.py)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--progressive", action="store_true", help="progressive JPEGs (Pillow's scan script)")
    a = ap.parse_args()
    from mmf_amd import io_utils
    mf, rob, texts, jpegs = _forensics(a.n, a.progressive)
    mf.analyze_pairs(texts, jpegs)  # warm (workspace growth, first launches)
    torch.cuda.synchronize()

    stages = {"tokenize": [], "decode": [], "pack_h2d_device_resample": [], "device_analyze": [],
              "result_dicts": [], "total": [], "host_resample_instead": []}
    for _ in range(a.reps):
        t0 = time.perf_counter()
        r = io_utils.tokenize_roberta_batch(rob, texts)
        rid, rm = io_utils.pad_ids(r, 1)
        cid, cm = mf._clip_ids(texts)
        t1 = time.perf_counter()
        rgb = io_utils.decode_rgb(jpegs)
        t2 = time.perf_counter()
        eff, cl = mf.engine.resize_images(rgb)
        t3 = time.perf_counter()
        out = mf.analyze_batch(rid, rm, cid, cm, eff, cl)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        mf.batch_to_dicts(out)
        t5 = time.perf_counter()
        io_utils.decode_batch(jpegs)  # the all-host alternative (decode + both Pillow resamplings)
        t6 = time.perf_counter()
        for k, v in zip(stages, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0, t6 - t5)):
            stages[k].append(v)
        # device JPEG path (mmf_amd/jpeg.py): host entropy decoding, then H2D + device
        # reconstruction + device resampling
        from mmf_amd import jpeg
        if mf._jpeg is None:
            mf._jpeg = jpeg.JpegStager()
        t6 = time.perf_counter()
        st = mf._jpeg.stage(jpegs)
        t7 = time.perf_counter()
        jpeg.device_windows(mf.engine, mf._jpeg, st)
        torch.cuda.synchronize()
        t8 = time.perf_counter()
        stages.setdefault("jpeg_entropy_host", []).append(t7 - t6)
        stages.setdefault("jpeg_h2d_reconstruct_resample", []).append(t8 - t7)
        for dj, key in ((False, "analyze_pairs_call_pillow_decode"), (True, "analyze_pairs_call")):
            mf.device_jpeg = dj
            t5 = time.perf_counter()
            mf.analyze_pairs(texts, jpegs)
            stages.setdefault(key, []).append(time.perf_counter() - t5)
    # a 4-chunk call: the host stage of chunk i + 1 overlaps chunk i's device work
    texts4, jpegs4 = texts * 4, jpegs * 4
    mf.analyze_pairs(texts4, jpegs4)
    for _ in range(a.reps):
        for dj, key in ((False, "analyze_pairs_4_chunks_pillow_decode"), (True, "analyze_pairs_4_chunks")):
            mf.device_jpeg = dj
            t0 = time.perf_counter()
            mf.analyze_pairs(texts4, jpegs4)
            stages.setdefault(key, []).append(time.perf_counter() - t0)
    best = {k: min(v) for k, v in stages.items()}
    from mmf_amd import benchrun
    res = {"n_pairs": a.n, "usable_cores": benchrun.usable_cpus(),
           "pairs_per_s": round(a.n / best["analyze_pairs_call"], 1),
           "pairs_per_s_4_chunks_pipelined": round(4 * a.n / best["analyze_pairs_4_chunks"], 1),
           "pairs_per_s_pillow_decode": round(a.n / best["analyze_pairs_call_pillow_decode"], 1),
           "pairs_per_s_4_chunks_pillow_decode": round(4 * a.n / best["analyze_pairs_4_chunks_pillow_decode"], 1),
           "stage_ms": {k: round(1e3 * v, 2) for k, v in best.items()},
           "note": "device JPEG decode (host entropy + device IDCT/upsample/colour) unless *_pillow_decode; synthetic 640x480 JPEGs" + (" (progressive)" if a.progressive else "") + ", ~40-word texts, synthetic BPE tokenizers and weights; stages timed "
                   "sequentially (analyze_pairs runs them in the same order)"}
    print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
