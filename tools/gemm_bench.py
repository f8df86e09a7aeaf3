"""Micro-benchmark of libmmf_hip's fp16 GEMM on the encoder shapes of the hot path.

    python tools/gemm_bench.py [--configs auto,10,11] [--iters 20] [--round] [--effnet]

Prints TFLOP/s (TB/s for the EfficientNet 1x1 convolutions) per (shape, tile config), measured with
HIP events on the stream the kernel is launched on; the process option "gemm_config"
(mmf_set_option with a NULL handle) forces the tile instantiation.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmf_amd.hip as hip  # noqa: E402

# (name, M, N, K, act, out) at B=256: RoBERTa L=128, ViT L=50, CLIP text L=77 (out-proj / FFN-2
# write their fp16 branch output; the fp32 residual add happens in add+LN)
SHAPES = [
    ("rob_qkv", 32768, 2304, 768, 0, "16"), ("rob_o", 32768, 768, 768, 0, "16"),
    ("rob_fc1", 32768, 3072, 768, 1, "16"), ("rob_fc2", 32768, 768, 3072, 0, "16"),
    ("vit_qkv", 12800, 2304, 768, 0, "16"), ("vit_o", 12800, 768, 768, 0, "16"),
    ("vit_fc1", 12800, 3072, 768, 2, "16"), ("vit_fc2", 12800, 768, 3072, 0, "16"),
    ("txt_qkv", 19712, 1536, 512, 0, "16"), ("txt_o", 19712, 512, 512, 0, "16"),
    ("txt_fc1", 19712, 2048, 512, 2, "16"), ("txt_fc2", 19712, 512, 2048, 0, "16"),
    ("patch", 12544, 768, 3072, 0, "32"), ("sq4096", 4096, 4096, 4096, 0, "16"),
]
# one persistent round of 256x256 tiles (256 tiles) at growing K: per-K-step slope vs fixed cost
ROUND = [("round_k%d" % k, 8192, 2048, k, 0, "16") for k in (256, 512, 768, 1536, 3072, 6144)]

# EfficientNet-B0 1x1 convolutions at B=256: (name, M, N, K, act, SE scale, fp16 residual, rows/image)
EFFNET = [
    ("e2.1", 256 * 12544, 96, 16, 3, 0, 0, 12544), ("e2.2", 256 * 3136, 144, 24, 3, 0, 0, 3136),
    ("e3.2", 256 * 784, 240, 40, 3, 0, 0, 784), ("e4.2", 256 * 196, 480, 80, 3, 0, 0, 196),
    ("e5.2", 256 * 196, 672, 112, 3, 0, 0, 196), ("e6.2", 256 * 49, 1152, 192, 3, 0, 0, 49),
    ("p1", 256 * 12544, 16, 32, 0, 1, 0, 12544), ("p2.1", 256 * 3136, 24, 96, 0, 1, 0, 3136),
    ("p2.2", 256 * 3136, 24, 144, 0, 1, 1, 3136), ("p3.1", 256 * 784, 40, 144, 0, 1, 0, 784),
    ("p3.2", 256 * 784, 40, 240, 0, 1, 1, 784), ("p4.2", 256 * 196, 80, 480, 0, 1, 1, 196),
    ("p5.2", 256 * 196, 112, 672, 0, 1, 1, 196), ("p6.2", 256 * 49, 192, 1152, 0, 1, 1, 49),
    ("p7", 256 * 49, 320, 1152, 0, 1, 0, 49), ("head", 256 * 49, 1280, 320, 3, 0, 0, 49),
]


def timed_us(call, iters):
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def force(cfg):
    hip.set_process_option("gemm_config", -1 if cfg == "auto" else int(cfg))


def effnet(a, lib, dev):
    for name, M, N, K, act, sc, rs, rpb in EFFNET:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.float16)
        bias = torch.randn(N, device=dev)
        S = torch.rand(M // rpb, K, device=dev) if sc else None
        R = torch.randn(M, N, device=dev).to(torch.float16) if rs else None
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        byts = 2.0 * M * (K + N + (N if rs else 0))
        row = {"shape": name, "M": M, "N": N, "K": K, "MB": round(byts / 1e6, 1)}
        for cfg in a.configs.split(","):
            force(cfg)
            us = timed_us(lambda: hip.check(lib.mmf_gemm_f16_ex(
                A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), hip.ptr(R), hip.ptr(S), rpb, C.data_ptr(), N, M,
                N, K, act, hip.stream_ptr())), a.iters)
            row[cfg] = f"{us:.1f}us {byts / us / 1e6:.2f}TB/s"
        force("auto")
        print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="auto,3,5,10,11")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=1, help="interleaved rounds over the configs (median reported)")
    ap.add_argument("--kscale", default="", help="comma list of K multipliers to time (fixed-cost probe)")
    ap.add_argument("--effnet", action="store_true", help="time the EfficientNet 1x1 convolutions instead")
    ap.add_argument("--round", action="store_true", help="one 256-tile round at K = 256 .. 6144")
    ap.add_argument("--group-m", default="", help="extra timed pass per config per gemm_group_m value (comma list)")
    ap.add_argument("--opt", default="gemm_group_m", help="process option swept by --vals (default gemm_group_m)")
    ap.add_argument("--vals", default="", help="extra timed pass per config per value of --opt (comma list)")
    ap.add_argument("--no-store", action="store_true",
                    help="also time each config with no output tensor (every store dropped by the buffer "
                         "descriptor): the epilogue's write cost is the difference")
    ap.add_argument("--shapes", default="", help="comma list of shape names to time (default all)")
    a = ap.parse_args()
    lib = hip.load()
    dev = torch.device("cuda")
    if a.effnet:
        effnet(a, lib, dev)
        return
    shapes = ROUND if a.round else SHAPES
    if a.shapes:
        shapes = [x for x in shapes if x[0] in a.shapes.split(",")]
    if a.kscale:
        shapes = [(f"{n}_k{m}", M, N, K * int(m), act, out) for n, M, N, K, act, out in shapes
                  for m in a.kscale.split(",")]
    for name, M, N, K, act, out in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.float16)
        bias = torch.randn(N, device=dev)
        c32 = torch.empty(M, N, device=dev) if "32" in out else None
        c16 = torch.empty(M, N, device=dev, dtype=torch.float16) if "16" in out else None

        def call(store=True):
            hip.check(lib.mmf_gemm_f16(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), None,
                                        hip.ptr(c32) if store else None, hip.ptr(c16) if store else None, N, M, N,
                                        K, act, hip.stream_ptr()))
        row = {"shape": name, "M": M, "N": N, "K": K}
        opt = "gemm_group_m" if a.group_m else a.opt
        vals = a.group_m or a.vals
        for v in [""] + [x for x in vals.split(",") if x]:
            hip.set_process_option(opt, int(v or 0))
            samples = {}
            for _ in range(a.rounds):
                for cfg in a.configs.split(","):
                    force(cfg)
                    samples.setdefault(cfg, []).append(timed_us(call, a.iters))
            for cfg in a.configs.split(","):
                force(cfg)
                us = sorted(samples[cfg])[len(samples[cfg]) // 2]
                row[(f"{opt}={v}:" if v else "") + cfg] = round(2.0 * M * N * K / (us / 1e6) / 1e12, 1)
                if a.no_store:
                    us0 = timed_us(lambda: call(False), a.iters)
                    row[(f"{opt}={v}:" if v else "") + cfg + ":us/us_nostore"] = f"{us:.1f}/{us0:.1f}"
        hip.set_process_option(opt, 0)
        force("auto")
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
