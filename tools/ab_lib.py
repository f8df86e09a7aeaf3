"""Interleaved A/B timing of two builds of libmmf_hip.so in ONE process (same device, same
clocks): for each GEMM shape, alternate lib A / lib B calls for several rounds and report the
median microseconds of each.

    python tools/ab_lib.py path/to/libA.so path/to/libB.so [--effnet] [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmf_amd.hip as hip  # noqa: E402
from tools.gemm_bench import EFFNET, ROUND, SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("liba")
    ap.add_argument("libb")
    ap.add_argument("--effnet", action="store_true")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    libs = [hip.load(a.liba), hip.load(a.libb)]
    dev = torch.device("cuda")
    shapes = ([(n, M, N, K, act, sc, rs, rpb) for n, M, N, K, act, sc, rs, rpb in EFFNET] if a.effnet else
              [(n, M, N, K, act, 0, 0, 1) for n, M, N, K, act, _ in SHAPES + ROUND])
    for name, M, N, K, act, sc, rs, rpb in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.float16)
        bias = torch.randn(N, device=dev)
        S = torch.rand((M + rpb - 1) // rpb, K, device=dev) if sc else None
        R = torch.randn(M, N, device=dev).to(torch.float16) if rs else None
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        times = [[], []]
        for _ in range(a.rounds):
            for i, lib in enumerate(libs):
                def call():
                    hip.check(lib.mmf_gemm_f16_ex(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), hip.ptr(R),
                                                   hip.ptr(S), rpb, C.data_ptr(), N, M, N, K, act,
                                                   hip.stream_ptr()))
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / a.iters * 1e3)
        ma, mb = statistics.median(times[0]), statistics.median(times[1])
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "A_us": round(ma, 1), "B_us": round(mb, 1),
                          "B_over_A": round(mb / ma, 3)}), flush=True)


if __name__ == "__main__":
    main()
