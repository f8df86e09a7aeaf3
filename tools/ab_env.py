"""Interleaved timing of option variants of libmmf_hip.so's GEMM in ONE process (process options
set with mmf_set_option on a NULL handle between calls), median over rounds.

    python tools/ab_env.py "gemm_group_m=0" "gemm_group_m=8" [--effnet] [--rounds 7]
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
    ap.add_argument("variants", nargs="+", help="'option=value[,option2=value]' per variant")
    ap.add_argument("--effnet", action="store_true")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    lib = hip.load()
    dev = torch.device("cuda")
    shapes = ([(n, M, N, K, act, sc, rs, rpb, "16") for n, M, N, K, act, sc, rs, rpb in EFFNET] if a.effnet else
              [(n, M, N, K, act, 0, 0, 1, out) for n, M, N, K, act, out in SHAPES + ROUND])
    variants = [{k: int(x) for k, x in (kv.split("=", 1) for kv in v.split(","))} for v in a.variants]
    for name, M, N, K, act, sc, rs, rpb, out in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.float16)
        bias = torch.randn(N, device=dev)
        S = torch.rand((M + rpb - 1) // rpb, K, device=dev) if sc else None
        R16 = torch.randn(M, N, device=dev).to(torch.float16) if rs else None
        c32 = torch.empty(M, N, device=dev) if "32" in out else None
        c16 = torch.empty(M, N, device=dev, dtype=torch.float16) if "16" in out else None
        R32 = torch.randn(M, N, device=dev) if "r" in out else None

        def call():
            if a.effnet:
                hip.check(lib.mmf_gemm_f16_ex(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), hip.ptr(R16),
                                               hip.ptr(S), rpb, c16.data_ptr(), N, M, N, K, act, hip.stream_ptr()))
            else:
                hip.check(lib.mmf_gemm_f16(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), hip.ptr(R32),
                                            hip.ptr(c32), hip.ptr(c16), N, M, N, K, act, hip.stream_ptr()))
        times = [[] for _ in variants]
        for _ in range(a.rounds):
            for i, opts in enumerate(variants):
                old = {k: hip.get_process_option(k) for k in opts}
                for k, v in opts.items():
                    hip.set_process_option(k, v)
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / a.iters * 1e3)
                for k, v in old.items():
                    hip.set_process_option(k, v)
        med = [statistics.median(t) for t in times]
        row = {"shape": name, "M": M, "N": N, "K": K}
        for v, m in zip(a.variants, med):
            row[v] = round(m, 1)
        row["best"] = a.variants[med.index(min(med))]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
