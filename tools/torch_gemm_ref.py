"""Reference point: torch (hipBLASLt) fp16 linear on the encoder GEMM shapes, same timing method
as tools/gemm_bench.py.  Diagnostic only (the product path never calls hipBLASLt)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import SHAPES  # noqa: E402


def main():
    dev = torch.device("cuda")
    for name, M, N, K, act, out in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.float16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.float16)
        b = torch.randn(N, device=dev).to(torch.float16)
        row = {"shape": name}
        for label, fn in (("linear", lambda: torch.nn.functional.linear(A, W, b)),
                          ("mm", lambda: A @ W.t()),
                          ("linear_gelu", lambda: torch.nn.functional.gelu(torch.nn.functional.linear(A, W, b)))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            row[label] = round(2.0 * M * N * K / (ms / 1e3) / 1e12, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
