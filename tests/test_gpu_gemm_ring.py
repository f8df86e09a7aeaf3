"""The pipelined encoder GEMMs of csrc/gemm_ring.hip (ring, loader / consumer) against the two-stage LDS-DMA kernel it
replaces and against a torch fp32 reference of the same op (C = act(A W^T + b), fp16 in / out,
fp32 accumulation).

Both kernels accumulate every output element in the same order (32-deep MFMA chunks, ascending
K), so the ring kernel must return BIT-IDENTICAL results -- on the encoder shapes of the hot path,
on ragged edges (M and N not multiples of the 256 x 192 tile, one tile, more tiles than
workgroups, K = 128 .. 3072) and with every epilogue activation."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, N, K, act)
    (32768, 768, 768, 0), (32768, 768, 3072, 0), (32768, 2304, 768, 0), (32768, 3072, 768, 1),
    (12800, 768, 3072, 0), (19712, 512, 2048, 0),
    (1000, 200, 128, 0), (256, 192, 256, 2), (777, 1544, 640, 3), (50, 8, 192, 4), (300000, 16, 64 * 2, 0),
]


def _run(lib, hip, A, W, bias, M, N, K, act, cfg):
    hip.set_process_option("gemm_config", cfg)
    C = torch.full((M, N), float("nan"), device=A.device, dtype=torch.float16)
    hip.check(lib.mmf_gemm_f16_ex(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), None, None, 1, C.data_ptr(), N,
                                   M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("cfg", [12, 17])  # 12 ring, 17 loader / consumer waves
@pytest.mark.parametrize("M,N,K,act", SHAPES)
def test_ring_matches_two_stage_bitwise(M, N, K, act, cfg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.hip as hip
    lib = hip.load()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
    A = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(torch.float16)
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.float16)
    bias = torch.randn(N, device="cuda", generator=g)
    try:
        ring = _run(lib, hip, A, W, bias, M, N, K, act, cfg)
        ref_cfg = 10 if K >= 192 else 6  # the pipelined two-stage kernel needs >= 3 K-steps of 64
        base = _run(lib, hip, A, W, bias, M, N, K, act, ref_cfg)
    finally:
        hip.set_process_option("gemm_config", -1)
    assert not torch.isnan(ring).any()
    assert torch.equal(ring, base), (ring.float() - base.float()).abs().max().item()
    # and the op itself, against torch fp32 (act 0 = none, 1 = GELU-erf, 2 = quick-GELU, 3 = SiLU, 4 = ReLU)
    ref = A.float() @ W.float().t() + bias
    ref = {0: ref, 1: torch.nn.functional.gelu(ref), 2: ref * torch.sigmoid(1.702 * ref),
           3: torch.nn.functional.silu(ref), 4: torch.relu(ref)}[act]
    err = (ring.float() - ref).abs().max().item()
    tol = 2e-3 * max(1.0, ref.abs().max().item())
    assert err <= tol, (err, tol)
