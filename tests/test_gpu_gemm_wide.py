"""The 256x384 LDS-DMA tiles of csrc/gemm.hip (config 20: descriptor fills, 192 accumulator
registers per lane) and the 4-wave 256x192 tiles (config 21: one wave per SIMD, 128x96 wave tiles,
accumulators in AGPRs) against the production 256x256 / 256x192 kernels and a torch fp32 reference of
the same op (C = act(A W^T + b) [+ res], fp16 in / out, fp32 accumulation).

Every tile shape accumulates each output element in the same order (32-deep MFMA chunks,
ascending K), so the wide tiles must return BIT-IDENTICAL results: on the RoBERTa encoder shapes,
on ragged row panels (M not a multiple of 256: the last panel takes the clamped pointer fill), with
every epilogue activation and with the fp16 residual epilogue."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, N, K, act, residual)
    (32768, 768, 768, 0, False), (32768, 768, 3072, 0, False), (32768, 2304, 768, 0, False),
    (32768, 3072, 768, 1, False), (32768, 768, 3072, 0, True),
    (1000, 384, 128, 0, False), (777, 1152, 640, 3, True), (50, 768, 192, 4, False), (257, 384, 64, 2, False),
    (9000, 1536, 1024, 0, True),
]


def _run(lib, hip, A, W, bias, res, M, N, K, act, cfg):
    hip.set_process_option("gemm_config", cfg)
    C = torch.full((M, N), float("nan"), device=A.device, dtype=torch.float16)
    hip.check(lib.mmf_gemm_f16_ex(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(),
                                   res.data_ptr() if res is not None else None, None, 1, C.data_ptr(), N,
                                   M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("cfg", [20, 21])
@pytest.mark.parametrize("M,N,K,act,resid", SHAPES)
def test_wide_tiles_match_production_bitwise(M, N, K, act, resid, cfg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.hip as hip
    lib = hip.load()
    g = torch.Generator(device="cuda").manual_seed(M * 5 + N * 3 + K)
    A = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(torch.float16)
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.float16)
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g).to(torch.float16) if resid else None
    try:
        wide = _run(lib, hip, A, W, bias, res, M, N, K, act, cfg)
        # (the half-step-pipelined 256x256 / 256x192 kernels need >= 3 K-steps of 64)
        base = {c: _run(lib, hip, A, W, bias, res, M, N, K, act, c) for c in ((11, 10) if K >= 192 else (4, 6))}
    finally:
        hip.set_process_option("gemm_config", -1)
    assert not torch.isnan(wide).any()
    for c, b in base.items():
        assert torch.equal(wide, b), (c, (wide.float() - b.float()).abs().max().item())
    ref = A.float() @ W.float().t() + bias
    ref = {0: ref, 1: torch.nn.functional.gelu(ref), 2: ref * torch.sigmoid(1.702 * ref),
           3: torch.nn.functional.silu(ref), 4: torch.relu(ref)}[act]
    if res is not None:
        ref = ref + res.float()
    err = (wide.float() - ref).abs().max().item()
    tol = 2e-3 * max(1.0, ref.abs().max().item())
    assert err <= tol, (err, tol)
