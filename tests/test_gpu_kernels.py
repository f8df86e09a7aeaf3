"""Per-kernel numerics of libmmf_hip.so on a real MI355X against plain PyTorch fp32 references
of the same op (computed on the CPU from the same fp16-rounded operands)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.hip as hip
    return hip.load()


def _f16(x):
    return x.to(torch.float16)


def _act(x, act):
    if act == 1:
        return torch.nn.functional.gelu(x)
    if act == 2:
        return x * torch.sigmoid(1.702 * x)
    if act == 3:
        return torch.nn.functional.silu(x)
    if act == 4:
        return torch.relu(x)
    return x


@pytest.mark.parametrize("M,N,K,act,res", [
    (256, 768, 768, 0, False), (300, 200, 136, 1, True), (1000, 2304, 768, 0, False),
    (4096, 3072, 768, 1, False), (2048, 768, 3072, 0, True), (777, 24, 16, 3, False),
    (5000, 40, 144, 0, True), (12544, 96, 16, 3, False), (64, 512, 512, 0, False), (49 * 3, 1280, 320, 2, False),
    (3000, 200, 128, 2, True), (2600, 1536, 512, 0, False), (1300, 392, 2048, 4, True),
])
def test_gemm_vs_torch_fp32(lib, M, N, K, act, res):
    import mmf_amd.hip as hip
    g = torch.Generator().manual_seed(M * 7 + N)
    A = _f16(torch.randn(M, K, generator=g))
    W = _f16(torch.randn(N, K, generator=g) * 0.05)
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g) if res else None
    ref = _act(A.float() @ W.float().T + bias, act)
    if res:
        ref = ref + R
    dev = torch.device("cuda")
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    Rd = R.to(dev) if res else None
    c32 = torch.empty(M, N, device=dev)
    c16 = torch.empty(M, N, device=dev, dtype=torch.float16)
    hip.check(lib.mmf_gemm_f16(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), hip.ptr(Rd), c32.data_ptr(),
                                c16.data_ptr(), N, M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    out = c32.cpu()
    scale = ref.abs().max().item() + 1e-6
    assert (out - ref).abs().max().item() / scale < 2e-5
    assert ((c16.cpu().float() - ref).abs() <= ref.abs() * 2 ** -7 + 1e-5 * scale).all()


@pytest.mark.parametrize("M,N,K,act", [(1000, 200, 128, 1), (2048, 2304, 768, 0), (777, 392, 512, 2),
                                       (4096, 3072, 768, 1), (300, 136, 64, 0)])
def test_gemm_f16_only_output(lib, M, N, K, act):
    """fp16-only epilogue (paired 16-B stores across lanes l, l^16), incl. column tails."""
    import mmf_amd.hip as hip
    g = torch.Generator().manual_seed(M + 3 * N)
    A = _f16(torch.randn(M, K, generator=g))
    W = _f16(torch.randn(N, K, generator=g) * 0.05)
    bias = torch.randn(N, generator=g)
    ref = _act(A.float() @ W.float().T + bias, act)
    dev = torch.device("cuda")
    c16 = torch.full((M, N + 8), 7.0, device=dev, dtype=torch.float16)  # ldc = N + 8: canary columns
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)  # keep the device buffers alive across the call
    hip.check(lib.mmf_gemm_f16(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), None,
                                None, c16.data_ptr(), N + 8, M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    out = c16.cpu().float()
    scale = ref.abs().max().item()
    assert ((out[:, :N] - ref).abs() <= ref.abs() * 2 ** -7 + 1e-5 * scale).all()
    assert (out[:, N:] == 7.0).all(), "wrote past N"


@pytest.fixture
def gemm_config(lib):
    """Force a GEMM instantiation for the handle-less ops of one test (process default option)."""
    import mmf_amd.hip as hip
    yield lambda c: hip.set_process_option("gemm_config", c)
    hip.set_process_option("gemm_config", -1)


@pytest.mark.parametrize("cfg", [3, 5, 10, 11])
@pytest.mark.parametrize("M,N,K,act,res", [(1000, 2304, 768, 1, False), (777, 392, 512, 0, True),
                                           (130, 136, 64, 2, False)])
def test_gemm_forced_configs(lib, gemm_config, cfg, M, N, K, act, res):
    """Every tile instantiation (process option gemm_config) on ragged M/N, both epilogues."""
    import mmf_amd.hip as hip
    gemm_config(cfg)
    g = torch.Generator().manual_seed(cfg * 1000 + M)
    A = _f16(torch.randn(M, K, generator=g))
    W = _f16(torch.randn(N, K, generator=g) * 0.05)
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g) if res else None
    ref = _act(A.float() @ W.float().T + bias, act)
    if res:
        ref = ref + R
    dev = torch.device("cuda")
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    Rd = torch.nn.functional.pad(R, (0, 8)).to(dev) if res else None  # residual shares ldc = N + 8
    c16 = torch.full((M, N + 8), 7.0, device=dev, dtype=torch.float16)
    c32 = torch.empty(M, N + 8, device=dev) if res else None
    hip.check(lib.mmf_gemm_f16(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), hip.ptr(Rd), hip.ptr(c32),
                                c16.data_ptr(), N + 8, M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    out = c16.cpu().float()
    assert ((out[:, :N] - ref).abs() <= ref.abs() * 2 ** -7 + 1e-5 * scale).all()
    assert (out[:, N:] == 7.0).all(), "wrote past N"
    if res:
        assert (c32.cpu()[:, :N] - ref).abs().max().item() / scale < 2e-5


def _attn_ref(qkv, mask, B, L, H, causal):
    D = H * 64
    x = qkv.float().view(B, L, 3, H, 64)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = q @ k.transpose(-1, -2) * 0.125
    allow = torch.ones(B, L, L, dtype=torch.bool)
    if mask is not None:
        allow &= mask.bool()[:, None, :]
    if causal:
        allow &= torch.tril(torch.ones(L, L, dtype=torch.bool))[None]
    s = s.masked_fill(~allow[:, None], float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2).reshape(B * L, D)


@pytest.mark.parametrize("B,L,H,causal,masked", [
    (3, 128, 12, 0, True), (4, 50, 12, 0, False), (5, 77, 8, 1, True), (2, 5, 12, 0, True), (2, 33, 8, 1, False),
    # L > 128: attention_long_kernel (K/V resident in LDS, online softmax over 128-key chunks)
    (3, 512, 12, 0, True), (2, 512, 12, 0, False), (3, 200, 12, 0, True), (2, 129, 8, 1, True),
    (2, 300, 12, 1, False),
])
def test_attention_vs_torch_fp32(lib, B, L, H, causal, masked):
    import mmf_amd.hip as hip
    g = torch.Generator().manual_seed(L * 13 + H)
    qkv = _f16(torch.randn(B * L, 3 * H * 64, generator=g))
    mask = None
    if masked:
        lens = torch.randint(1, L + 1, (B,), generator=g)
        lens[0] = L
        mask = (torch.arange(L)[None] < lens[:, None]).int()
    ref = _attn_ref(qkv, mask, B, L, H, causal)
    dev = torch.device("cuda")
    out = torch.empty(B * L, H * 64, device=dev, dtype=torch.float16)
    md = mask.to(dev, torch.int32) if mask is not None else None
    qkv_d = qkv.to(dev)
    hip.check(lib.mmf_attention_f16(qkv_d.data_ptr(), hip.ptr(md), out.data_ptr(), B, L, H, causal,
                                     hip.stream_ptr()))
    torch.cuda.synchronize()
    got = out.cpu().float()
    if mask is not None:  # padded query rows are don't-care in every caller; compare real rows
        keep = mask.reshape(-1).bool()
        got, ref = got[keep], ref[keep]
    # P is rounded to fp16 before P.V (fp32 accumulate): ~2^-8 relative per term
    assert (got - ref).abs().max().item() < 2e-2
    assert (got - ref).abs().mean().item() < 2e-3


# EfficientNet 1x1 convolutions (M = B*H*W pixels): expand (SiLU) and project (SE scale on A,
# optional fp16 residual); shapes of the real blocks at small batch, plus ragged M / N tails.
@pytest.mark.parametrize("M,N,K,act,scale,res", [
    (8 * 3136, 96, 16, 3, False, False), (4 * 3136, 144, 24, 3, False, False), (2 * 784, 240, 40, 3, False, False),
    (3 * 196, 480, 80, 3, False, False), (3 * 196, 672, 112, 3, False, False), (2 * 12544, 16, 32, 0, True, False),
    (3 * 3136, 24, 96, 0, True, False), (3 * 3136, 24, 144, 0, True, True), (2 * 784, 40, 240, 0, True, True),
    (5 * 49, 192, 1152, 0, True, True), (2 * 49, 320, 1152, 0, True, False), (4099, 40, 144, 0, True, True),
    (2053, 136, 48, 3, False, False),
])
def test_gemm_effnet_convs(lib, M, N, K, act, scale, res):
    import mmf_amd.hip as hip
    g = torch.Generator().manual_seed(M + N + K)
    rpb = {8 * 3136: 3136, 4 * 3136: 3136, 3 * 3136: 3136, 2 * 784: 784, 3 * 196: 196, 2 * 12544: 12544,
           5 * 49: 49, 2 * 49: 49}.get(M, 1000)
    A = _f16(torch.randn(M, K, generator=g))
    W = _f16(torch.randn(N, K, generator=g) * (2.0 / K) ** 0.5)
    bias = torch.randn(N, generator=g) * 0.1
    S = torch.rand((M + rpb - 1) // rpb, K, generator=g) if scale else None
    R = _f16(torch.randn(M, N, generator=g)) if res else None
    Af = A.float()
    if scale:
        Af = (Af * S.repeat_interleave(rpb, 0)[:M]).to(torch.float16).float()  # A*s rounded to fp16
    ref = _act(Af @ W.float().T + bias, act)
    if res:
        ref = ref + R.float()
    dev = torch.device("cuda")
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    Sd = S.to(dev) if scale else None
    Rd = R.to(dev) if res else None
    out = torch.full((M, N), 7.0, device=dev, dtype=torch.float16)
    hip.check(lib.mmf_gemm_f16_ex(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), hip.ptr(Rd), hip.ptr(Sd), rpb,
                                   out.data_ptr(), N, M, N, K, act, hip.stream_ptr()))
    torch.cuda.synchronize()
    got = out.cpu().float()
    scale_ = ref.abs().max().item()
    assert ((got - ref).abs() <= ref.abs() * 2 ** -7 + 2e-5 * scale_).all()


@pytest.mark.parametrize("cfg", [10, 11])
@pytest.mark.parametrize("split_lo", [0, 1])
@pytest.mark.parametrize("M,N,K", [(1000, 3072, 768), (777, 392, 512), (4096, 768, 2304)])
def test_gemm_split_operand_epilogue_bit_identical(lib, gemm_config, cfg, split_lo, M, N, K):
    """The precise mode's FFN-1 epilogue (epi 4: GELU output written as hi | lo | hi fp16 thirds) is
    bit-identical to the fp32 output of the same tile split on the host: hi = fp16(c32),
    lo = fp16(c32 - hi); nothing is written past N (split_lo 0) / 3N (split_lo 1)."""
    import mmf_amd.hip as hip
    gemm_config(cfg)
    g = torch.Generator().manual_seed(M + 5 * N + K)
    A = _f16(torch.randn(M, K, generator=g))
    W = _f16(torch.randn(N, K, generator=g) * 0.05)
    bias = torch.randn(N, generator=g)
    dev = torch.device("cuda")
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    c32 = torch.empty(M, N, device=dev)
    hip.check(lib.mmf_gemm_f16(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), None, c32.data_ptr(), None, N,
                                M, N, K, 1, hip.stream_ptr()))
    ld = 3 * N + 8
    s3 = torch.full((M, ld), 7.0, device=dev, dtype=torch.float16)
    hip.check(lib.mmf_gemm_f16_split(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), s3.data_ptr(), ld, M, N, K,
                                      1, split_lo, hip.stream_ptr()))
    torch.cuda.synchronize()
    c = c32.cpu()
    hi = c.half()
    lo = (c - hi.float()).half()
    out = s3.cpu()
    assert torch.equal(out[:, :N].view(torch.int16), hi.view(torch.int16))
    if split_lo:
        assert torch.equal(out[:, N:2 * N].view(torch.int16), lo.view(torch.int16))
        assert torch.equal(out[:, 2 * N:3 * N].view(torch.int16), hi.view(torch.int16))
        assert (out[:, 3 * N:] == 7.0).all(), "wrote past 3N"
    else:
        assert (out[:, N:] == 7.0).all(), "wrote past N"
