"""The event profiler behind bench.py's roofline (mmf_profile_begin / mmf_profile_end,
mmf_amd/profiling.py) under every GEMM tile option.

Each profiled launch is binned by (tile instantiation, epilogue, activation).  The kind table
must cover every instantiation gemm_config can return: a kind past the table would index past the
caller's arrays.  Also: the profiled flops of the text tower equal its algorithmic work, whatever
the tiles."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opts", [{}, {"qkv_attn": 0}])
def test_profile_kinds_cover_every_tile_option(det_sd, opts):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from mmf_amd.profiling import profile_kernels
    B, L = 256, 128
    eng = Engine(0, det_sd, None, max_batch=B)
    for k, v in opts.items():
        eng.set_option(k, v)
    ids, mask = syn.roberta_ids(B, L, 3)
    rows = profile_kernels(eng, lambda: eng.text_forward(ids, mask), 2)
    assert rows
    names = [r["kernel"] for r in rows]
    assert all(n and not n.startswith("gemm_f16<?>") for n in names), names
    # (a library with more kinds than NK would have failed mmf_profile_end inside profile_kernels)
    gemm = [r for r in rows if r["kernel"].startswith("gemm")]
    # 12 layers of QKV / out-proj / FFN at M = B*L (the last layer's rows below the attention are
    # the B CLS rows; its K/V GEMM covers every row, its Q the CLS rows)
    flops = sum(r["flops_per_launch"] * r["launches_per_step"] for r in gemm)
    H, I, M = 768, 3072, B * L
    att = 4.0 * B * 12 * L * L * 64 if opts.get("qkv_attn", 1) else 0.0  # attention in the QKV epilogue
    full = 2.0 * M * H * (3 * H + H + 2 * I) + att
    q1 = 2.0 * M * H * 2 * H + 2.0 * B * H * (H + H + 2 * I)  # compact queries (option last_q1)
    q_all = 2.0 * M * H * 3 * H + att + 2.0 * B * H * (H + 2 * I)  # split-stream checkpoints: full QKV
    assert any(flops == pytest.approx(11 * full + last, rel=0.02) for last in (q1, q_all)), flops
