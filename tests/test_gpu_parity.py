"""End-to-end parity of the HIP path (through the C-ABI) against the reference-generated golden
fixtures and the fp32 CPU oracle.  Tolerance (BASELINE.json north_star): the 5-score vector and
the fusion probabilities within 1e-3 of the fp32 reference; verdicts equal."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-3


@pytest.fixture(scope="module")
def engine(det_sd, clip_sd, golden, golden_inputs):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mmf_amd.engine import Engine
    eng = Engine(0, det_sd, clip_sd, eos_token_id=golden_inputs["eos"], max_batch=256)
    assert eng.ready == 31
    gi = golden_inputs
    tmask = np.zeros((2170, 77), np.int32)
    for j, t in enumerate(gi["title_ids"]):
        tmask[j, :len(t)] = 1
    eng.set_vault(gi["vault"], golden["title_clip_ids"], tmask)
    assert eng.ready == 63
    return eng


def _sm1(lg):
    return torch.softmax(torch.as_tensor(lg, dtype=torch.float32), 1)[:, 1].numpy()


def test_text_signals(engine, golden):
    ai, mi, sc = engine.text_forward(golden["rob_ids"], golden["rob_mask"])
    torch.cuda.synchronize()
    sc = sc.cpu().numpy()
    np.testing.assert_allclose(sc[:, 0], _sm1(golden["ai_logits"]), atol=TOL)
    np.testing.assert_allclose(sc[:, 1], _sm1(golden["misinfo_logits"]), atol=TOL)
    np.testing.assert_allclose(ai.cpu().numpy(), golden["ai_logits"], atol=5e-3)


@pytest.fixture(scope="module")
def precise_engine(det_sd, clip_sd, golden_inputs):
    """The golden draw with text_precision "precise": every GEMM kind's hi / lo weights stay packed
    (under "auto" the calibration keeps the fp16 stream here and releases them)."""
    from mmf_amd.engine import Engine
    eng = Engine(0, det_sd, clip_sd, eos_token_id=golden_inputs["eos"], max_batch=8, text_precision="precise")
    yield eng
    eng.close()


def test_text_precise_mode_vs_golden(precise_engine, golden):
    """RoBERTa precise mode (option text_hilo = 2, precise.hip: ~22-bit GEMM operands through the
    K-concatenated [hi | lo | hi] x [W_hi | W_hi | W_lo] product, fp32 stream / LayerNorm /
    attention) against the reference-run logits: fp32-level agreement, far inside the fp16 modes'
    bar; batch 1 too (the skinny split-K path at K = 2304 / 9216)."""
    engine = precise_engine
    assert engine.get_option("text_hilo_effective") == 2 and engine.get_option("text_prec_mask") == 255
    ai, mi, sc = engine.text_forward(golden["rob_ids"], golden["rob_mask"])
    ai1, _, sc1 = engine.text_forward(golden["rob_ids"][:1], golden["rob_mask"][:1])
    torch.cuda.synchronize()
    sc = sc.cpu().numpy()
    da = np.abs(ai.cpu().numpy() - golden["ai_logits"]).max()
    dm = np.abs(mi.cpu().numpy() - golden["misinfo_logits"]).max()
    ds = max(np.abs(sc[:, 0] - _sm1(golden["ai_logits"])).max(), np.abs(sc[:, 1] - _sm1(golden["misinfo_logits"])).max())
    print(f"precise mode vs golden: logits {da:.2e} / {dm:.2e}, scores {ds:.2e}")
    assert ds < 2e-5 and da < 2e-4 and dm < 2e-4
    np.testing.assert_allclose(sc1.cpu().numpy()[0], sc[0], atol=2e-5)


def test_text_precise_mode_long_texts(det_sd, clip_sd):
    """Precise mode past 128 tokens (attention32 over several 128-query blocks and 32-key chunks,
    ragged masks) against the oracle's unpadded single-text analyze_text."""
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle.pipeline import OracleForensics
    lens = [512, 300, 129, 17]
    ids, mask = syn.roberta_ids(len(lens), 512, 79, lens)
    eng = Engine(0, det_sd, None, max_batch=len(lens), max_text_len=512, text_precision="precise")
    assert eng.get_option("text_hilo_effective") == 2
    _, _, sc = eng.text_forward(ids, mask)
    torch.cuda.synchronize()
    sc = sc.cpu().numpy()
    orc = OracleForensics(det_sd, clip_sd)
    d = 0.0
    for i, n in enumerate(lens):
        r = orc.analyze_text(ids[i, :n])
        d = max(d, abs(sc[i, 0] - r["ai_score"]), abs(sc[i, 1] - r["misinfo_score"]))
    print(f"precise mode, L <= 512: max |d score| {d:.2e}")
    assert d < 2e-5
    eng.close()


def test_effnet_signal(engine, golden, golden_inputs):
    lg, sc = engine.effnet_forward(golden_inputs["imgs"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(sc.cpu().numpy(), _sm1(golden["effnet_logits"]), atol=TOL)


def test_effnet_fp32_tower_vs_golden(engine, golden, golden_inputs):
    """The fp32 tower (option effnet_fp32) against the reference-generated logits: fp32 rounding
    throughout, so the logits themselves agree to ~1e-4 (the fp16 tower is checked on its scores)."""
    engine.set_option("effnet_fp32", 1)
    try:
        lg, sc = engine.effnet_forward(golden_inputs["imgs"])
        x = torch.as_tensor(golden_inputs["imgs"]).permute(0, 3, 1, 2).float().div(255.0)
        mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
        std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
        lgf, _ = engine.effnet_forward_f32(((x - mean) / std).contiguous())
        torch.cuda.synchronize()
    finally:
        engine.set_option("effnet_fp32", 0)
    np.testing.assert_allclose(lg.cpu().numpy(), golden["effnet_logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(lgf.cpu().numpy(), golden["effnet_logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(sc.cpu().numpy(), _sm1(golden["effnet_logits"]), atol=1e-5)


def test_fp32_tower_mfma_pointwise_bit_identical(det_sd, clip_sd):
    """The fp32 tower's 1x1 convolutions on the fp32-input MFMA (option pw32_mfma = 1: loads one
    K-chunk ahead; 2: three chunks ahead where K allows -- v_mfma_f32_16x16x4_f32 is a k-ordered
    fp32 fmaf chain; 3, round 5: + whole-row tiles with row-contiguous stores for the K <= 64,
    N <= 256 launches; 4: for every N <= 256 launch; 5, default: 4 where the grid has >= 512-1024
    row blocks) against the fp32-FMA VALU kernel
    (pw32_mfma = 0): every logit bit-identical, on the ill-conditioned He draw the mode exists for."""
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from mmf_amd.engine import Engine
    eng = Engine(0, W.synthetic_detector_state(0, effnet_gain=2 ** 0.5), None, max_batch=64)
    try:
        eng.set_option("effnet_fp32", 1)
        imgs = syn.images(64, 29)
        eng.set_option("pw32_mfma", 0)
        lg0, _ = eng.effnet_forward(imgs)
        for mode in (1, 2, 3, 4, 5):
            eng.set_option("pw32_mfma", mode)
            lg1, _ = eng.effnet_forward(imgs)
            torch.cuda.synchronize()
            assert torch.isfinite(lg1).all()
            assert torch.equal(lg0, lg1), (mode, (lg0 - lg1).abs().max().item())
    finally:
        eng.close()


@pytest.mark.parametrize("B", [3, 37])
def test_compact_last_layer_queries(engine, B):
    """Option last_q1 (round 4): the last encoder layer computes K / V for every row but Q and the
    attention only for the pooled rows (RoBERTa CLS: bit 1, default; CLIP CLS / EOS: bit 2), one
    query per (sequence, head).  The 5 scores and probabilities of every combination agree with the
    full last layer at the north-star tolerance; B = 3 runs the materialised-LN small-batch CLIP path,
    B = 37 the lazy-LN one; ragged texts / captions exercise the key masks and the causal EOS query."""
    import mmf_amd.synthetic as syn
    rid, rm = syn.roberta_ids(B, 128, 41, [128, 90, 7, 33])
    cid, cm = syn.clip_ids(B, 77, 41, [77, 30, 5, 12])
    imgs = syn.images(B, 41)
    outs = {}
    try:
        for v in (0, 1, 3):
            engine.set_option("last_q1", v)
            o = engine.analyze_batch(rid, rm, cid, cm, imgs)
            torch.cuda.synchronize()
            outs[v] = {k: t.cpu().numpy() for k, t in o.items()}
    finally:
        engine.set_option("last_q1", 1)
    for v in (1, 3):
        assert np.isfinite(outs[v]["scores"]).all()
        np.testing.assert_allclose(outs[v]["scores"], outs[0]["scores"], atol=2e-4)
        np.testing.assert_allclose(outs[v]["probs"], outs[0]["probs"], atol=2e-4)
    # bit 1 leaves the CLIP towers untouched: their signals are bit-identical
    np.testing.assert_array_equal(outs[1]["scores"][:, 2:], outs[0]["scores"][:, 2:])


def test_clip_embeddings(engine, golden, golden_inputs):
    ie = engine.clip_image(golden_inputs["imgs"]).cpu().numpy()
    te = engine.clip_text(golden["clip_ids"], golden["clip_mask"]).cpu().numpy()
    # unit vectors: compare directions
    assert (ie * golden["clip_image_embeds"]).sum(1).min() > 1 - 1e-4
    assert (te * golden["clip_text_embeds"]).sum(1).min() > 1 - 1e-4
    np.testing.assert_allclose((ie * te).sum(1), golden["clip_similarity"], atol=TOL)


@pytest.mark.parametrize("B", [3, 37])
def test_lazy_layernorm_clip_matches_materialised(engine, clip_sd, golden_inputs, B):
    """CLIP towers with the LayerNorms folded into the GEMM epilogues (option lazy_ln, default)
    against the materialised add+LN path and the fp32 oracle, at a few rows (B = 3: M = 150 / 231,
    below the persistent GEMM's 256-row tile) and at ragged M (B = 37: 1850 / 2849 rows)."""
    import mmf_amd.synthetic as syn
    from oracle import models as M
    cid, cm = syn.clip_ids(B, 77, 21)
    imgs = syn.images(B, 21)
    out = {}
    try:
        for v in (0, 1):
            engine.set_option("lazy_ln", v)
            out[v] = (engine.clip_image(imgs).cpu().numpy(), engine.clip_text(cid, cm).cpu().numpy())
    finally:
        engine.set_option("lazy_ln", 1)
    csd = M.to_torch(clip_sd)
    with torch.no_grad():
        ie = M.l2n(M.clip_image_features(csd, M.clip_preprocess(torch.as_tensor(imgs)))).numpy()
        te = M.l2n(M.clip_text_features(csd, torch.as_tensor(cid), torch.as_tensor(cm), golden_inputs["eos"])).numpy()
    for v in (0, 1):
        assert (out[v][0] * ie).sum(1).min() > 1 - 1e-4, v
        assert (out[v][1] * te).sum(1).min() > 1 - 1e-4, v
        np.testing.assert_allclose((out[v][0] * out[v][1]).sum(1), (ie * te).sum(1), atol=TOL)
    assert (out[0][0] * out[1][0]).sum(1).min() > 1 - 1e-5
    assert (out[0][1] * out[1][1]).sum(1).min() > 1 - 1e-5


def test_analyze_batch_vs_golden(engine, golden, golden_inputs):
    out = engine.analyze_batch(golden["rob_ids"], golden["rob_mask"], golden["clip_ids"], golden["clip_mask"],
                               golden_inputs["imgs"])
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    np.testing.assert_allclose(o["scores"], golden["scores"], atol=TOL)
    np.testing.assert_allclose(o["probs"], golden["fusion_probs"], atol=TOL)
    np.testing.assert_array_equal(o["verdict"], (golden["fusion_probs"][:, 1] > 0.5).astype(np.int32))
    np.testing.assert_array_equal(o["top_idx"], golden["vault_top_idx"])
    np.testing.assert_allclose(o["top_sims"], golden["vault_top_sim"], atol=TOL)
    # text_similarity (misinfo_forensics.py:467-484, not a fusion input: quirk Q7) at the same bar
    np.testing.assert_allclose(o["text_similarity"], golden["text_similarity"], atol=TOL)


def test_fusion_config1(engine, golden):
    probs, verdict, conf, rule = engine.fusion(golden["fusion_c1_inputs"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(probs.cpu().numpy(), golden["fusion_c1_probs"], atol=1e-5)
    p = golden["fusion_c1_probs"]
    np.testing.assert_array_equal(verdict.cpu().numpy(), (p[:, 1] > 0.5).astype(np.int32))


def test_batch_invariance_full_size(engine, det_sd):
    """B=256, L=128 (the benchmark workload): every row is bit-identical to the same row run in a
    batch of 8 -> sharding rows over GPUs cannot change results."""
    import mmf_amd.synthetic as syn
    B = 256
    rid, rm = syn.roberta_ids(B, 128, 5)
    cid, cm = syn.clip_ids(B, 77, 5)
    imgs = syn.images(B, 5)
    full = engine.analyze_batch(rid, rm, cid, cm, imgs)
    part = engine.analyze_batch(rid[40:48], rm[40:48], cid[40:48], cm[40:48], imgs[40:48])
    torch.cuda.synchronize()
    for k in ("scores", "probs", "top_sims", "top_idx", "text_similarity"):
        a, b = full[k].cpu().numpy(), part[k].cpu().numpy()
        assert np.isfinite(a).all()
        np.testing.assert_array_equal(a[40:48], b, err_msg=k)
    s = full["scores"].cpu().numpy()
    assert ((s[:, :3] >= 0) & (s[:, :3] <= 1)).all() and (np.abs(s[:, 3]) <= 1 + 1e-5).all()


def test_fused_expand_dwconv_bit_identical(engine):
    """The fused MBConv front (1x1 expand computed per tile into the depthwise conv's LDS tile)
    produces bit-identical EfficientNet outputs to the separate expand GEMM + depthwise launches
    (same MFMA operand order over K, same bias / SiLU / fp16 rounding), on a full 256 batch.  The
    separate depthwise launches run the fused kernel's 48-channel groups (dw_cw32 = 0), so the SE pool
    partials are summed in the same order too."""
    import mmf_amd.synthetic as syn
    imgs = syn.images(256, 17)
    engine.set_option("dw_cw32", 0)
    try:
        engine.set_option("fuse_expand", 0)
        lg0, _ = engine.effnet_forward(imgs)
        engine.set_option("fuse_expand", 1)
        lg1, _ = engine.effnet_forward(imgs)
        torch.cuda.synchronize()
    finally:
        engine.set_option("dw_cw32", 1)
    assert torch.equal(lg0, lg1)


def test_fused_stem_dwconv_matches_separate(engine):
    """Stem fused into the stage-1 depthwise conv (stem recomputed per halo tile on the MFMA with
    hi/lo-split fp16 operands) vs the separate fp32-FMA stem kernel + depthwise launch.  The two
    stems round differently in the last fp32 bits, which flips occasional fp16 roundings of the
    stem activation, so the comparison is at the north-star tolerance on deepfake_score and a
    tight bound on the logits; both entry points (uint8 pixels, normalised fp32 NCHW)."""
    import mmf_amd.synthetic as syn
    imgs = syn.images(64, 23)
    engine.set_option("fuse_stem", 0)
    lg0, s0 = engine.effnet_forward(imgs)
    engine.set_option("fuse_stem", 1)
    lg1, s1 = engine.effnet_forward(imgs)
    torch.cuda.synchronize()
    np.testing.assert_allclose(s1.cpu().numpy(), s0.cpu().numpy(), atol=TOL)
    np.testing.assert_allclose(lg1.cpu().numpy(), lg0.cpu().numpy(), atol=2e-2)
    if hasattr(engine, "effnet_forward_f32"):
        mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
        std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
        x = ((torch.as_tensor(imgs[:16]).permute(0, 3, 1, 2).float() / 255.0) - mean) / std
        engine.set_option("fuse_stem", 0)
        _, f0 = engine.effnet_forward_f32(x)
        engine.set_option("fuse_stem", 1)
        _, f1 = engine.effnet_forward_f32(x)
        torch.cuda.synchronize()
        np.testing.assert_allclose(f1.cpu().numpy(), f0.cpu().numpy(), atol=TOL)


def test_long_text_up_to_512(det_sd, clip_sd):
    """RoBERTa inputs past 128 tokens (the reference truncates at 512, misinfo_forensics.py:327-333):
    each padded row must score like the oracle's unpadded single-text analyze_text."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle.pipeline import OracleForensics
    lens = [512, 300, 129, 17]
    ids, mask = syn.roberta_ids(len(lens), 512, 77, lens)
    eng = Engine(0, det_sd, clip_sd, max_batch=len(lens), max_text_len=512)
    _, _, sc = eng.text_forward(ids, mask)
    torch.cuda.synchronize()
    sc = sc.cpu().numpy()
    orc = OracleForensics(det_sd, clip_sd)
    for i, n in enumerate(lens):
        r = orc.analyze_text(ids[i, :n])
        assert abs(sc[i, 0] - r["ai_score"]) < TOL and abs(sc[i, 1] - r["misinfo_score"]) < TOL, (i, n, sc[i], r)
    eng.close()


def test_host_pipeline_matches_device_batches(engine, golden_inputs):
    """engine.HostPipeline (host inputs, H2D on a copy stream, three slots in flight) returns, per
    submitted batch, exactly what analyze_batch returns for the same device-resident batch -- over
    more batches than slots, so every slot is reused."""
    import mmf_amd.synthetic as syn
    B = 16
    batches = []
    for seed in (5, 6, 7, 8, 9, 10, 11):
        rid, rm = syn.roberta_ids(B, 128, seed, [128, 70, 9])
        cid, cm = syn.clip_ids(B, 77, seed, [77, 30, 4])
        batches.append({"rid": torch.from_numpy(rid).pin_memory(), "rm": torch.from_numpy(rm).pin_memory(),
                        "cid": torch.from_numpy(cid).pin_memory(), "cm": torch.from_numpy(cm).pin_memory(),
                        "img": torch.from_numpy(syn.images(B, seed)).pin_memory()})
    pipe = engine.host_pipeline(B, 128, 77)
    got = []
    for i, b in enumerate(batches):
        slot = pipe.submit(b)
        if i >= 1:
            got.append({k: v.clone() for k, v in pipe.result(prev).items()})
        prev = slot
    got.append({k: v.clone() for k, v in pipe.result(prev).items()})
    for b, g in zip(batches, got):
        ref = engine.analyze_batch(b["rid"], b["rm"], b["cid"], b["cm"], b["img"])
        torch.cuda.synchronize()
        for k, v in ref.items():
            assert torch.equal(v.cpu(), g[k]), k


def test_splitk_compact_layers_match_unsplit(engine, golden):
    """The compact last encoder layers and projections (M = batch, K = 512..3072) run split-K
    (fp32 partials over 256-deep K slices + a reduction with the same bias/act/residual order);
    against the unsplit kernel only the fp32 summation order differs."""
    import mmf_amd.synthetic as syn
    B = 64
    rid, rm = syn.roberta_ids(B, 128, 21, [128, 77, 12])
    cid, cm = syn.clip_ids(B, 77, 21, [77, 33, 6])
    imgs = syn.images(B, 21)
    outs = []
    for v in (0, 1):
        engine.set_option("gemm_splitk", v)
        try:
            o = engine.analyze_batch(rid, rm, cid, cm, imgs)
            torch.cuda.synchronize()
            outs.append({k: t.cpu().numpy() for k, t in o.items()})
        finally:
            engine.set_option("gemm_splitk", 1)
    a, b = outs
    np.testing.assert_allclose(a["scores"], b["scores"], atol=2e-4)
    np.testing.assert_allclose(a["probs"], b["probs"], atol=2e-4)
    np.testing.assert_allclose(a["top_sims"], b["top_sims"], atol=2e-4)
    # the top-5 orders agree except where the summation order under test reorders near-equal
    # similarities (the golden vault plants scaled copies of random-init image embeddings, which all
    # point in nearly one direction): a position may differ only between entries whose similarities
    # are within 2e-4 in both runs
    for r in range(B):
        ia, ib = a["top_idx"][r], b["top_idx"][r]
        if np.array_equal(ia, ib):
            continue
        sa = dict(zip(ia.tolist(), a["top_sims"][r].tolist()))
        sb = dict(zip(ib.tolist(), b["top_sims"][r].tolist()))
        for k in np.flatnonzero(ia != ib):
            assert abs(a["top_sims"][r][k] - b["top_sims"][r][k]) < 2e-4, (r, ia, ib)
            assert abs(sa[int(ia[k])] - a["top_sims"][r][k]) < 1e-12
            if int(ib[k]) in sa:
                assert abs(sa[int(ib[k])] - sb[int(ib[k])]) < 2e-4


def test_effnet_config3_batch512(det_sd, clip_sd):
    """BASELINE configs[2]: EfficientNet-B0 at B = 512 (the bench runs 256).  Sampled rows against
    the fp32 oracle at the north-star tolerance, and every row of a slice bit-identical to the
    same images run as a batch of 8 (size-independent property)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    from oracle import models as M
    eng = Engine(0, det_sd, clip_sd, max_batch=512)
    imgs = syn.images(512, 31)
    lg, sc = eng.effnet_forward(imgs)
    lg8, sc8 = eng.effnet_forward(imgs[200:208])
    torch.cuda.synchronize()
    sc, sc8 = sc.cpu().numpy(), sc8.cpu().numpy()
    assert np.isfinite(sc).all() and ((sc >= 0) & (sc <= 1)).all()
    np.testing.assert_array_equal(sc[200:208], sc8)
    np.testing.assert_array_equal(lg.cpu().numpy()[200:208], lg8.cpu().numpy())
    rows = [0, 137, 311, 511]
    sd = M.to_torch(det_sd)
    with torch.no_grad():
        ref = torch.softmax(M.effnet_forward(sd, M.effnet_preprocess(torch.as_tensor(imgs[rows]))), 1)[:, 1].numpy()
    np.testing.assert_allclose(sc[rows], ref, atol=TOL)
    eng.close()


@pytest.mark.parametrize("last_q1", [0, 1])
@pytest.mark.parametrize("B,lengths", [(256, None), (37, [128, 97, 40, 5, 128, 64, 2])])
def test_qkv_attention_epilogue_bit_identical(det_sd, B, lengths, last_q1):
    """RoBERTa at L = 128: the attention run inside the QKV GEMM's epilogue (gemm.hip EPI 3, option
    qkv_attn, head-interleaved QKV weight rows) against the QKV GEMM + attention_kernel<128> pair --
    bit-identical heads, with padded keys, an odd batch (the last tile holds one sequence) and the
    last layer both compact (last_q1) and full."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    eng = Engine(0, det_sd, None, max_batch=256)
    ids, mask = syn.roberta_ids(B, 128, 11, lengths)
    eng.set_option("last_q1", last_q1)
    outs = {}
    for qa in (0, 1):
        eng.set_option("qkv_attn", qa)
        res = eng.text_forward(ids, mask)
        torch.cuda.synchronize()
        outs[qa] = [t.clone() for t in res]
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()


@pytest.mark.parametrize("B", [1, 4, 8])
def test_threaded_tower_enqueue_bit_identical(engine, golden, B):
    """Small batches with the towers enqueued by host threads side by side (option mt_enqueue:
    three workers own the text, CLIP-text and EfficientNet streams, the caller's thread the ViT):
    every output of analyze_batch and clip_consistency bit-identical to the one-thread enqueue, over
    repeated calls."""
    import mmf_amd.synthetic as syn
    rid, rm = syn.roberta_ids(B, 128, 31, [128, 60, 7])
    cid, cm = syn.clip_ids(B, 77, 31, [77, 20])
    imgs = syn.images(B, 31)
    def run():
        out = {k: v.clone() for k, v in engine.analyze_batch(rid, rm, cid, cm, imgs).items()}
        out.update({"cons_" + k: v.clone() for k, v in engine.clip_consistency(imgs, cid, cm).items()})
        torch.cuda.synchronize()
        return out

    mt = engine.get_option("mt_enqueue")
    try:
        engine.set_option("mt_enqueue", 0)
        ref = run()
        engine.set_option("mt_enqueue", 8)
        for _ in range(25):
            out = run()
            for k, v in ref.items():
                assert torch.equal(v, out[k]), k
    finally:
        engine.set_option("mt_enqueue", mt)


@pytest.mark.parametrize("B", [100, 256])
def test_tower_order_bit_identical(engine, B):
    """Option after_text (round 5): in the concurrent B > mt_enqueue step the chosen towers' streams
    wait on an event the RoBERTa stream records after its last layer.  Only the start order of
    independent towers changes, so every output of analyze_batch is bit-identical to the fully
    concurrent step (and to concurrent = 0); ragged texts / captions exercise the masks."""
    import mmf_amd.synthetic as syn
    rid, rm = syn.roberta_ids(B, 128, 91, [128, 64, 9])
    cid, cm = syn.clip_ids(B, 77, 91, [77, 33, 6, 50])
    imgs = syn.images(B, 91)

    def run():
        out = {k: v.clone() for k, v in engine.analyze_batch(rid, rm, cid, cm, imgs).items()}
        torch.cuda.synchronize()
        return out
    names = ("after_text", "concurrent")
    old = {n: engine.get_option(n) for n in names}
    try:
        engine.set_option("concurrent", 1)
        engine.set_option("after_text", 0)
        ref = run()
        for conc, at in ((1, 12), (1, 14), (1, 2), (1, 4), (0, 12)):
            engine.set_option("concurrent", conc)
            engine.set_option("after_text", at)
            for _ in range(2):
                out = run()
                for k, v in ref.items():
                    assert torch.equal(v, out[k]), (conc, at, k)
    finally:
        for n, v in old.items():
            engine.set_option(n, v)
