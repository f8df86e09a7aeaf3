"""Truth-Vault edge cases on the HIP path against the reference's own search_vault results
(tests/golden/golden_vault_edge.json, made by tests/golden/make_golden.py --vault-edge, which ran
misinfo_forensics.py:410-491 on the tests/golden/vault_edge.py inputs).

What is compared, per query and top_k in {5, 12} (the register top-k and the LDS-sort top-k):
* similarities within 1e-6 (fp32 dot products in another summation order), NaN where the
  reference has NaN (zero rows, 0/0 in the renormalisation);
* vault_discrepancy (> 0.85 rule; NaN is never a hit) within 1e-6;
* indices equal, except inside groups of rows whose similarities are equal to within 1e-6: the
  reference ranks those with numpy's default argsort, which is not stable (its tie order varies with
  the data and the platform; the fixtures show ascending, descending and mixed orders), so there
  the test checks that both sides picked rows of the same tie group.  The HIP ranking orders ties
  by descending index (what a stable argsort gives)."""
import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


@pytest.fixture(scope="module")
def fixture():
    with open(os.path.join(HERE, "golden", "golden_vault_edge.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def engine(det_sd, clip_sd):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mmf_amd.engine import Engine
    eng = Engine(0, None, clip_sd, max_batch=8)
    yield eng
    eng.close()


@pytest.mark.parametrize("name", ["fp16", "ties", "zero", "threshold"])
def test_vault_edge_case(engine, fixture, name):
    import zlib
    import vault_edge as VE
    from mmf_amd import io_utils
    vault, q = VE.case(name)
    case = fixture["cases"][name]
    assert str(vault.dtype) == case["dtype"] and zlib.crc32(np.ascontiguousarray(vault).tobytes()) == case["vault_crc"]
    engine.set_vault(vault)
    # the reference's query: get_image_features / its norm in torch fp32 (misinfo_forensics.py:439)
    qt = torch.as_tensor(q)
    qu = (qt / qt.norm(dim=-1, keepdim=True)).numpy()
    # tie groups from the reference's own arithmetic (numpy, the vault's dtype)
    sims_np = io_utils.vault_unit_rows(vault) @ qu.T  # [N, NQ]
    for r in case["results"]:
        i, k = r["query"], r["top_k"]
        sims, idx, disc, _ = engine.vault_topk(torch.as_tensor(qu[i:i + 1]).cuda(), k, 0.85)
        torch.cuda.synchronize()
        sims, idx, disc = sims.cpu().numpy()[0], idx.cpu().numpy()[0], float(disc.item())
        ref_s = np.array(r["sims"], dtype=np.float64)
        assert len(ref_s) == k
        np.testing.assert_array_equal(np.isnan(sims), np.isnan(ref_s), err_msg=f"{name} q{i} k{k} NaN rows")
        fin = ~np.isnan(ref_s)
        np.testing.assert_allclose(sims[fin], ref_s[fin], atol=1e-6, err_msg=f"{name} q{i} k{k}")
        assert abs(disc - r["vault_discrepancy"]) < 1e-6, (name, i, k, disc, r["vault_discrepancy"])
        for p, (a, b) in enumerate(zip(idx.tolist(), r["idx"])):
            if a == b:
                continue
            sa, sb = sims_np[a, i], sims_np[b, i]
            same = (np.isnan(sa) and np.isnan(sb)) or abs(float(sa) - float(sb)) <= 1e-6
            assert same, f"{name} q{i} k{k} pos {p}: got row {a} ({sa}), reference row {b} ({sb})"


def test_top_k_any_size(engine, fixture):
    """search_vault's top_k is free: k = 1 .. N (k > 8 takes the LDS sort kernel); the result is
    always the first k of the full ranking."""
    import vault_edge as VE
    vault, q = VE.case("threshold")
    engine.set_vault(vault)
    qu = torch.as_tensor(q / np.linalg.norm(q, axis=1, keepdims=True)).cuda()
    full_s, full_i, _, _ = engine.vault_topk(qu, VE.N, 0.85)
    for k in (1, 5, 8, 9, 64, 700):
        s, i, _, _ = engine.vault_topk(qu, k, 0.85)
        torch.cuda.synchronize()
        assert torch.equal(i, full_i[:, :k]) and torch.equal(s, full_s[:, :k]), k
    fs = full_s.cpu().numpy()
    assert (np.diff(fs, axis=1) <= 0).all()  # descending
    assert sorted(full_i.cpu().numpy()[0].tolist()) == list(range(VE.N))  # a permutation


@pytest.mark.parametrize("N", [3, 7, 1001, 2171])
def test_vault_kernels_match_reference_kernels(engine, N):
    """the production vault path (fp32-MFMA similarities, register top-k with its
    block / merge structure) against the reference kernels kept callable at run time (option
    vault_ref: the VALU similarity kernel -- one fp32 FMA chain per output in k order -- and the full
    LDS sort): bit-identical similarities, indices, discrepancies and caption similarities, on
    ragged vault sizes (N % 4 != 0, N < 8) and every register-kernel k <= N."""
    rng = np.random.default_rng(N)
    vault = rng.standard_normal((N, 512)).astype(np.float32)
    B = 8  # (the fixture engine's reserved batch)
    q = rng.standard_normal((B, 512)).astype(np.float32)
    q[:5] = vault[rng.integers(0, N, 5)] * 3.0  # planted hits above the 0.85 threshold
    ids = np.full((N, 77), 49407, np.int32)
    ids[:, 0] = 49406
    mask = np.zeros_like(ids)
    mask[:, :2] = 1
    engine.set_vault(vault, ids, mask)
    qu = torch.as_tensor(q / np.linalg.norm(q, axis=1, keepdims=True)).cuda()
    temb = torch.nn.functional.normalize(torch.randn(B, 512, generator=torch.Generator().manual_seed(N))).cuda()
    old = engine.get_option("vault_ref")
    try:
        for k in [k for k in (1, 3, 5, 8) if k <= N]:  # (mmf_vault_topk: k <= N, as search_vault's argsort)
            engine.set_option("vault_ref", 0)
            got = [t.clone() for t in engine.vault_topk(qu, k, 0.85, temb)]
            engine.set_option("vault_ref", 1)
            ref = [t.clone() for t in engine.vault_topk(qu, k, 0.85, temb)]
            torch.cuda.synchronize()
            for name, a, b in zip(("sims", "idx", "disc", "text_sim"), got, ref):
                assert torch.equal(a, b), (N, k, name)
    finally:
        engine.set_option("vault_ref", old)


def test_vault_reload_frees_device_memory(engine):
    """mmf_set_vault_normalized / mmf_set_vault_titles replace (and free) the previous vault: ten
    reloads leave the handle's device bytes and the device's free memory where they were."""
    import vault_edge as VE
    vault, _ = VE.case("ties")
    ids = np.full((VE.N, 77), 49407, np.int32)
    ids[:, 0] = 49406
    mask = np.zeros_like(ids)
    mask[:, :2] = 1
    engine.set_vault(vault, ids, mask)
    torch.cuda.synchronize()
    b0, f0 = engine.device_bytes, torch.cuda.mem_get_info()[0]
    for _ in range(10):
        engine.set_vault(vault, ids, mask)
    torch.cuda.synchronize()
    assert engine.device_bytes == b0
    assert abs(torch.cuda.mem_get_info()[0] - f0) < 8 << 20


@pytest.mark.parametrize("n_rows", [1, 2, 3])
def test_analyze_batch_with_short_vault(det_sd, clip_sd, n_rows):
    """A vault of fewer than 5 rows through the 5-signal batch: the reference's
    argsort(sims)[-5:][::-1] keeps all N rows, so analyze_batch returns N matches per pair (slots
    N..4 hold idx -1, which the dict builder drops), ranked as search_vault ranks them, and the
    discrepancy of the top-1 row."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mmf_amd.synthetic as syn
    from mmf_amd.engine import Engine
    B = 4
    eng = Engine(0, det_sd, clip_sd, max_batch=B, max_text_len=32)
    try:
        rid, rm = syn.roberta_ids(B, 32, 5, [32, 20, 7, 3])
        cid, cm = syn.clip_ids(B, 77, 5, [77, 12, 5, 2])
        imgs = syn.images(B, 5)
        emb = eng.clip_image(imgs)
        vault = syn.vault(n_rows, 512, 7)
        vault[0] = emb[1].cpu().numpy() * 2.0  # a planted hit for pair 1 (> 0.85)
        eng.set_vault(vault)
        out = eng.analyze_batch(rid, rm, cid, cm, imgs)
        s_all, i_all, d_all, _ = eng.vault_topk(emb, n_rows, 0.85)
        torch.cuda.synchronize()
        idx = out["top_idx"].cpu().numpy()
        assert (idx[:, n_rows:] == -1).all()
        np.testing.assert_array_equal(idx[:, :n_rows], i_all.cpu().numpy())
        np.testing.assert_allclose(out["top_sims"].cpu().numpy()[:, :n_rows], s_all.cpu().numpy(), atol=1e-6)
        np.testing.assert_allclose(out["scores"].cpu().numpy()[:, 4], d_all.cpu().numpy(), atol=1e-6)
        assert out["scores"][1, 4].item() > 0.85
    finally:
        eng.close()
