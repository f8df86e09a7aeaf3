"""Device JPEG decode (csrc/jpeg_host.cpp + csrc/jpeg.hip, mmf_amd/jpeg.py) on the MI355X: decoded
pixels bit-exact with Pillow's decoder (the reference's Image.open(...).convert("RGB")) on every
supported kind of file, and analyze_pairs over encoded files equal -- dict for dict -- to the same
call with every image decoded by Pillow, including chunks that mix device-decoded JPEGs with files
the device path declines (CMYK, lossless, PNG) and PIL images; progressive files included."""
import io
import os

import numpy as np
import pytest
import torch

from tests import jpeg_cases as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine(det_sd):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mmf_amd.engine import Engine
    e = Engine(0, det_sd, None, max_batch=8)
    yield e
    e.close()


@pytest.fixture(scope="module")
def stager():
    from mmf_amd import jpeg
    s = jpeg.JpegStager(workers=4)
    yield s
    s.close()


def test_device_pixels_match_pillow(engine, stager):
    from mmf_amd import jpeg
    cases = C.supported_jpegs(large=True, progressive=True)
    st = stager.stage([d for _, d in cases])
    assert st.index == list(range(len(cases)))
    got = jpeg.device_rgb(engine, stager, st)
    for (name, d), g in zip(cases, got):
        np.testing.assert_array_equal(g, C.pillow_rgb(d), err_msg=name)


def test_staging_slot_growth(engine):
    """A first packed-section guess far too small: records that do not fit are placed after the slot
    grows, and the pixels are unchanged."""
    from mmf_amd import jpeg
    s = jpeg.JpegStager(workers=3)
    s.guess_bytes_per_block = 1
    try:
        cases = C.supported_jpegs(large=True, progressive=True)
        for _ in range(2):  # second pass: the grown slots are reused
            st = s.stage([d for _, d in cases])
            got = jpeg.device_rgb(engine, s, st)
            for (name, d), g in zip(cases, got):
                np.testing.assert_array_equal(g, C.pillow_rgb(d), err_msg=name)
    finally:
        s.close()


def test_declined_files_are_left_to_pillow(engine, stager):
    from mmf_amd import jpeg
    files = C.unsupported_files()
    good = C.supported_jpegs()[0][1]
    st = stager.stage([files[0][1], good, files[1][1], None, files[2][1], good])
    assert st.index == [1, 5]
    a, b = jpeg.device_rgb(engine, stager, st)
    np.testing.assert_array_equal(a, C.pillow_rgb(good))
    np.testing.assert_array_equal(b, a)


def test_oversized_jpeg_left_to_the_host_path(engine, stager):
    """a JPEG whose shortest side is past mmf_resize_pil's tap budget is not staged for the
    device (its windows would fail the whole chunk); the smaller file beside it is."""
    big = C.encode(C.photo_like(5400, 5300, seed=1), quality=60)
    info = np.zeros(16, np.int32)
    assert engine.lib.mmf_jpeg_header(big, len(big), info.ctypes.data) == 0
    assert not engine.resize_supported(5400, 5300)
    good = C.supported_jpegs()[0][1]
    st = stager.stage([big, good])
    assert st.index == [1]


def test_windows_match_pillow_resampling(engine, stager):
    """Device decode -> device resampling == Pillow decode -> Pillow resampling (io_utils)."""
    from PIL import Image

    from mmf_amd import io_utils, jpeg
    cases = C.supported_jpegs(large=True, progressive=True)
    st = stager.stage([d for _, d in cases])
    eff, clp = jpeg.device_windows(engine, stager, st)
    for k, (name, d) in enumerate(cases):
        pil = Image.open(io.BytesIO(d)).convert("RGB")
        np.testing.assert_array_equal(eff[k].cpu().numpy(), io_utils.effnet_pixels(pil), err_msg=name)
        np.testing.assert_array_equal(clp[k].cpu().numpy(), io_utils.clip_pixels(pil), err_msg=name)


@pytest.fixture(scope="module")
def forensics(golden, golden_inputs, det_sd, clip_sd):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from tables import TableClipProcessor, TableRobertaTokenizer
    from misinfo_forensics import MisinfoForensics
    from tests.test_gpu_api import _tables
    rob, clp = _tables(golden, golden_inputs)
    mf = MisinfoForensics(fusion_weights="/nonexistent", faiss_index_path="/nonexistent",
                          roberta_tokenizer=TableRobertaTokenizer(rob), clip_processor=TableClipProcessor(clp),
                          detector_state=det_sd, clip_state=clip_sd, max_batch=4, verbose=False)
    mf.set_vault(golden_inputs["vault"], golden_inputs["meta"])
    return mf


def test_analyze_pairs_on_encoded_files(forensics, golden_inputs, tmp_path):
    """10 pairs in chunks of 4 (both pinned staging slots reused): JPEG bytes, a JPEG file path,
    a progressive JPEG, a CMYK JPEG and a PNG (both declined: Pillow), a PIL image, against the
    all-Pillow run of the same call."""
    from PIL import Image
    imgs = golden_inputs["imgs"]
    n = imgs.shape[0]
    items = []
    for i in range(10):
        a = imgs[i % n]
        if i == 3:
            items.append(C.encode(a, quality=90, progressive=True))
        elif i == 5:
            items.append(C.encode(a, "CMYK", quality=90))
        elif i == 6:
            b = io.BytesIO()
            Image.fromarray(a).save(b, "PNG")
            items.append(b.getvalue())
        elif i == 7:
            items.append(Image.fromarray(a))
        elif i == 8:
            p = tmp_path / "pair8.jpg"
            p.write_bytes(C.encode(a, quality=85, subsampling=1))
            items.append(str(p))
        else:
            items.append(C.encode(a, quality=80 + i, subsampling=2 if i % 2 else 0))
    texts = [f"sample text {i % n}" for i in range(10)]
    forensics.device_jpeg = True
    dev = forensics.analyze_pairs(texts, items)
    forensics.device_jpeg = False
    try:
        host = forensics.analyze_pairs(texts, items)
    finally:
        forensics.device_jpeg = True
    assert len(dev) == 10
    assert dev == host


def test_analyze_pairs_oversized_and_truncated_jpegs(forensics, golden_inputs):
    """An oversized JPEG (shortest side 5300 px > the device resampler's budget) goes through Pillow
    decode + host resampling inside the same chunk, with dicts equal to the all-Pillow call; a
    truncated JPEG raises Pillow's OSError, as the reference's Image.open(...).convert does."""
    imgs = golden_inputs["imgs"]
    big = C.encode(C.photo_like(5400, 5300, seed=1), quality=60)
    items = [C.encode(imgs[0], quality=90), big, C.encode(imgs[1], quality=85)]
    texts = ["sample text 0", "sample text 1", "sample text 1"]
    forensics.device_jpeg = True
    dev = forensics.analyze_pairs(texts, items)
    forensics.device_jpeg = False
    try:
        host = forensics.analyze_pairs(texts, items)
    finally:
        forensics.device_jpeg = True
    assert dev == host
    cut = items[0][:len(items[0]) * 2 // 3]
    with pytest.raises(OSError, match="truncated"):
        forensics.analyze_pairs(texts[:2], [items[2], cut])
