"""Device resampling of decoded images (mmf_resize_pil) against Pillow and the
oracle restatement: bit-exact EfficientNet squash and CLIP shortest-edge + crop windows for up- and
down-scaling, odd and extreme sizes; the API's analyze_pairs (host decode + device resample)
equals the all-host path."""
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

Image = pytest.importorskip("PIL.Image")

SIZES = [(640, 480), (480, 640), (224, 224), (225, 224), (224, 300), (37, 500), (3, 2), (1500, 224),
         (2000, 1500), (800, 800), (1, 1), (4000, 3000)]


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mmf_amd.engine import Engine
    return Engine(0, None, None, max_batch=8)


def test_resize_matches_pillow(engine):
    from mmf_amd import io_utils
    g = np.random.default_rng(1)
    imgs = [g.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for w, h in SIZES]
    eff, clp = engine.resize_images(imgs)
    eff, clp = eff.cpu().numpy(), clp.cpu().numpy()
    for i, a in enumerate(imgs):
        pil = Image.fromarray(a)
        np.testing.assert_array_equal(eff[i], io_utils.effnet_pixels(pil), err_msg=f"effnet {SIZES[i]}")
        np.testing.assert_array_equal(clp[i], io_utils.clip_pixels(pil), err_msg=f"clip {SIZES[i]}")
    # RGBX sources (Pillow's in-memory layout, 4 bytes per pixel) give the same windows
    e4, c4 = engine.resize_images([np.concatenate([a, np.full(a.shape[:2] + (1,), 7, np.uint8)], -1) for a in imgs])
    np.testing.assert_array_equal(e4.cpu().numpy(), eff)
    np.testing.assert_array_equal(c4.cpu().numpy(), clp)


def test_decoded_views_through_the_device(engine):
    """io_utils.decode_rgb (zero-copy RGBX views when Pillow exports Arrow) -> resize_images equals
    the all-host decode_batch on JPEG bytes, PNG paths and non-RGB modes."""
    from mmf_amd import io_utils
    g = np.random.default_rng(2)
    items = []
    for k, (w, h) in enumerate([(640, 480), (300, 500), (224, 224), (50, 80)]):
        im = Image.fromarray(g.integers(0, 256, size=(h, w, 3), dtype=np.uint8))
        if k == 1:
            im = im.convert("L")
        b = io.BytesIO()
        im.save(b, format="JPEG" if k % 2 == 0 else "PNG")
        items.append(b.getvalue())
    eff, clp = engine.resize_images(io_utils.decode_rgb(items))
    he, hc = io_utils.decode_batch(items)
    np.testing.assert_array_equal(eff.cpu().numpy(), he)
    np.testing.assert_array_equal(clp.cpu().numpy(), hc)


def test_resize_single_output_and_structured_images(engine):
    from oracle import pil_resample as R
    yy, xx = np.mgrid[0:333, 0:517]
    a = np.stack([(xx * 3 + yy) % 256, (xx * yy) % 256, (255 - xx) % 256], -1).astype(np.uint8)
    eff, clp = engine.resize_images([a], clip=False)
    assert clp is None
    np.testing.assert_array_equal(eff.cpu().numpy()[0], R.effnet_window(a))
    _, clp = engine.resize_images([a], effnet=False)
    np.testing.assert_array_equal(clp.cpu().numpy()[0], R.clip_window(a))


def test_resize_rejects_beyond_tap_limit(engine):
    from mmf_amd.hip import MMFError
    with pytest.raises(MMFError):
        engine.resize_images([np.zeros((224, 20000, 3), np.uint8)])
