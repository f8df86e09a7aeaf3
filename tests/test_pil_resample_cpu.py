"""Pins oracle/pil_resample.py (the restatement the device resampler is checked against) to Pillow
itself, bit for bit, for both filters, up- and down-scaling, odd sizes and extreme aspect ratios,
and the two tower windows to io_utils' PIL-based geometry."""
import numpy as np
import pytest

from oracle import pil_resample as R

Image = pytest.importorskip("PIL.Image")
from mmf_amd import io_utils  # noqa: E402

CASES = [(640, 480, 224, 224, "bilinear"), (480, 640, 224, 298, "bicubic"), (100, 50, 224, 224, "bilinear"),
         (300, 301, 224, 224, "bicubic"), (1000, 224, 224, 224, "bilinear"), (225, 224, 224, 224, "bilinear"),
         (1200, 900, 298, 224, "bicubic"), (37, 500, 224, 224, "bicubic"), (3, 2, 224, 224, "bicubic"),
         (224, 1000, 224, 224, "bilinear")]


@pytest.mark.parametrize("w,h,ow,oh,name", CASES)
def test_restatement_matches_pillow(w, h, ow, oh, name):
    a = np.random.default_rng(w * 7 + h).integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(a).resize((ow, oh), Image.BILINEAR if name == "bilinear" else Image.BICUBIC))
    np.testing.assert_array_equal(R.resize(a, ow, oh, name), ref)


@pytest.mark.parametrize("w,h", [(640, 480), (480, 640), (224, 224), (225, 300), (50, 80), (1500, 224)])
def test_tower_windows_match_io_utils(w, h):
    a = np.random.default_rng(w + h).integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    pil = Image.fromarray(a)
    np.testing.assert_array_equal(R.effnet_window(a), io_utils.effnet_pixels(pil))
    np.testing.assert_array_equal(R.clip_window(a), io_utils.clip_pixels(pil))
