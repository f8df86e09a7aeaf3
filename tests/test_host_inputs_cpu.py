"""Host input stage: the threaded batch decode returns exactly the serial per-image
geometry of both towers (EfficientNet squash-resize, CLIP shortest-edge resize + centre crop) for
paths, PIL images and encoded bytes of any size / mode."""
import io

import numpy as np
import pytest

from mmf_amd import io_utils

Image = pytest.importorskip("PIL.Image")


def _images(tmp_path):
    g = np.random.default_rng(5)
    out = []
    for k, (w, h, mode) in enumerate([(640, 480, "RGB"), (300, 500, "L"), (224, 224, "RGBA"), (50, 80, "RGB"),
                                      (1000, 224, "RGB"), (225, 224, "RGB")]):
        a = g.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        im = Image.fromarray(a).convert(mode)
        if k % 3 == 0:
            b = io.BytesIO()
            im.convert("RGB").save(b, format="JPEG", quality=90)
            out.append(b.getvalue())
        elif k % 3 == 1:
            p = tmp_path / f"im{k}.png"
            im.save(p)
            out.append(str(p))
        else:
            out.append(im)
    return out


def test_decode_batch_matches_serial(tmp_path):
    ims = _images(tmp_path)
    eff, clp = io_utils.decode_batch(ims, workers=4)
    for i, im in enumerate(ims):
        pil = io_utils.to_pil(Image.open(io.BytesIO(im)) if isinstance(im, bytes) else im)
        np.testing.assert_array_equal(eff[i], io_utils.effnet_pixels(pil))
        np.testing.assert_array_equal(clp[i], io_utils.clip_pixels(pil))
    eff1, clp1 = io_utils.decode_batch(ims, workers=1)
    np.testing.assert_array_equal(eff, eff1)
    np.testing.assert_array_equal(clp, clp1)


def test_decode_batch_into_caller_buffers(tmp_path):
    ims = _images(tmp_path)[:3]
    buf = (np.zeros((3, 224, 224, 3), np.uint8), np.zeros((3, 224, 224, 3), np.uint8))
    eff, clp = io_utils.decode_batch(ims, out=buf)
    assert eff is buf[0] and clp is buf[1] and eff.any()
