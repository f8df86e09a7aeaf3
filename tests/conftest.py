"""Shared fixtures.  `-m gpu` tests need a real MI355X; everything else runs on CPU."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libmmf_hip.so")


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(os.path.join(GOLDEN, "golden.npz")))


@pytest.fixture(scope="session")
def golden_json():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def det_sd():
    import mmf_amd.weights as W
    return W.synthetic_detector_state(0)


@pytest.fixture(scope="session")
def clip_sd():
    import mmf_amd.weights as W
    return W.synthetic_clip_state(0)


@pytest.fixture(scope="session")
def golden_inputs(golden, golden_json):
    """Inputs of the golden run, regenerated from seeds (images, base vault) + stored ids."""
    import zlib
    import mmf_amd.synthetic as syn
    meta = golden_json["meta"]
    seeds = meta["seeds"]
    imgs = syn.images(meta["B"], seeds[1])
    assert zlib.crc32(imgs.tobytes()) == meta["images_crc"], "synthetic image generator drifted"
    vault = syn.vault(2170, 512, seeds[2])
    assert zlib.crc32(vault.tobytes()) == meta["vault_base_crc"], "synthetic vault generator drifted"
    for s, row in meta["plant"].items():
        vault[int(row)] = golden["clip_image_features_raw"][int(s)] * np.float32(3.0)
    titles = [{"title": f"Guardian article {j}", "url": f"https://example.org/a/{j}", "date": "N/A"}
              for j in range(2170)]
    title_ids = [golden["title_clip_ids"][j, :golden["title_lens"][j]] for j in range(2170)]
    return dict(imgs=imgs, vault=vault, meta=titles, title_ids=title_ids,
                rob_lens=meta["rob_lens"], clip_lens=meta["clip_lens"], eos=meta["eos_token_id"])
