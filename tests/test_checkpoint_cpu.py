"""Host logic of the weight paths (no GPU): the reference's fallback-checkpoint quirks Q2/Q3
(misinfo_forensics.py:260-317 load nothing from the files its own training scripts write), the
detector's change tracking that re-packs device weights after construction, and the constructor's
weight resolution."""
import time

import numpy as np
import pytest
import torch

import mmf_amd.weights as W
from mmf_amd.api import MisinfoForensics, MultiModalMisinfoDetector, resolve_states


def _detector():
    det = MultiModalMisinfoDetector()
    det.load_state_dict({k: torch.as_tensor(v) for k, v in W.synthetic_detector_state(0).items()}, strict=False)
    return det


def _snapshot(det):
    return {k: v.clone() for k, v in det.state_dict().items()}


def _fake_forensics(det):
    fs = object.__new__(MisinfoForensics)
    fs._verbose = False
    fs.detector = det
    return fs


def test_q2_q3_fallback_files_load_nothing(tmp_path):
    """Q2: ai_head_best.pth (train_ai_head.py:50, 495-504) holds a Linear(768,2) `ai_head.weight/bias`
    -> stripped to `weight/bias`, no match in the Sequential's `0.* / 3.*` under strict=False;
    roberta_detective_best.pth (train_roberta_detective.py:223, 309-318) has no misinfo_head keys.
    Q3: efficientnet_cifake_best.pth (train_cifake_forensics.py:374) is a raw timm-named state dict
    (training_pipeline.py:40-44) -> no key matches torchvision's names.  Q1: clip weights are never
    applied.  Every detector tensor must be unchanged afterwards."""
    det = _detector()
    before = _snapshot(det)
    g = torch.Generator().manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    ai = str(tmp_path / "ai_head_best.pth")
    torch.save({"epoch": 4, "model_state_dict": {"ai_head.weight": r(2, 768), "ai_head.bias": r(2),
                                                  "misinfo_head.weight": r(2, 768), "misinfo_head.bias": r(2),
                                                  "fusion_layer.0.weight": r(512, 516)}}, ai)
    rob = str(tmp_path / "roberta_detective_best.pth")
    torch.save({"epoch": 2, "model_state_dict": {"roberta.pooler.dense.weight": r(768, 768),
                                                  "classifier.dense.weight": r(768, 768),
                                                  "classifier.out_proj.weight": r(2, 768),
                                                  "classifier.out_proj.bias": r(2)}}, rob)
    eff = str(tmp_path / "efficientnet_cifake_best.pth")
    torch.save({"efficientnet.conv_stem.weight": r(32, 3, 3, 3), "efficientnet.bn1.weight": r(32),
                "efficientnet.blocks.0.0.conv_dw.weight": r(32, 1, 3, 3),
                "efficientnet.classifier.weight": r(1, 1280), "efficientnet.classifier.bias": r(1),
                "fusion_layer.0.weight": r(512, 1538)}, eff)
    clip = str(tmp_path / "clip_detective_best.pth")
    torch.save({"model_state_dict": {"clip.logit_scale": torch.tensor(2.0)}, "epoch": 1}, clip)
    _fake_forensics(det)._load_individual_weights(ai, rob, eff, clip)
    after = det.state_dict()
    for k, v in before.items():
        assert torch.equal(after[k], v), k


def test_fallback_loader_does_load_matching_keys(tmp_path):
    """Positive control for the test above: a head file whose keys DO match the Sequential
    (`ai_head.0.*`, `ai_head.3.*`) and a torchvision-named EfficientNet file are applied."""
    det = _detector()
    g = torch.Generator().manual_seed(1)
    w0 = torch.randn(256, 768, generator=g)
    ai = str(tmp_path / "ai.pth")
    torch.save({"model_state_dict": {"ai_head.0.weight": w0}}, ai)
    cls = torch.randn(2, 1280, generator=g)
    eff = str(tmp_path / "eff.pth")
    torch.save({"classifier.1.weight": cls}, eff)
    _fake_forensics(det)._load_individual_weights(ai, "/nonexistent", eff, "/nonexistent")
    assert torch.equal(det.ai_head[0].weight, w0)
    assert torch.equal(det.efficientnet.state_dict()["classifier.1.weight"], cls)


class _RecordingEngine:
    """Stands in for the device engine: records what the detector stages and finalizes."""

    def __init__(self):
        self.staged, self.finalized, self.calibrated = [], 0, []

    def load_state(self, sd, prefix=""):
        self.staged.append(sorted(sd))

    def finalize(self):
        self.finalized += 1

    def calibrate(self, components):
        self.calibrated.append(list(components))


def test_detector_change_tracking():
    det = _detector()
    eng = _RecordingEngine()
    det.bind(eng)
    assert det.uploads == {"text": 1, "effnet": 1, "fusion": 1} and eng.finalized == 1
    # every re-pack is followed by the load-time precision calibration of exactly those components
    assert eng.calibrated == [["text", "effnet", "fusion"]]
    assert det.sync() == [] and det.stale_components() == []
    t0 = time.perf_counter()
    for _ in range(20):
        det.sync()
    print(f"unchanged sync(): {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")
    # head-level load (misinfo_forensics.py:274) -> the text component only
    det.ai_head.load_state_dict({k: v + 1 for k, v in det.ai_head.state_dict().items()})
    assert det.stale_components() == ["text"]
    assert det.sync() == ["text"]
    assert any(k.startswith("roberta.") for k in eng.staged[-1]) and "ai_head.0.weight" in eng.staged[-1]
    # an optimizer-style in-place update of the fusion layer
    with torch.no_grad():
        det.fusion_layer[3].bias.add_(0.1)
    assert det.sync() == ["fusion"]
    # a full load_state_dict (train_fusion_judge.py:297, strict) -> every component
    full = {k: torch.as_tensor(v) for k, v in W.synthetic_detector_state(3).items()}
    det.load_state_dict(full)
    assert sorted(det.sync()) == ["effnet", "fusion", "text"]
    # assign=True replaces the tensors (new storage) -> detected through data_ptr
    det.efficientnet.load_state_dict({k[len("efficientnet."):]: v.clone() for k, v in full.items()
                                      if k.startswith("efficientnet.")}, assign=True)
    assert det.sync() == ["effnet"]
    assert det.sync(force=True) == ["text", "effnet", "fusion"]


def test_detector_state_dict_keys_cover_all_components():
    det = _detector()
    comps = {"roberta": "text", "ai_head": "text", "misinfo_head": "text", "efficientnet": "effnet",
             "fusion_layer": "fusion"}
    assert {k.split(".")[0] for k in det.state_dict()} == set(comps)


def test_resolve_states_keeps_explicit_detector_state():
    """An explicit detector_state survives when only the CLIP weights come from disk (the round-1
    constructor replaced it with the synthetic default)."""
    det = {"roberta.x": np.ones(3, np.float32)}
    clip = {"logit_scale": np.zeros(())}
    calls = []

    def loader(d):
        calls.append(d)
        return None, clip
    got_det, got_clip = resolve_states(det, None, None, "/clipdir", loader=loader)
    assert got_det is det and got_clip is clip and calls == ["/clipdir"]
    # both given: nothing is loaded
    assert resolve_states(det, clip, None, "/x", loader=lambda d: pytest.fail("loaded")) == (det, clip)
    # seed fills only the missing one
    d2, c2 = resolve_states(det, None, 0, "/x", loader=lambda d: pytest.fail("loaded"))
    assert d2 is det and "logit_scale" in c2
    with pytest.raises(RuntimeError, match="CLIP"):
        resolve_states(det, None, None, "/x", loader=lambda d: (None, None))
