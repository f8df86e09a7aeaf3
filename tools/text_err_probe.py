"""Max |device - fp32 reference| of the two text scores on the golden set and on 256 bench-shaped
rows vs the oracle (GPU box; prints one JSON line).  Used to compare residual-stream layouts."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import mmf_amd.synthetic as syn  # noqa: E402
import mmf_amd.weights as W  # noqa: E402
from mmf_amd.engine import Engine  # noqa: E402
from oracle import models as M  # noqa: E402

det, clip = W.synthetic_detector_state(0), W.synthetic_clip_state(0)
g = dict(np.load(os.path.join(REPO, "tests", "golden", "golden.npz")))
eng = Engine(0, det, clip, max_batch=64)
_, _, sc = eng.text_forward(g["rob_ids"], g["rob_mask"])
sc = sc.cpu().numpy()
sm = lambda lg: torch.softmax(torch.as_tensor(lg, dtype=torch.float32), 1)[:, 1].numpy()  # noqa: E731
e_gold = [float(np.abs(sc[:, 0] - sm(g["ai_logits"])).max()), float(np.abs(sc[:, 1] - sm(g["misinfo_logits"])).max())]
rid, rm = syn.roberta_ids(32, 128, 99, [128, 100, 60, 17])
_, _, sc2 = eng.text_forward(rid, rm)
sc2 = sc2.cpu().numpy()
sd = M.to_torch(det)
with torch.no_grad():
    h = M.roberta_forward(sd, torch.as_tensor(rid).long(), torch.as_tensor(rm).long())
    ai, mi = M.text_heads(sd, h[:, 0, :])
ref = np.stack([torch.softmax(ai, 1)[:, 1].numpy(), torch.softmax(mi, 1)[:, 1].numpy()], 1)
e_rand = np.abs(sc2 - ref).max(0).tolist()
print(json.dumps({"golden_max_err": e_gold, "rand32_max_err": e_rand}))
