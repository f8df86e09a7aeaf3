"""Inputs of the analyze_video fixtures (DATA shared by make_golden.py --video and the tests).

Frame k of a video is synthetic sample image FRAMES[k] (fed as BGR, as OpenCV decodes it).  The
video fixtures use their own Truth-Vault: the golden base vault with samples 0 / 3 / 5 planted at
DISTINCT cosines (0.97 / 0.92 / 0.88), so the reference's "first frame whose discrepancy strictly
exceeds the running best" is decided by margins of >= 0.04, not by float rounding of equal 1.0s."""
import numpy as np

VIDEOS = {
    "v_stride.mp4": {"fps": 10.0, "frames": [1, 2, 4, 6, 7, 6, 2, 1, 4, 3, 0, 2, 2, 7, 1, 6, 5, 5, 4, 1,
                                             6, 4, 2, 3, 1, 7, 7, 0, 5, 3]},
    "v_nofps.mp4": {"fps": 0.0, "frames": [(k * 3) % 8 for k in range(40)]},
    "v_many.mp4": {"fps": 2.0, "frames": [(k * 5 + 1) % 8 for k in range(60)]},
    "v_empty.mp4": {"fps": 30.0, "frames": []},
}
# (video, text sample or None, max_frames, stride_seconds)
VIDEO_CALLS = [("v_stride.mp4", 0, 12, 1.0), ("v_stride.mp4", None, 12, 1.0), ("v_nofps.mp4", 3, 12, 1.0),
               ("v_many.mp4", 5, 12, 0.5), ("v_many.mp4", 2, 4, 2.0), ("v_stride.mp4", 6, 12, 0.05)]
ANALYZE_CALLS = [("v_stride.mp4", 0), ("v_stride.mp4", None), ("v_many.mp4", 5)]
PLANT = {0: (100, 0.97), 3: (1000, 0.92), 5: (2000, 0.88)}  # sample -> (vault row, cosine)


def video_vault(base_vault: np.ndarray, raw_img_emb: np.ndarray) -> np.ndarray:
    """Base vault with each planted row = cos * e + sin * r (unit e = the sample's image embedding
    direction, r a fixed unit vector orthogonal to it), times 2."""
    v = base_vault.copy()
    g = np.random.Generator(np.random.PCG64(2718))
    for s, (row, c) in PLANT.items():
        e = raw_img_emb[s].astype(np.float64)
        e /= np.linalg.norm(e)
        r = g.standard_normal(e.shape[0])
        r -= (r @ e) * e
        r /= np.linalg.norm(r)
        v[row] = (2.0 * (c * e + np.sqrt(1.0 - c * c) * r)).astype(np.float32)
    return v


def bgr_videos(imgs: np.ndarray) -> dict:
    """{path: (fps, [BGR frames])} for cv2_stub.install."""
    return {k: (v["fps"], [imgs[i][:, :, ::-1] for i in v["frames"]]) for k, v in VIDEOS.items()}
