"""Minimal stand-in for the three OpenCV calls analyze_video makes (misinfo_forensics.py:501-548):
VideoCapture over an in-memory list of BGR uint8 frames, CAP_PROP_FPS, cvtColor(BGR2RGB).
Test infrastructure: OpenCV is absent from this image, and video DECODE is out of scope (SURVEY
§8f F3); what the fixtures pin is the reference's frame sampling and aggregation."""
import sys
import types

import numpy as np

CAP_PROP_FPS = 5
COLOR_BGR2RGB = 4
_VIDEOS = {}


class VideoCapture:
    def __init__(self, path):
        self._v = _VIDEOS.get(str(path))
        self._k = 0

    def isOpened(self):
        return self._v is not None

    def get(self, prop):
        return float(self._v[0]) if prop == CAP_PROP_FPS else 0.0

    def read(self):
        frames = self._v[1]
        if self._k >= len(frames):
            return False, None
        f = np.ascontiguousarray(frames[self._k])
        self._k += 1
        return True, f

    def release(self):
        pass


def cvtColor(frame, code):
    assert code == COLOR_BGR2RGB
    return np.ascontiguousarray(frame[:, :, ::-1])


def install(videos):
    """videos: {path: (fps, [BGR uint8 frames])}; registers this module as ``cv2``."""
    _VIDEOS.clear()
    _VIDEOS.update(videos)
    mod = sys.modules[__name__]
    sys.modules["cv2"] = mod
    return mod
