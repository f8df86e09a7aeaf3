"""mmf_amd — MI355X-native MisinfoForensics.analyze() 5-signal forward path.

Layout:
  csrc/        hand-written HIP kernels for gfx950 + the C-ABI (libmmf_hip.so)
  hip.py       ctypes binding of the C-ABI (fails loudly when the library is missing)
  weights.py   state-dict layout + deterministic synthetic weights
  synthetic.py seeded synthetic inputs (token ids, uint8 images, vault)
  engine.py    per-device handle: weight upload, analyze_batch()
  api.py       drop-in MisinfoForensics / MultiModalMisinfoDetector / CLIPSimilarityEngine
"""
__version__ = "0.1.0"
