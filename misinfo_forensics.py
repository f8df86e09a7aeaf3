"""Drop-in replacement for the reference module ``misinfo_forensics`` (MI355X / HIP).

Callers keep their imports unchanged:
    from misinfo_forensics import MisinfoForensics                         # forensics_dashboard.py:10
    from misinfo_forensics import MultiModalMisinfoDetector, MisinfoForensics  # train_fusion_judge.py:21
Everything is implemented in the ``mmf_amd`` package (multi-modal-misinformation-detection-with-
explanation-generation_amd/api.py) on top of libmmf_hip.so.
"""
import json
import os

import mmf_amd  # noqa: F401  (registers the package)
from mmf_amd.api import CLIPSimilarityEngine, MisinfoForensics, MultiModalMisinfoDetector  # noqa: F401

__all__ = ["MisinfoForensics", "MultiModalMisinfoDetector"]


def main():
    """misinfo_forensics.py:930-965 command line."""
    import argparse
    p = argparse.ArgumentParser(description="Misinformation Forensics Analysis")
    p.add_argument("--text", type=str, help="News headline or article text")
    p.add_argument("--image", type=str, help="Path to image file")
    p.add_argument("--video", type=str, help="Path to video file")
    p.add_argument("--gemini-key", type=str, help="Google Gemini API key (optional)")
    p.add_argument("--output", type=str, help="Save results to JSON file")
    a = p.parse_args()
    if not (a.text or a.image or a.video):
        p.error("Provide at least one of --text, --image, or --video")
    forensics = MisinfoForensics(gemini_api_key=a.gemini_key or os.getenv("GOOGLE_API_KEY"))
    results = forensics.analyze(text=a.text, image_path=a.image, video_path=a.video, verbose=True)
    if a.output:
        with open(a.output, "w", encoding="utf-8") as f:
            json.dump(results, f, indent=2, ensure_ascii=False)
        print(f"\n✓ Results saved to {a.output}")


if __name__ == "__main__":
    main()
