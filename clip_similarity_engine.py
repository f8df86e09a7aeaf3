"""Drop-in replacement for the reference module ``clip_similarity_engine`` (MI355X / HIP):
``CLIPSimilarityEngine(model_name, threshold)`` with calculate_similarity /
analyze_with_explanation / load_image and the same exceptions (clip_similarity_engine.py:13-174)."""
import mmf_amd  # noqa: F401
from mmf_amd.api import CLIPSimilarityEngine  # noqa: F401

__all__ = ["CLIPSimilarityEngine"]
