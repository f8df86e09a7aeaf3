"""Host-side text products of the path: the rule-based explanation (the reference's Gemini
fallback), the Gemini prompt, and the CLIP engine's explanation bands.  Pure string formatting of
numbers the HIP path produced; the rule INDEX is also computed on device by the fusion kernel
(mmf_fusion `rule` output), so a batch can be explained without re-evaluating the cascade.
"""
from __future__ import annotations

from typing import Dict, List

RULE_VAULT, RULE_DEEPFAKE, RULE_AI, RULE_MISINFO, RULE_CLIP, RULE_DEFAULT = range(6)


def explanation_rule(s: Dict) -> int:
    """Which branch of misinfo_forensics.py:747-765 fires."""
    if s["vault_discrepancy"] > 0.7:
        return RULE_VAULT
    if s["deepfake_score"] > 0.7:
        return RULE_DEEPFAKE
    if s["ai_score"] > 0.7:
        return RULE_AI
    if s["misinfo_score"] > 0.7:
        return RULE_MISINFO
    if s["clip_similarity"] < 0.3:
        return RULE_CLIP
    return RULE_DEFAULT


def fallback_explanation(all_scores: Dict, vault_matches: List[Dict], rule: int | None = None) -> str:
    """_generate_fallback_explanation (misinfo_forensics.py:742-765), same strings."""
    v = "FAKE" if all_scores["verdict"] == 1 else "REAL"
    r = explanation_rule(all_scores) if rule is None else int(rule)
    head = f"This content is classified as {v}. "
    if r == RULE_VAULT:
        return (head + "Our database found this image was previously published in a different context "
                f"(\"{vault_matches[0]['title']}\"), suggesting potential misuse.")
    if r == RULE_DEEPFAKE:
        return head + ("The image shows strong signs of digital manipulation (deepfake probability: "
                       f"{all_scores['deepfake_score']:.1%}).")
    if r == RULE_AI:
        return head + "The text exhibits characteristics typical of AI-generated content."
    if r == RULE_MISINFO:
        return head + "The text uses language patterns commonly associated with misinformation."
    if r == RULE_CLIP:
        return head + "The image and caption show poor alignment, suggesting potential mismatching."
    return (f"This content is classified as {v} with {all_scores['confidence']:.1%} confidence. "
            "Multiple signals from text analysis, image forensics, and database checks support this assessment.")


def gemini_prompt(all_scores: Dict, vault_matches: List[Dict]) -> str:
    """build_gemini_prompt (misinfo_forensics.py:617-693).  Only used when a Gemini client is
    configured (network, out of scope); kept so the prompt text is available offline."""
    verdict_text = "FAKE" if all_scores.get("verdict", 0) == 1 else "REAL"
    confidence = float(all_scores.get("confidence", 0.0) or 0.0)
    lines = [
        "You are a senior misinformation forensics analyst writing a detailed but concise report for a dashboard.",
        "",
        "    Write the response in Markdown with the exact section headers below, using the provided numeric "
        "signals verbatim where relevant.",
        "",
        "    Rules:",
        "    - Be specific: cite key numbers (probabilities/similarities) and explain what they imply.",
        "    - Rank the top signals (strongest to weakest) and explain how they contributed.",
        "    - If a modality is missing (text/image/video), explicitly note what was skipped and how that limits "
        "confidence.",
        "    - Avoid generic advice; focus on evidence-based reasoning.",
        "    - Keep it readable: 120–220 words total.",
        "",
        "    Use this format:",
        "    ### Verdict",
        "    <1–2 sentences with verdict + confidence and the core reason>",
        "",
        "    ### Key Evidence (ranked)",
        "    - <bullet 1>",
        "    - <bullet 2>",
        "    - <bullet 3>",
        "",
        "    ### Cross-Checks & Caveats",
        "    - <1–2 bullets about vault/consistency or missing signals>",
        "",
        "    ### Recommended Next Step",
        "    <1 sentence: what the user should do to verify>",
        "",
        "FORENSIC ANALYSIS SCORES:",
        "",
        "1. Final Verdict & Confidence:",
        f"   - Verdict: {verdict_text}",
        f"   - Confidence Score: {confidence:.1%} (derived from softmax probabilities)",
        f"   - REAL Probability: {all_scores.get('real_probability', 0.0):.2%}",
        f"   - FAKE Probability: {all_scores.get('fake_probability', 0.0):.2%}",
        "",
        "2. AI-Text & Propaganda Probability:",
        f"   - AI-Generated Score: {all_scores.get('ai_score', 0.0):.2%} (RoBERTa classifier, higher = more AI-like)",
        f"   - Propaganda/Misinfo Score: {all_scores.get('misinfo_score', 0.0):.2%} (trained on WELFake dataset)",
        "",
        "3. Deepfake Visual Score:",
        f"   - Deepfake Probability: {all_scores.get('deepfake_score', 0.0):.2%} (EfficientNet on CIFAKE dataset)",
        "",
        "4. Consistency (CLIP) & Vault Discrepancy:",
        f"    - Image-Text Consistency: {float(all_scores.get('clip_similarity', 0.0) or 0.0):.4f} "
        "(cosine similarity, -1 to 1)",
        f"    - Historical Database Match: {float(all_scores.get('vault_discrepancy', 0.0) or 0.0):.2%} "
        "(image found in Guardian archive)",
        "",
    ]
    prompt = "\n".join(lines)
    if vault_matches and all_scores.get("vault_discrepancy", 0.0) > 0.5:
        top = vault_matches[0]
        ts = float(all_scores.get("text_similarity", 0.0) or 0.0)
        prompt += (f"\n5. Truth Vault Cross-Check:\n   - Match Found: \"{top['title']}\"\n"
                   f"   - Image Similarity: {top['similarity']:.1%}\n"
                   f"   - Text Similarity Score: {ts:.2%} (CLIP text encoder comparison)\n"
                   f"   - Published: {top.get('date', 'N/A')}\n   - Context: Image reused from different story\n")
    prompt += ("\n\nTask: Produce the Markdown report using the structure above. Emphasize the strongest "
               "quantitative signals and any contradictions (e.g., high vault match but low text similarity, "
               "or strong text signal but weak visual signal).")
    return prompt


def clip_engine_explanation(similarity: float, label: str) -> str:
    """CLIPSimilarityEngine._generate_explanation (clip_similarity_engine.py:152-174)."""
    if label == "Match":
        if similarity >= 0.7:
            return f"Strong match detected (score: {similarity:.4f}). The image and text are highly consistent."
        if similarity >= 0.5:
            return f"Moderate match detected (score: {similarity:.4f}). The image and text show reasonable alignment."
        return f"Weak match detected (score: {similarity:.4f}). The image and text are barely above the threshold."
    if similarity < 0.1:
        return f"Strong mismatch detected (score: {similarity:.4f}). The image and text appear completely unrelated."
    return (f"Mismatch detected (score: {similarity:.4f}). The image and text show inconsistencies that may "
            "indicate misinformation.")
