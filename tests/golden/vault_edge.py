"""Truth-Vault edge cases (inputs only), shared by make_golden.py (which runs the reference's own
search_vault, misinfo_forensics.py:410-491, on them) and tests/test_gpu_vault_edge.py (which runs
the HIP vault path on the same inputs).  Every case is rebuilt from seeds here: no array is stored.

* fp16      - the vault pickled as float16 rows (search_vault then renormalises in float16,
              misinfo_forensics.py:443-445); three rows hold scaled copies of query directions.
* ties      - exact duplicate rows (one photo reused by several articles): exact ties at the top
              and inside the top 5.
* zero      - all-zero rows: 0/0 = NaN similarities, which numpy's argsort puts last, so the
              reversed tail lists them FIRST (and NaN > 0.85 is False: discrepancy 0).
* threshold - rows planted at cosine 0.85 +- {1e-3, 5e-4, 5e-5} of their query (the > 0.85 rule
              of misinfo_forensics.py:463-468 on both sides of the boundary).
"""
import numpy as np

N, D, NQ = 2170, 512, 6


def _rng(tag: str) -> np.random.Generator:
    import zlib
    return np.random.Generator(np.random.PCG64(zlib.crc32(tag.encode())))


def _unit(v):
    return (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(np.float32)


def queries(tag: str) -> np.ndarray:
    """Raw (un-normalised) fp32 query image features [NQ, D] (the reference normalises them)."""
    return (_rng("q" + tag).standard_normal((NQ, D)) * 3.0).astype(np.float32)


def _base(tag: str) -> np.ndarray:
    return _rng("v" + tag).standard_normal((N, D)).astype(np.float32)


def case(name: str):
    """(vault [N, D] in the case's dtype, raw queries [NQ, D] fp32)."""
    q = queries(name)
    v = _base(name)
    if name == "fp16":
        for i, r in ((0, 17), (2, 905), (4, 2169)):
            v[r] = q[i] * np.float32(2.5)
        v = v.astype(np.float16)
    elif name == "ties":
        for r in (10, 500, 2000):           # exact copies of q0 -> a 3-way tie at the top
            v[r] = q[0] * np.float32(3.0)
        v[700] = q[0] * np.float32(3.0) + np.float32(1e-3)  # near (not exact) tie
        d = _unit(q[1]) * np.float32(0.6) + _unit(_rng("t").standard_normal(D)) * np.float32(0.8)
        for r in (3, 1500, 1501, 2100):      # a 4-way tie inside q1's top 5 (sim 0.6 each)
            v[r] = d * np.float32(4.0)
        v[42] = q[1] * np.float32(1.5)      # q1's top 1 (sim 1)
    elif name == "zero":
        for r in (5, 1234, 2169):
            v[r] = 0.0
        v[300] = q[2] * np.float32(2.0)     # a real > 0.85 match behind the NaN rows
    elif name == "threshold":
        deltas = (1e-3, -1e-3, 5e-4, -5e-4, 5e-5, -5e-5)
        g = _rng("perp")
        for i, dl in enumerate(deltas):
            u = _unit(q[i])
            p = g.standard_normal(D).astype(np.float64)
            p -= p.dot(u) * u
            p /= np.linalg.norm(p)
            c = 0.85 + dl
            v[100 + 300 * i] = ((c * u + np.sqrt(1 - c * c) * p) * 2.0).astype(np.float32)
    else:
        raise KeyError(name)
    return v, q


CASES = ("fp16", "ties", "zero", "threshold")
