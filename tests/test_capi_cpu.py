"""CPU-side checks of the C-ABI library: it loads and exports every symbol include/mmf_hip.h
declares (no compute — there is no GPU here), and the Python binding declares each of them."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mmf_hip.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    names = _declared()
    assert "mmf_analyze_batch" in names and "mmf_create" in names and len(names) >= 15


def test_library_exports_every_declared_symbol():
    import mmf_amd.hip as hip
    if not os.path.exists(hip.LIB_PATH):
        pytest.skip("libmmf_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(hip.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_declared()) == set(hip.SIGNATURES), set(_declared()) ^ set(hip.SIGNATURES)
    lib = hip.load()
    assert lib.mmf_version().decode().startswith("mmf_hip")
    assert lib.mmf_last_error() is not None


def test_missing_library_fails_loudly(tmp_path):
    import mmf_amd.hip as hip
    with pytest.raises(hip.MMFError):
        hip.load(str(tmp_path / "nope.so"))
