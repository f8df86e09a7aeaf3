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


def test_resize_tap_budget_host_only():
    """mmf_resize_supported (host arithmetic only, no device): Pillow's tap count per output pixel,
    ks = 2 * ceil(support) + 1 with support = filter_support * scale, must fit kResizeKMax = 96 in
    both geometries -- bicubic CLIP (support 2) on the shortest side, bilinear EfficientNet squash
    (support 1) on each side."""
    import mmf_amd.hip as hip
    lib = hip.load()
    assert lib.mmf_resize_supported(224, 224) == 1
    assert lib.mmf_resize_supported(640, 480) == 1
    assert lib.mmf_resize_supported(5264, 5264) == 1   # scale 23.5 -> support 47 -> 95 taps
    assert lib.mmf_resize_supported(5265, 5265) == 0   # 97 taps
    assert lib.mmf_resize_supported(8000, 6000) == 0   # a 48 MP photo: host Pillow for that image
    assert lib.mmf_resize_supported(10528, 200) == 1   # squash: scale 47 -> 95 taps
    assert lib.mmf_resize_supported(10529, 200) == 0
    assert lib.mmf_resize_supported(0, 10) == 0


def test_header_options_match_library():
    """include/mmf_hip.h lists exactly the library's run-time options
    (mmf_option_name enumerates kOptNames), and every listed name round-trips through the process
    defaults (mmf_get_option / mmf_set_option with a NULL handle: no device call)."""
    import re
    import mmf_amd.hip as hip
    text = open(HEADER).read()
    block = text[text.index("/* Run-time options."):text.index("const char* mmf_option_name(int i);")]
    listed = re.findall(r'^ \*   "(\w+)"\s+(-?\d+):', block, flags=re.M)
    assert listed, "no option list in the header"
    lib = hip.load()
    names = []
    while True:
        n = lib.mmf_option_name(len(names))
        if n is None:
            break
        names.append(n.decode())
    assert sorted(n for n, _ in listed) == sorted(names)
    for name, default in listed:
        v = hip.get_process_option(name)
        env = "MMF_" + name.upper()
        if env not in os.environ:
            assert v == int(default), (name, v, default)
        hip.set_process_option(name, v)  # round trip
        assert hip.get_process_option(name) == v
    with pytest.raises(hip.MMFError):
        hip.get_process_option("gemm_prio")  # removed in round 5: rejected
