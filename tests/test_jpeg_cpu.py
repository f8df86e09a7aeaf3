"""Pins oracle/jpeg_decode.py (the restatement of Pillow's libjpeg-turbo baseline decode) to Pillow
itself, bit for bit, and checks the product's host entropy decoder (csrc/jpeg_host.cpp, host code of
libmmf_hip.so: no GPU needed) against the restatement's coefficients -- and through the
restatement's reconstruction, against Pillow's pixels."""
import ctypes

import numpy as np
import pytest

from oracle import jpeg_decode as J
from tests import jpeg_cases as C

pytest.importorskip("PIL.Image")


def lib():
    from mmf_amd import hip
    try:
        return hip.load()
    except hip.MMFError as e:
        pytest.skip(f"libmmf_hip.so not built: {e}")


def c_decode(L, d):
    info = np.zeros(16, np.int32)
    rc = L.mmf_jpeg_header(d, len(d), info.ctypes.data)
    if rc:
        return rc, info, None, None
    co = np.full((int(info[11]), 64), 0x5A5A, np.int16)  # garbage: the decoder must zero every block
    qt = np.zeros((3, 64), np.uint16)
    rc = L.mmf_jpeg_entropy(d, len(d), co.ctypes.data, qt.ctypes.data)
    return rc, info, co, qt


CASES = C.supported_jpegs()


@pytest.mark.parametrize("name,data", CASES, ids=[n for n, _ in CASES])
def test_restatement_matches_pillow(name, data):
    np.testing.assert_array_equal(J.decode(data), C.pillow_rgb(data))


@pytest.mark.parametrize("name,data", CASES, ids=[n for n, _ in CASES])
def test_host_entropy_decoder_matches_restatement(name, data):
    rc, info, co, qt = c_decode(lib(), data)
    assert rc == 0
    inf = J.parse(data)
    ref = J.entropy_decode(data, inf)
    hmax, vmax, mcux, mcuy = J.geometry(inf)
    assert list(info[:5]) == [inf.width, inf.height, len(inf.comps), hmax, vmax]
    off = 0
    planes = []
    for c, (cid, h, v, tq) in enumerate(inf.comps):
        bw, bh = int(info[5 + 2 * c]), int(info[6 + 2 * c])
        assert (bw, bh) == (mcux * h, mcuy * v)
        got = co[off:off + bw * bh].reshape(bh, bw, 64)
        np.testing.assert_array_equal(got, ref[c])
        np.testing.assert_array_equal(qt[c], inf.qt[tq])
        planes.append(got)
        off += bw * bh
    assert off == info[11]
    # the C coefficients through the restatement's IDCT / upsampling / colour: Pillow's pixels
    J_entropy = J.entropy_decode
    try:
        J.entropy_decode = lambda d, i: planes
        np.testing.assert_array_equal(J.decode(data), C.pillow_rgb(data))
    finally:
        J.entropy_decode = J_entropy


@pytest.mark.parametrize("name,data", C.unsupported_files(), ids=[n for n, _ in C.unsupported_files()])
def test_unsupported_files_are_declined(name, data):
    L = lib()
    info = np.zeros(16, np.int32)
    rc = L.mmf_jpeg_header(data, len(data), info.ctypes.data)
    assert rc == (-22 if name == "png" else -95)
    with pytest.raises((NotImplementedError, ValueError)):
        J.decode(data)


def test_truncated_and_corrupt_streams_do_not_crash():
    """Truncated scans decode with zeros past the end (as libjpeg: a warning, not an error); a
    damaged header is rejected."""
    L = lib()
    d = CASES[1][1]
    info = np.zeros(16, np.int32)
    assert L.mmf_jpeg_header(d[:40], 40, info.ctypes.data) != 0
    t = d[:len(d) * 2 // 3]
    rc, info, co, _ = c_decode(L, t)
    assert rc == 0 and co is not None
    rng = np.random.default_rng(3)
    for _ in range(20):
        bad = bytearray(d)
        i = int(rng.integers(len(bad) // 2, len(bad) - 2))
        bad[i] ^= 0x5C
        c_decode(L, bytes(bad))  # any rc; must not crash or write out of bounds
