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


def unpack(packed, block_off, blocks):
    """The packed records (mmf_jpeg_entropy_packed) back to dense natural-order blocks."""
    out = np.zeros((blocks, 64), np.int16)
    zz = J.ZIGZAG
    for b in range(blocks):
        o = int(block_off[b])
        assert o % 8 == 0
        mask = int(packed[o:o + 8].view(np.uint64)[0])
        ks = [k for k in range(64) if mask >> k & 1]
        vals = packed[o + 8:o + 8 + 2 * len(ks)].view(np.int16)
        assert np.all(vals != 0)
        for k, v in zip(ks, vals):
            out[b, zz[k]] = v
    return out


@pytest.mark.parametrize("name,data", CASES, ids=[n for n, _ in CASES])
def test_packed_records_equal_dense_coefficients(name, data):
    """The H2D format (sparse records) carries exactly the dense decoder's coefficients and tables;
    a too-small output buffer is refused, not overrun."""
    L = lib()
    rc, info, co, qt = c_decode(L, data)
    assert rc == 0
    blocks = int(info[11])
    bound = int(L.mmf_jpeg_packed_bound(blocks))
    packed = np.zeros(bound, np.uint8)
    boff = np.full(blocks, 0xFFFFFFFF, np.uint32)
    qt2 = np.zeros((3, 64), np.uint16)
    used = ctypes.c_int64(-1)
    assert L.mmf_jpeg_entropy_packed(data, len(data), packed.ctypes.data, bound, boff.ctypes.data, qt2.ctypes.data,
                                     ctypes.byref(used)) == 0
    assert 8 <= used.value <= bound and used.value % 8 == 0
    assert np.all(boff < used.value)
    np.testing.assert_array_equal(unpack(packed, boff, blocks), co)
    np.testing.assert_array_equal(qt2, qt)
    if used.value > 16:
        assert L.mmf_jpeg_entropy_packed(data, len(data), packed.ctypes.data, used.value - 8, boff.ctypes.data,
                                         qt2.ctypes.data, ctypes.byref(used)) == -34


@pytest.mark.parametrize("name,prog,seq", C.progressive_pairs(), ids=[n for n, _, _ in C.progressive_pairs()])
def test_progressive_coefficients_equal_sequential(name, prog, seq):
    """Progressive (SOF2) decoding -- every scan of Pillow's successive-approximation script, DHT
    between scans, restarts -- yields exactly the coefficients of the sequential file of the same
    pixels (pinned above to the restatement and Pillow); the packed records carry them too."""
    L = lib()
    rc_p, info_p, co_p, qt_p = c_decode(L, prog)
    rc_s, info_s, co_s, qt_s = c_decode(L, seq)
    assert rc_p == 0 and rc_s == 0
    np.testing.assert_array_equal(info_p, info_s)
    np.testing.assert_array_equal(qt_p, qt_s)
    np.testing.assert_array_equal(co_p, co_s)
    blocks = int(info_p[11])
    packed = np.zeros(int(L.mmf_jpeg_packed_bound(blocks)), np.uint8)
    boff = np.zeros(blocks, np.uint32)
    qt2 = np.zeros((3, 64), np.uint16)
    used = ctypes.c_int64(0)
    assert L.mmf_jpeg_entropy_packed(prog, len(prog), packed.ctypes.data, packed.size, boff.ctypes.data,
                                     qt2.ctypes.data, ctypes.byref(used)) == 0
    np.testing.assert_array_equal(unpack(packed, boff, blocks), co_s)


def test_stage_packed_reserves_and_refuses_overflow():
    """mmf_jpeg_stage_packed (the staging call of mmf_amd/jpeg.py): records at the reserved offsets equal
    mmf_jpeg_entropy_packed's; an image that does not fit keeps its reservation and reports ERANGE."""
    L = lib()
    imgs = [d for _, d in CASES[:4]]
    infos = [c_decode(L, d)[1] for d in imgs]
    dst = np.zeros(1 << 20, np.uint8)
    cursor = np.zeros(1, np.int64)
    off = np.zeros(len(imgs), np.int64)
    for k, d in enumerate(imgs):
        blocks = int(infos[k][11])
        boff = np.zeros(blocks, np.uint32)
        qt = np.zeros((3, 64), np.uint16)
        assert L.mmf_jpeg_stage_packed(d, len(d), dst.ctypes.data, dst.size, cursor.ctypes.data, boff.ctypes.data,
                                       qt.ctypes.data, off[k:].ctypes.data) == 0
        ref = np.zeros(int(L.mmf_jpeg_packed_bound(blocks)), np.uint8)
        used = ctypes.c_int64(0)
        boff2 = np.zeros(blocks, np.uint32)
        assert L.mmf_jpeg_entropy_packed(d, len(d), ref.ctypes.data, ref.size, boff2.ctypes.data, qt.ctypes.data,
                                         ctypes.byref(used)) == 0
        assert off[k] % 8 == 0 and (k == 0 or off[k] >= off[k - 1])
        np.testing.assert_array_equal(dst[off[k]:off[k] + used.value], ref[:used.value])
        np.testing.assert_array_equal(boff, boff2)
    before = int(cursor[0])
    small = np.zeros(before + 8, np.uint8)
    d = imgs[0]
    boff = np.zeros(int(infos[0][11]), np.uint32)
    qt = np.zeros((3, 64), np.uint16)
    o = np.zeros(1, np.int64)
    assert L.mmf_jpeg_stage_packed(d, len(d), small.ctypes.data, small.size, cursor.ctypes.data, boff.ctypes.data,
                                   qt.ctypes.data, o.ctypes.data) == -34
    assert o[0] == before and cursor[0] > before and not small[before:].any()


@pytest.mark.parametrize("name,data", C.unsupported_files(), ids=[n for n, _ in C.unsupported_files()])
def test_unsupported_files_are_declined(name, data):
    L = lib()
    info = np.zeros(16, np.int32)
    rc = L.mmf_jpeg_header(data, len(data), info.ctypes.data)
    assert rc == (-22 if name == "png" else -95)
    with pytest.raises((NotImplementedError, ValueError)):
        J.decode(data)
    if name == "cmyk":  # files Pillow opens; the relabelled lossless one is not a real file
        assert C.pillow_rgb(data).shape == (40, 48, 3)


def test_truncated_and_corrupt_streams_do_not_crash():
    """A file whose data ends before its EOI marker is declined (Pillow then raises "image file is
    truncated", as the reference's Image.open(...).convert does); a scan cut short but followed by an
    EOI decodes with zeros past the cut (libjpeg: a warning, not an error); a damaged header is
    rejected."""
    L = lib()
    d = CASES[1][1]
    info = np.zeros(16, np.int32)
    assert L.mmf_jpeg_header(d[:40], 40, info.ctypes.data) != 0
    t = d[:len(d) * 2 // 3]
    for cut in (t, d[:-2], d[:-1]):
        assert L.mmf_jpeg_header(cut, len(cut), info.ctypes.data) == -95
        with pytest.raises(OSError, match="truncated"):
            C.pillow_rgb(cut)
    rc, info, co, _ = c_decode(L, t + b"\xff\xd9")
    assert rc == 0 and co is not None
    rng = np.random.default_rng(3)
    for _ in range(20):
        bad = bytearray(d)
        i = int(rng.integers(len(bad) // 2, len(bad) - 2))
        bad[i] ^= 0x5C
        c_decode(L, bytes(bad))  # any rc; must not crash or write out of bounds


def test_header_batch_equals_per_file():
    L = lib()
    files = [d for _, d in CASES] + [d for _, d in C.unsupported_files()] + [None, b"", b"\xff\xd8"]
    n = len(files)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = np.array([len(d) if d is not None else 0 for d in files], np.int64)
    infos = np.full((n, 16), -7, np.int32)
    rcs = np.full(n, 7, np.int32)
    assert L.mmf_jpeg_header_batch(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, infos.ctypes.data,
                                   rcs.ctypes.data, 3) == 0
    for k, d in enumerate(files):
        if d is None:
            assert rcs[k] == -22
            continue
        info = np.zeros(16, np.int32)
        assert rcs[k] == L.mmf_jpeg_header(d, len(d), info.ctypes.data)
        np.testing.assert_array_equal(infos[k], info)


def test_stage_packed_batch_equals_per_file_records():
    """mmf_jpeg_stage_packed_batch (jpeg.py's chunk call, the library's own threads): every file's
    records, block offsets and tables equal mmf_jpeg_entropy_packed's, at its reserved offset; a
    file past the capacity reports ERANGE."""
    L = lib()
    files = [d for _, d in CASES] + [p for _, p, _ in C.progressive_pairs()]
    infos = [c_decode(L, d)[1] for d in files]
    blocks = np.array([int(i[11]) for i in infos], np.int64)
    base = np.r_[0, np.cumsum(blocks)[:-1]].astype(np.int64)
    n = len(files)
    dst = np.zeros(1 << 22, np.uint8)
    cursor = np.zeros(1, np.int64)
    boff = np.zeros(int(blocks.sum()), np.uint32)
    qt = np.zeros((n, 3, 64), np.uint16)
    rec = np.zeros(n, np.int64)
    rcs = np.full(n, 7, np.int32)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = np.array([len(d) for d in files], np.int64)
    assert L.mmf_jpeg_stage_packed_batch(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, dst.ctypes.data,
                                         dst.size, cursor.ctypes.data, boff.ctypes.data, base.ctypes.data,
                                         qt.ctypes.data, rec.ctypes.data, 4, rcs.ctypes.data) == 0
    assert not rcs.any()
    for k, d in enumerate(files):
        ref = np.zeros(int(L.mmf_jpeg_packed_bound(int(blocks[k]))), np.uint8)
        b2 = np.zeros(int(blocks[k]), np.uint32)
        q2 = np.zeros((3, 64), np.uint16)
        used = ctypes.c_int64(0)
        assert L.mmf_jpeg_entropy_packed(d, len(d), ref.ctypes.data, ref.size, b2.ctypes.data, q2.ctypes.data,
                                         ctypes.byref(used)) == 0
        np.testing.assert_array_equal(dst[rec[k]:rec[k] + used.value], ref[:used.value])
        np.testing.assert_array_equal(boff[base[k]:base[k] + blocks[k]], b2)
        np.testing.assert_array_equal(qt[k], q2)
    cursor[0] = 0
    small = 4096
    assert L.mmf_jpeg_stage_packed_batch(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, dst.ctypes.data,
                                         small, cursor.ctypes.data, boff.ctypes.data, base.ctypes.data,
                                         qt.ctypes.data, rec.ctypes.data, 4, rcs.ctypes.data) == 0
    assert set(rcs.tolist()) <= {0, -34} and (rcs == -34).any()


@pytest.mark.parametrize("which", ["sequential", "progressive"])
def test_packed_staging_of_truncated_and_corrupt_streams(which):
    """The product's staging call on damaged scans: records stay inside the bound, every block offset
    points inside the written records (8-aligned), and the guard bytes after them are untouched."""
    L = lib()
    # 300x200 with restart markers
    d = CASES[9][1] if which == "sequential" else [p for n, p, _ in C.progressive_pairs() if "300x200" in n][0]
    info = np.zeros(16, np.int32)
    assert L.mmf_jpeg_header(d, len(d), info.ctypes.data) == 0
    blocks = int(info[11])
    bound = int(L.mmf_jpeg_packed_bound(blocks))
    rng = np.random.default_rng(7)
    variants = [d[:len(d) * 2 // 3] + b"\xff\xd9", d[:len(d) // 3] + b"\xff\xd9"]
    for _ in range(30):
        bad = bytearray(d)
        for _ in range(3):
            i = int(rng.integers(len(bad) // 3, len(bad) - 2))
            bad[i] ^= int(rng.integers(1, 256))
        variants.append(bytes(bad))
    for v in variants:
        dst = np.full(bound + 64, 0xA5, np.uint8)
        cursor = np.zeros(1, np.int64)
        boff = np.full(blocks, 0xFFFFFFFF, np.uint32)
        qt = np.zeros((3, 64), np.uint16)
        off = np.zeros(1, np.int64)
        rc = L.mmf_jpeg_stage_packed(v, len(v), dst.ctypes.data, bound, cursor.ctypes.data, boff.ctypes.data,
                                     qt.ctypes.data, off.ctypes.data)
        if rc != 0:
            continue  # a header the damage made unparseable: declined, nothing written
        used = int(cursor[0])
        assert 8 <= used <= bound and off[0] == 0
        assert np.all(boff % 8 == 0) and np.all(boff < used)
        assert np.all(dst[bound:] == 0xA5)
        for o in boff[::37]:  # each record's mask counts values that fit before the next offset bound
            n = bin(int(dst[o:o + 8].view(np.uint64)[0])).count("1")
            assert o + 8 + 2 * n <= used


def test_malformed_scan_headers_are_rejected():
    """repeated SOS component ids (their Huffman table slots would stay unset) and an SOS
    segment shorter than its component list are EINVAL, with no read past the buffer."""
    L = lib()
    info = np.zeros(16, np.int32)
    d = C.duplicate_sos_ids()
    assert L.mmf_jpeg_header(d, len(d), info.ctypes.data) == -22
    d = C.short_sos_at_eof()
    buf = ctypes.create_string_buffer(d, len(d))  # exact-size copy
    assert L.mmf_jpeg_header(buf, len(d), info.ctypes.data) == -22


def test_rgb_component_ids_go_to_pillow():
    """No JFIF / Adobe marker and ids 'R' 'G' 'B': libjpeg decodes without the YCbCr transform, so the
    device path (which always converts) declines the file and Pillow decodes it."""
    L = lib()
    d = C.rgb_component_ids()
    info = np.zeros(16, np.int32)
    assert L.mmf_jpeg_header(d, len(d), info.ctypes.data) == -95
    px = C.pillow_rgb(d)
    assert px.shape == (32, 40, 3)
    # the same bytes with ids 1 2 3 are YCbCr to libjpeg: different pixels, so the distinction matters
    e = bytearray(d)
    for m, a, b in C._segments(d):
        if m in (0xC0, 0xDA):
            for k in range(3):
                e[a + (10 + 3 * k if m == 0xC0 else 5 + 2 * k)] = k + 1
    assert L.mmf_jpeg_header(bytes(e), len(e), info.ctypes.data) == 0
    assert not np.array_equal(C.pillow_rgb(bytes(e)), px)
