"""Test infrastructure only (never imported by the product path): a numpy restatement of the baseline
JPEG decode behind the reference's image loading -- `Image.open(path).convert("RGB")`
(misinfo_forensics.py:255-258, forensics_dashboard.py:180-185) decodes through Pillow's bundled
libjpeg-turbo (Pillow 12.2, libjpeg API 6.2) with its defaults: islow integer IDCT, fancy
(triangle-filter) chroma upsampling, table-driven YCbCr -> RGB.  Restated from the IJG/libjpeg-turbo
algorithms:
  * entropy decoding (jdhuff.c): baseline Huffman, DC prediction per component, restart intervals;
  * jidctint.c jpeg_idct_islow: CONST_BITS 13, PASS1_BITS 2, columns then rows, DESCALE rounding,
    the 1024-entry post-IDCT range-limit table (jdmaster.c prepare_range_limit_table);
  * jdsample.c h2v1 / h1v2 / h2v2 fancy upsampling (context rows replicated at the top and bottom
    edges, jdmainct.c make_funny_pointers / set_bottom_pointers);
  * jdcolor.c ycc_rgb_convert with build_ycc_rgb_table (SCALEBITS 16).
Pinned against Pillow itself in this container (tests/test_jpeg_cpu.py: bit-exact pixels on every
case); the host entropy decoder (csrc/jpeg_host.cpp) and the device reconstruction (csrc/jpeg.hip)
are checked against this restatement and against Pillow.

Supported: 8-bit baseline sequential (SOF0/SOF1) Huffman JPEGs with 1 component or 3 YCbCr
components sampled 4:4:4, 4:2:2, 4:2:0 or 4:4:0.  Everything else raises NotImplementedError
(the product falls back to Pillow for those files).
"""
import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21,
    28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61,
    54, 47, 55, 62, 63], np.int64)  # zigzag index -> natural index


class JpegInfo:
    def __init__(self):
        self.width = self.height = 0
        self.comps = []        # [(id, h, v, tq)]
        self.qt = {}           # tq -> uint16[64] natural order
        self.dc, self.ac = {}, {}  # table id -> (maxcode, valptr, mincode, huffval)
        self.restart = 0
        self.adobe = None      # Adobe APP14 transform flag
        self.jfif = False


def _build_huff(bits, vals):
    """jdhuff.c jpeg_make_d_derived_tbl: canonical codes by length."""
    codes = {}
    code = 0
    k = 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            codes[(length, code)] = vals[k]
            k += 1
            code += 1
        code <<= 1
    return codes


def parse(data: bytes) -> JpegInfo:
    info = JpegInfo()
    if data[:2] != b"\xff\xd8":
        raise ValueError("not a JPEG")
    p = 2
    while p < len(data):
        if data[p] != 0xFF:
            raise ValueError("marker expected")
        m = data[p + 1]
        p += 2
        if m == 0xFF:
            p -= 1
            continue
        if m in (0xD8, 0x01) or 0xD0 <= m <= 0xD7:
            continue
        L = (data[p] << 8) | data[p + 1]
        seg = data[p + 2:p + L]
        if m in (0xC0, 0xC1):
            if seg[0] != 8:
                raise NotImplementedError("12-bit precision")
            info.height = (seg[1] << 8) | seg[2]
            info.width = (seg[3] << 8) | seg[4]
            n = seg[5]
            for i in range(n):
                cid, hv, tq = seg[6 + 3 * i], seg[7 + 3 * i], seg[8 + 3 * i]
                info.comps.append((cid, hv >> 4, hv & 15, tq))
        elif 0xC2 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            raise NotImplementedError(f"SOF{m - 0xC0} (progressive / lossless / arithmetic)")
        elif m == 0xDB:
            q = 0
            while q < len(seg):
                pq, tq = seg[q] >> 4, seg[q] & 15
                q += 1
                if pq:
                    vals = [(seg[q + 2 * i] << 8) | seg[q + 2 * i + 1] for i in range(64)]
                    q += 128
                else:
                    vals = list(seg[q:q + 64])
                    q += 64
                t = np.zeros(64, np.int64)
                t[ZIGZAG] = vals
                info.qt[tq] = t
        elif m == 0xC4:
            q = 0
            while q < len(seg):
                tc, th = seg[q] >> 4, seg[q] & 15
                bits = list(seg[q + 1:q + 17])
                n = sum(bits)
                vals = list(seg[q + 17:q + 17 + n])
                q += 17 + n
                (info.ac if tc else info.dc)[th] = _build_huff(bits, vals)
        elif m == 0xDD:
            info.restart = (seg[0] << 8) | seg[1]
        elif m == 0xEE and seg[:5] == b"Adobe":
            info.adobe = seg[11]
        elif m == 0xE0 and seg[:5] == b"JFIF\x00":
            info.jfif = True
        elif m == 0xDA:
            ns = seg[0]
            sc = [(seg[1 + 2 * i], seg[2 + 2 * i] >> 4, seg[2 + 2 * i] & 15) for i in range(ns)]
            info.scan = sc
            info.scan_data_at = p + L
            return info
        elif m == 0xD9:
            break
        p += L
    raise ValueError("no scan")


class _Bits:
    """jdhuff.c bit reader: 0xFF00 stuffing removed; a marker ends the data (zeros follow)."""

    def __init__(self, data, pos):
        self.d, self.p, self.acc, self.n = data, pos, 0, 0

    def _fill(self):
        b = 0
        if self.p < len(self.d):
            b = self.d[self.p]
            if b == 0xFF:
                nb = self.d[self.p + 1] if self.p + 1 < len(self.d) else 0
                if nb == 0:
                    self.p += 2
                else:
                    b = 0  # marker: feed zeros, do not advance
            else:
                self.p += 1
        self.acc = (self.acc << 8) | b
        self.n += 8

    def bit(self):
        if self.n == 0:
            self._fill()
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, k):
        v = 0
        for _ in range(k):
            v = (v << 1) | self.bit()
        return v

    def restart(self):
        """Discard the partial byte, skip the RSTn marker."""
        self.acc = self.n = 0
        while self.p + 1 < len(self.d) and not (self.d[self.p] == 0xFF and 0xD0 <= self.d[self.p + 1] <= 0xD7):
            self.p += 1
        self.p += 2


def _decode_sym(br, codes):
    code = 0
    for length in range(1, 17):
        code = (code << 1) | br.bit()
        v = codes.get((length, code))
        if v is not None:
            return v
    return 0  # corrupt data: libjpeg warns and returns 0


def _extend(v, t):
    return v - (1 << t) + 1 if t and v < (1 << (t - 1)) else v


def geometry(info):
    hmax = max(c[1] for c in info.comps)
    vmax = max(c[2] for c in info.comps)
    mcux = -(-info.width // (8 * hmax))
    mcuy = -(-info.height // (8 * vmax))
    return hmax, vmax, mcux, mcuy


def entropy_decode(data: bytes, info: JpegInfo):
    """-> list per component of int16 [by, bx, 64] natural-order quantised coefficients; the block
    grid is the MCU-padded one (mcuy * v_c, mcux * h_c); single-component scans cover only the
    blocks of the component's own extent (ceil(comp size / 8)), as jdhuff.c does."""
    hmax, vmax, mcux, mcuy = geometry(info)
    comps = {c[0]: i for i, c in enumerate(info.comps)}
    out = [np.zeros((mcuy * c[2], mcux * c[1], 64), np.int64) for c in info.comps]
    sc = info.scan
    if len(sc) != len(info.comps):
        raise NotImplementedError("multi-scan sequential JPEG")
    br = _Bits(data, info.scan_data_at)
    pred = [0] * len(info.comps)
    ri = info.restart
    if len(sc) == 1:
        ci = comps[sc[0][0]]
        c = info.comps[ci]
        cw = -(-info.width * c[1] // hmax)
        ch = -(-info.height * c[2] // vmax)
        units = [(ci, by, bx) for by in range(-(-ch // 8)) for bx in range(-(-cw // 8))]
        groups = [[u] for u in units]
    else:
        groups = []
        for my in range(mcuy):
            for mx in range(mcux):
                g = []
                for cid, td, ta in sc:
                    ci = comps[cid]
                    _, h, v, _ = info.comps[ci]
                    for yy in range(v):
                        for xx in range(h):
                            g.append((ci, my * v + yy, mx * h + xx))
                groups.append(g)
    tables = {comps[cid]: (td, ta) for cid, td, ta in sc}
    for n, g in enumerate(groups):
        if ri and n and n % ri == 0:
            br.restart()
            pred = [0] * len(info.comps)
        for ci, by, bx in g:
            td, ta = tables[ci]
            blk = np.zeros(64, np.int64)
            t = _decode_sym(br, info.dc[td])
            diff = _extend(br.bits(t), t) if t else 0
            pred[ci] += diff
            blk[0] = pred[ci]
            k = 1
            while k < 64:
                rs = _decode_sym(br, info.ac[ta])
                r, s = rs >> 4, rs & 15
                if s:
                    k += r
                    if k > 63:
                        break
                    blk[ZIGZAG[k]] = _extend(br.bits(s), s)
                    k += 1
                else:
                    if r != 15:
                        break
                    k += 16
            out[ci][by, bx] = blk
    return [o.astype(np.int16) for o in out]


# ---- jidctint.c jpeg_idct_islow ----
CONST_BITS, PASS1_BITS = 13, 2
F = dict(f0_298631336=2446, f0_390180644=3196, f0_541196100=4433, f0_765366865=6270, f0_899976223=7373,
         f1_175875602=9633, f1_501321110=12299, f1_847759065=15137, f1_961570560=16069, f2_053119869=16819,
         f2_562915447=20995, f3_072711026=25172)


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _idct_1d(d0, d1, d2, d3, d4, d5, d6, d7, shift, pass2):
    z2, z3 = d2, d6
    z1 = (z2 + z3) * F["f0_541196100"]
    tmp2 = z1 + z3 * (-F["f1_847759065"])
    tmp3 = z1 + z2 * F["f0_765366865"]
    tmp0 = (d0 + d4) << CONST_BITS
    tmp1 = (d0 - d4) << CONST_BITS
    tmp10, tmp13 = tmp0 + tmp3, tmp0 - tmp3
    tmp11, tmp12 = tmp1 + tmp2, tmp1 - tmp2
    t0, t1, t2, t3 = d7, d5, d3, d1
    z1, z2, z3, z4 = t0 + t3, t1 + t2, t0 + t2, t1 + t3
    z5 = (z3 + z4) * F["f1_175875602"]
    t0 = t0 * F["f0_298631336"]
    t1 = t1 * F["f2_053119869"]
    t2 = t2 * F["f3_072711026"]
    t3 = t3 * F["f1_501321110"]
    z1 = z1 * (-F["f0_899976223"])
    z2 = z2 * (-F["f2_562915447"])
    z3 = z3 * (-F["f1_961570560"]) + z5
    z4 = z4 * (-F["f0_390180644"]) + z5
    t0 += z1 + z3
    t1 += z2 + z4
    t2 += z2 + z3
    t3 += z1 + z4
    return [_descale(v, shift) for v in (tmp10 + t3, tmp11 + t2, tmp12 + t1, tmp13 + t0,
                                         tmp13 - t0, tmp12 - t1, tmp11 - t2, tmp10 - t3)]


def _range_limit(v):
    """post-IDCT range limit: table[(v) & 1023] with CENTERJSAMPLE folded in."""
    m = v & 1023
    return np.where(m < 128, m + 128, np.where(m < 512, 255, np.where(m < 896, 0, m - 896)))


def idct_islow(coef, qt):
    """coef int [..., 64] natural order, qt [64] -> uint8 [..., 8, 8] samples.  (The zero-AC
    shortcuts of jidctint.c give the same values as the full computation.)"""
    c = coef.astype(np.int64) * qt.astype(np.int64)
    c = c.reshape(coef.shape[:-1] + (8, 8))  # [row (v), col (u)]
    cols = _idct_1d(*[c[..., r, :] for r in range(8)], CONST_BITS - PASS1_BITS, False)  # per column
    ws = np.stack(cols, axis=-2)  # [..., row, col]
    rows = _idct_1d(*[ws[..., :, k] for k in range(8)], CONST_BITS + PASS1_BITS + 3, True)
    out = np.stack(rows, axis=-1)
    return _range_limit(out).astype(np.uint8)


def component_planes(coefs, info):
    """IDCT every block -> uint8 plane [bh*8, bw*8] per component."""
    planes = []
    for (cid, h, v, tq), cf in zip(info.comps, coefs):
        b = idct_islow(cf, info.qt[tq])  # [by, bx, 8, 8]
        by, bx = b.shape[:2]
        planes.append(b.transpose(0, 2, 1, 3).reshape(by * 8, bx * 8))
    return planes


def _fancy(plane, dw, dh, fh, fv):
    """jdsample.c fancy upsampling of the real dw x dh samples by (fh, fv) in {1,2}^2."""
    x = plane[:dh, :dw].astype(np.int64)
    if fv == 2:
        up = np.concatenate([x[:1], x[:-1]], 0)
        dn = np.concatenate([x[1:], x[-1:]], 0)
        if fh == 2:
            cs0, cs1 = 3 * x + up, 3 * x + dn  # column sums for output rows 2i, 2i+1
            res = []
            for cs in (cs0, cs1):
                lf = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
                rt = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
                e = (3 * cs + lf + 8) >> 4
                o = (3 * cs + rt + 7) >> 4
                res.append(np.stack([e, o], -1).reshape(dh, 2 * dw))
            return np.stack(res, 1).reshape(2 * dh, 2 * dw)
        r0, r1 = (3 * x + up + 1) >> 2, (3 * x + dn + 2) >> 2
        return np.stack([r0, r1], 1).reshape(2 * dh, dw)
    if fh == 2:
        lf = np.concatenate([x[:, :1], x[:, :-1]], 1)
        rt = np.concatenate([x[:, 1:], x[:, -1:]], 1)
        e = (3 * x + lf + 1) >> 2
        o = (3 * x + rt + 2) >> 2
        return np.stack([e, o], -1).reshape(dh, 2 * dw)
    return x


def _ycc_tables():
    x = np.arange(256, dtype=np.int64) - 128
    fix = lambda f: int(f * 65536 + 0.5)  # noqa: E731
    half = 1 << 15
    cr_r = (fix(1.40200) * x + half) >> 16
    cb_b = (fix(1.77200) * x + half) >> 16
    cr_g = -fix(0.71414) * x
    cb_g = -fix(0.34414) * x + half
    return cr_r, cb_b, cr_g, cb_g


def decode(data: bytes) -> np.ndarray:
    """-> uint8 [H, W, 3], equal to np.asarray(Image.open(...).convert("RGB"))."""
    info = parse(data)
    n = len(info.comps)
    if n not in (1, 3):
        raise NotImplementedError(f"{n} components")
    if n == 3 and info.adobe is not None and info.adobe == 0:
        raise NotImplementedError("Adobe RGB (untransformed) JPEG")
    hmax, vmax, _, _ = geometry(info)
    coefs = entropy_decode(data, info)
    planes = component_planes(coefs, info)
    W, H = info.width, info.height
    if n == 1:
        g = planes[0][:H, :W]
        return np.stack([g, g, g], -1)
    up = []
    for (cid, h, v, tq), pl in zip(info.comps, planes):
        fh, fv = hmax // h, vmax // v
        if (fh, fv) not in ((1, 1), (2, 1), (1, 2), (2, 2)) or hmax * 1 > 2 or vmax > 2:
            raise NotImplementedError(f"sampling {h}x{v} of {hmax}x{vmax}")
        dw, dh = -(-W * h // hmax), -(-H * v // vmax)
        up.append(_fancy(pl, dw, dh, fh, fv)[:H, :W])
    y, cb, cr = up
    cr_r, cb_b, cr_g, cb_g = _ycc_tables()
    r = np.clip(y + cr_r[cr], 0, 255)
    g = np.clip(y + ((cb_g[cb] + cr_g[cr]) >> 16), 0, 255)
    b = np.clip(y + cb_b[cb], 0, 255)
    return np.stack([r, g, b], -1).astype(np.uint8)
