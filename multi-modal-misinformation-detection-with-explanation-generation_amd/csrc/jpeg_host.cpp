// Host half of the device JPEG decode: marker parsing and baseline
// Huffman entropy decoding into quantised DCT coefficient planes -- the only inherently serial part
// of a JPEG decode.  Dequantisation, the islow IDCT, fancy chroma upsampling and YCbCr -> RGB run on
// the device (jpeg.hip); the pixels equal Pillow's decoder (libjpeg-turbo: jdhuff.c, jidctint.c,
// jdsample.c, jdcolor.c), which is what the reference's Image.open(...).convert("RGB")
// (misinfo_forensics.py:255-258) runs.  Restatement and pinning: oracle/jpeg_decode.py.
//
// Supported (mmf_jpeg_header returns 0): 8-bit baseline / extended sequential Huffman (SOF0/SOF1)
// with one scan holding every component, or progressive Huffman (SOF2, any scan script; jdphuff.c), 1 component or 3 YCbCr components with luma sampling h, v <= 2
// and chroma 1x1 (4:4:4, 4:2:2, 4:2:0); anything else returns MMF_EUNSUPPORTED and the caller decodes
// that file on the host (Pillow).
//
// Coefficient layout (mmf_jpeg_entropy): component c's blocks as [bh_c][bw_c][64] int16, natural
// (row-major) order, c = 0, 1, 2 back to back; bw_c = mcux * h_c, bh_c = mcuy * v_c (the MCU-padded
// block grid; blocks outside a single-component scan's extent stay zero, as in libjpeg).
#include <cstdint>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/mmf_hip.h"

namespace {

constexpr uint8_t kZigzag[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    // run-off guard: a corrupt run that passes 63 writes into position 63's slot (ignored, as libjpeg)
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int kLook = 10;  // lookahead bits of the fast symbol / AC tables

struct Huff {
  bool present = false;
  // jdhuff.c jpeg_make_d_derived_tbl
  int32_t maxcode[18];
  int32_t valoff[17];
  uint8_t huffval[256];
  uint16_t look[1 << kLook];  // (length << 8) | symbol, 0 = longer than kLook bits
  // AC fast path (libjpeg-turbo's idea): code + value bits within the lookahead ->
  // (value << 16) | (run << 8) | total bits; 0 = take the symbol path; (1 << 15) | bits = end of block
  int32_t acfast[1 << kLook];
};

bool build_huff(Huff& t, const uint8_t* bits, const uint8_t* vals, int nvals, bool dc) {
  int code = 0, k = 0;
  if (dc)  // jdhuff.c jpeg_make_d_derived_tbl: a DC symbol is a bit count, at most 15
    for (int i = 0; i < nvals; ++i)
      if (vals[i] > 15) return false;
  uint16_t huffcode[257];
  uint8_t huffsize[257];
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < bits[l - 1]; ++i) {
      if (k >= 256) return false;
      huffsize[k++] = (uint8_t)l;
    }
  if (k != nvals) return false;
  huffsize[k] = 0;
  int si = huffsize[0];
  k = 0;
  while (huffsize[k]) {
    while (huffsize[k] == si) huffcode[k++] = (uint16_t)code++;
    if (code >= (1 << si)) return false;  // bad table
    code <<= 1;
    ++si;
  }
  int p = 0;
  for (int l = 1; l <= 16; ++l) {
    if (bits[l - 1]) {
      t.valoff[l] = p - huffcode[p];
      p += bits[l - 1];
      t.maxcode[l] = huffcode[p - 1];
    } else {
      t.maxcode[l] = -1;
    }
  }
  t.maxcode[17] = 0x7fffffff;
  memcpy(t.huffval, vals, nvals);
  memset(t.look, 0, sizeof(t.look));
  p = 0;
  for (int l = 1; l <= kLook; ++l)
    for (int i = 0; i < bits[l - 1]; ++i, ++p) {
      const int lookbits = huffcode[p] << (kLook - l);
      for (int c = 0; c < (1 << (kLook - l)); ++c) t.look[lookbits + c] = (uint16_t)((l << 8) | vals[p]);
    }
  for (int lk = 0; lk < (1 << kLook); ++lk) {
    t.acfast[lk] = 0;
    const int e = t.look[lk];
    if (!e) continue;
    const int l = e >> 8, rs = e & 0xFF, r = rs >> 4, sz = rs & 15;
    if (rs == 0) {  // end of block: flagged so the packed decoder ends the block without decode_sym
      t.acfast[lk] = (1 << 15) | l;
      continue;
    }
    if (!sz || l + sz > kLook) continue;
    int v = (lk >> (kLook - l - sz)) & ((1 << sz) - 1);
    if (v < (1 << (sz - 1))) v -= (1 << sz) - 1;
    t.acfast[lk] = (int32_t)((uint32_t)v << 16) | (r << 8) | (l + sz);
  }
  t.present = true;
  return true;
}

struct Comp {
  int id = 0, h = 0, v = 0, tq = 0, td = 0, ta = 0;
};

struct Jpeg {
  int width = 0, height = 0, ncomp = 0, restart = 0, adobe = -1;
  bool jfif = false;
  Comp comp[4];
  int nscan = 0, scomp[4] = {0, 0, 0, 0};
  uint16_t qt[4][64];
  bool qt_present[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  const uint8_t* scan = nullptr;  // entropy-coded segment start (progressive: the first SOS marker)
  const uint8_t* end = nullptr;
  bool progressive = false;
  int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
};

// marker walk up to the first SOS; 0 = supported, else MMF_EUNSUPPORTED / MMF_EINVAL
int parse(const uint8_t* d, int64_t n, Jpeg& j) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return MMF_EINVAL;
  int64_t p = 2;
  bool sof = false;
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return MMF_EINVAL;
    const int m = d[p + 1];
    if (m == 0xFF) { ++p; continue; }
    p += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) return MMF_EINVAL;
    const int L = (d[p] << 8) | d[p + 1];
    if (L < 2 || p + L > n) return MMF_EINVAL;
    const uint8_t* s = d + p + 2;
    const int sl = L - 2;
    if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
      if (sl < 6 || s[0] != 8) return MMF_EUNSUPPORTED;  // 12-bit
      j.progressive = m == 0xC2;
      j.height = (s[1] << 8) | s[2];
      j.width = (s[3] << 8) | s[4];
      j.ncomp = s[5];
      if (j.ncomp != 1 && j.ncomp != 3) return MMF_EUNSUPPORTED;
      if (sl < 6 + 3 * j.ncomp || j.width <= 0 || j.height <= 0) return MMF_EINVAL;
      // Pillow refuses images past 2 x MAX_IMAGE_PIXELS (178,956,970 px) as decompression bombs; the
      // staging buffers are sized from this header, so larger claims are declined here too
      if ((int64_t)j.width * j.height > 178956970) return MMF_EUNSUPPORTED;
      for (int i = 0; i < j.ncomp; ++i) {
        j.comp[i].id = s[6 + 3 * i];
        j.comp[i].h = s[7 + 3 * i] >> 4;
        j.comp[i].v = s[7 + 3 * i] & 15;
        j.comp[i].tq = s[8 + 3 * i] & 3;
        if (j.comp[i].h < 1 || j.comp[i].v < 1) return MMF_EINVAL;
      }
      sof = true;
    } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return MMF_EUNSUPPORTED;  // lossless, arithmetic, hierarchical
    } else if (m == 0xDB) {
      int q = 0;
      while (q < sl) {
        const int pq = s[q] >> 4, tq = s[q] & 3;
        ++q;
        if (q + (pq ? 128 : 64) > sl) return MMF_EINVAL;
        for (int i = 0; i < 64; ++i) {
          const int v = pq ? ((s[q + 2 * i] << 8) | s[q + 2 * i + 1]) : s[q + i];
          j.qt[tq][kZigzag[i]] = (uint16_t)v;
        }
        q += pq ? 128 : 64;
        j.qt_present[tq] = true;
      }
    } else if (m == 0xC4) {
      int q = 0;
      while (q < sl) {
        if (q + 17 > sl) return MMF_EINVAL;
        const int tc = s[q] >> 4, th = s[q] & 3;
        int nv = 0;
        for (int i = 0; i < 16; ++i) nv += s[q + 1 + i];
        if (nv > 256 || q + 17 + nv > sl) return MMF_EINVAL;
        if (!build_huff(tc ? j.ac[th] : j.dc[th], s + q + 1, s + q + 17, nv, !tc)) return MMF_EINVAL;
        q += 17 + nv;
      }
    } else if (m == 0xDD) {
      if (sl < 2) return MMF_EINVAL;
      j.restart = (s[0] << 8) | s[1];
    } else if (m == 0xE0) {
      if (sl >= 5 && memcmp(s, "JFIF", 5) == 0) j.jfif = true;
    } else if (m == 0xEE) {
      if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) j.adobe = s[11];
    } else if (m == 0xDA) {
      if (!sof) return MMF_EINVAL;
      if (j.progressive) {  // scans (and the tables between them) are walked by decode_progressive
        j.scan = d + p - 2;
        j.end = d + n;
        break;
      }
      if (sl < 1 || sl < 4 + 2 * s[0]) return MMF_EINVAL;  // Ns, Ns x (Cs, Td/Ta), Ss, Se, Ah/Al
      j.nscan = s[0];
      if (j.nscan != j.ncomp) return MMF_EUNSUPPORTED;  // multi-scan sequential
      bool seen[4] = {false, false, false, false};
      for (int i = 0; i < j.nscan; ++i) {
        const int cid = s[1 + 2 * i], tt = s[2 + 2 * i];
        int ci = -1;
        for (int c = 0; c < j.ncomp; ++c)
          if (j.comp[c].id == cid) ci = c;
        // libjpeg's JERR_BAD_COMPONENT_ID: unknown or repeated ids (with Ns == Nf and no repeats, every
        // frame component is in the scan, so every td / ta below is set)
        if (ci < 0 || seen[ci]) return MMF_EINVAL;
        seen[ci] = true;
        j.scomp[i] = ci;
        j.comp[ci].td = (tt >> 4) & 3;
        j.comp[ci].ta = tt & 3;
      }
      j.scan = d + p + L;
      j.end = d + n;
      break;
    }
    p += L;
  }
  if (!j.scan) return MMF_EINVAL;
  // Pillow raises "image file is truncated" when the data ends before the EOI marker (its decoder
  // asks for more bytes); such files go to Pillow so the error is the reference's.  Entropy-coded
  // data stuffs every 0xFF data byte as FF 00, so FF D9 can only be a marker.
  {
    const uint8_t* q = j.scan;
    bool eoi = false;
    while (!eoi && q + 1 < j.end) {
      q = (const uint8_t*)memchr(q, 0xFF, (size_t)(j.end - 1 - q));
      if (!q) break;
      eoi = q[1] == 0xD9;
      ++q;
    }
    if (!eoi) return MMF_EUNSUPPORTED;
  }
  for (int c = 0; c < j.ncomp; ++c) {
    if (!j.qt_present[j.comp[c].tq]) return MMF_EINVAL;
    if (!j.progressive && (!j.dc[j.comp[c].td].present || !j.ac[j.comp[c].ta].present)) return MMF_EINVAL;
    j.hmax = j.hmax > j.comp[c].h ? j.hmax : j.comp[c].h;
    j.vmax = j.vmax > j.comp[c].v ? j.vmax : j.comp[c].v;
  }
  if (j.ncomp == 3) {
    if (j.adobe == 0) return MMF_EUNSUPPORTED;  // untransformed (RGB) JPEG
    // libjpeg's default_decompress_parms: no JFIF and no Adobe marker, component ids 'R' 'G' 'B'
    // -> an RGB file (decoded by Pillow)
    if (!j.jfif && j.adobe < 0 && j.comp[0].id == 82 && j.comp[1].id == 71 && j.comp[2].id == 66)
      return MMF_EUNSUPPORTED;
    // luma h, v in {1, 2}, chroma 1x1 (4:4:4, 4:2:2, 4:2:0; 4:4:0 decodes through Pillow)
    if (j.comp[0].h > 2 || j.comp[0].v > 2 || j.comp[1].h != 1 || j.comp[1].v != 1 || j.comp[2].h != 1 ||
        j.comp[2].v != 1 || (j.comp[0].h == 1 && j.comp[0].v == 2))
      return MMF_EUNSUPPORTED;
  }
  j.mcux = (j.width + 8 * j.hmax - 1) / (8 * j.hmax);
  j.mcuy = (j.height + 8 * j.vmax - 1) / (8 * j.vmax);
  return 0;
}

// jdhuff.c bit reader: 0xFF00 unstuffed; at a marker, zeros are fed (the marker is not consumed)
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int n = 0;
  void fill() {
    if (n > 56) return;
    if (end - p >= 8) {  // fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker)
      uint64_t w;
      memcpy(&w, p, 8);
      w = __builtin_bswap64(w);
      const uint64_t x = ~w;
      if (((x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL) == 0) {
        const int k = (64 - n) >> 3;
        acc |= w >> n;
        n += 8 * k;
        p += k;
        if (n < 64) acc &= ~(~0ULL >> n);
        return;
      }
    }
    while (n <= 56) {
      uint32_t b = 0;
      if (p < end) {
        b = *p;
        if (b == 0xFF) {
          const uint32_t nb = p + 1 < end ? p[1] : 0;
          if (nb == 0) p += 2;
          else b = 0;  // marker: zeros from here, p stays
        } else {
          ++p;
        }
      }
      acc |= (uint64_t)b << (56 - n);
      n += 8;
    }
  }
  uint32_t peek(int k) { return (uint32_t)(acc >> (64 - k)); }
  void skip(int k) {
    acc <<= k;
    n -= k;
  }
  int get(int k) {
    if (n < k) fill();
    const int v = (int)peek(k);
    skip(k);
    return v;
  }
  void restart() {  // byte-align, find and skip RSTn
    acc = 0;
    n = 0;
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) p += 2;
  }
};

inline int decode_sym(Bits& b, const Huff& t) {
  if (b.n < 16) b.fill();
  const uint32_t lk = b.peek(kLook);
  const uint16_t e = t.look[lk];
  if (e) {
    b.skip(e >> 8);
    return e & 0xFF;
  }
  int l = kLook + 1;
  int code = (int)b.peek(l);
  while (l <= 16 && code > t.maxcode[l]) {
    ++l;
    code = (int)b.peek(l);
  }
  if (l > 16) {  // corrupt: libjpeg warns and returns symbol 0
    b.skip(16);
    return 0;
  }
  b.skip(l);
  return t.huffval[(code + t.valoff[l]) & 0xFF];
}

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

inline void decode_block(Bits& b, const Huff& dc, const Huff& ac, int& pred, int16_t* blk) {
  memset(blk, 0, 64 * sizeof(int16_t));  // zeroed here, while the block's line is being written anyway
  int t = decode_sym(b, dc);
  int diff = 0;
  if (t) {
    if (b.n < t) b.fill();
    diff = extend(b.get(t), t);
  }
  pred = (int)((uint32_t)pred + (uint32_t)diff);  // (wraps on corrupt data only)
  blk[0] = (int16_t)pred;
  for (int k = 1; k < 64; ++k) {
    if (b.n < 16) b.fill();
    const int32_t f = ac.acfast[b.peek(kLook)];
    if (f) {
      b.skip(f & 0xFF);
      if (f & 0x8000) break;  // end of block
      k += (f >> 8) & 15;
      blk[kZigzag[k]] = (int16_t)(f >> 16);
      continue;
    }
    const int rs = decode_sym(b, ac);
    const int r = rs >> 4, s = rs & 15;
    if (s) {
      k += r;
      if (b.n < s) b.fill();
      const int v = extend(b.get(s), s);
      blk[kZigzag[k]] = (int16_t)v;  // k <= 63 + 15: the guard slots alias 63 (corrupt data only)
    } else {
      if (r != 15) break;
      k += 15;
    }
  }
}

}  // namespace

extern "C" int mmf_jpeg_header(const uint8_t* data, int64_t nbytes, int32_t* info) {
  if (!data || !info) return MMF_EINVAL;
  Jpeg j;
  const int rc = parse(data, nbytes, j);
  memset(info, 0, sizeof(int32_t) * MMF_JPEG_INFO_LEN);
  info[0] = j.width;
  info[1] = j.height;
  info[2] = j.ncomp;
  if (rc) return rc;
  info[3] = j.hmax;
  info[4] = j.vmax;
  int64_t blocks = 0;
  for (int c = 0; c < j.ncomp; ++c) {
    info[5 + 2 * c] = j.mcux * j.comp[c].h;  // bw_c
    info[6 + 2 * c] = j.mcuy * j.comp[c].v;  // bh_c
    blocks += (int64_t)info[5 + 2 * c] * info[6 + 2 * c];
  }
  if (blocks > 0x7fffffff) return MMF_EUNSUPPORTED;
  info[11] = (int32_t)blocks;
  return 0;
}

namespace {

// Entropy decoding of every block of the scan(s); on_block(global block index, dc, ac, pred) decodes
// one block into the caller's representation, on_skip(global block index) marks a block of the
// MCU-padded grid that no scan codes (non-interleaved scans cover only the component's extent).
template <class OnBlock, class OnSkip>
int walk_blocks(Jpeg& j, OnBlock&& on_block, OnSkip&& on_skip) {
  int64_t base[3];
  int bw[3], bh[3];
  int64_t off = 0;
  for (int c = 0; c < j.ncomp; ++c) {
    bw[c] = j.mcux * j.comp[c].h;
    bh[c] = j.mcuy * j.comp[c].v;
    base[c] = off;
    off += (int64_t)bw[c] * bh[c];
  }
  Bits b{j.scan, j.end};
  int pred[3] = {0, 0, 0};
  const int ri = j.restart;
  int64_t unit = 0;
  if (j.ncomp == 1) {
    const Comp& c = j.comp[0];
    const int cw = (j.width * c.h + j.hmax - 1) / j.hmax, ch = (j.height * c.v + j.vmax - 1) / j.vmax;
    const int nbx = (cw + 7) / 8, nby = (ch + 7) / 8;
    for (int by = 0; by < bh[0]; ++by)
      for (int bx = (by < nby ? nbx : 0); bx < bw[0]; ++bx) on_skip((int64_t)by * bw[0] + bx);
    for (int by = 0; by < nby; ++by)
      for (int bx = 0; bx < nbx; ++bx, ++unit) {
        if (ri && unit && unit % ri == 0) {
          b.restart();
          pred[0] = 0;
        }
        on_block(b, (int64_t)by * bw[0] + bx, j.dc[c.td], j.ac[c.ta], pred[0]);
      }
    return 0;
  }
  for (int my = 0; my < j.mcuy; ++my)
    for (int mx = 0; mx < j.mcux; ++mx, ++unit) {
      if (ri && unit && unit % ri == 0) {
        b.restart();
        pred[0] = pred[1] = pred[2] = 0;
      }
      for (int si = 0; si < j.nscan; ++si) {
        const int ci = j.scomp[si];
        const Comp& c = j.comp[ci];
        for (int yy = 0; yy < c.v; ++yy)
          for (int xx = 0; xx < c.h; ++xx)
            on_block(b, base[ci] + (int64_t)(my * c.v + yy) * bw[ci] + mx * c.h + xx, j.dc[c.td], j.ac[c.ta],
                     pred[ci]);
      }
    }
  return 0;
}

// Packed block record (mmf_jpeg_entropy_packed): uint64 mask of the nonzero ZIGZAG positions, then
// their int16 values in zigzag (= decode) order, padded to 8 bytes.  Returns the record's bytes.
inline int decode_block_packed(Bits& b, const Huff& dc, const Huff& ac, int& pred, uint8_t* rec) {
  uint64_t mask = 0;
  int16_t* val = reinterpret_cast<int16_t*>(rec + 8);
  int n = 0;
  int t = decode_sym(b, dc);
  int diff = 0;
  if (t) {
    if (b.n < t) b.fill();
    diff = extend(b.get(t), t);
  }
  pred = (int)((uint32_t)pred + (uint32_t)diff);  // (wraps on corrupt data only)
  if (pred) {
    mask = 1;
    val[n++] = (int16_t)pred;
  }
  for (int k = 1; k < 64; ++k) {
    if (b.n < 16) b.fill();
    const int32_t f = ac.acfast[b.peek(kLook)];
    int v;
    if (f) {
      b.skip(f & 0xFF);
      if (f & 0x8000) break;  // end of block
      k += (f >> 8) & 15;
      v = f >> 16;
    } else {
      const int rs = decode_sym(b, ac);
      const int r = rs >> 4, sz = rs & 15;
      if (!sz) {
        if (r != 15) break;
        k += 15;
        continue;
      }
      k += r;
      if (b.n < sz) b.fill();
      v = extend(b.get(sz), sz);
    }
    if (k > 63) break;  // corrupt run past the block: libjpeg drops the coefficient
    mask |= 1ull << k;  // (k only grows: each position is written at most once)
    val[n++] = (int16_t)v;
  }
  memcpy(rec, &mask, 8);
  for (int i = n; i & 3; ++i) val[i] = 0;  // deterministic padding
  return (8 + 2 * n + 7) & ~7;
}

// ---- progressive Huffman (SOF2), restating libjpeg's jdphuff.c: every scan is decoded into the
// dense coefficient planes (DC first / refine, AC first / refine with end-of-band runs); the
// complete planes are what a sequential file of the same image would carry.

// pack one dense natural-order block into a record (see decode_block_packed), its nonzero zigzag
// positions given by `mask`; 0 bytes for an all-zero block (it then shares record 0)
inline int pack_block(const int16_t* blk, uint64_t mask, uint8_t* rec) {
  if (!mask) return 0;
  int16_t* val = reinterpret_cast<int16_t*>(rec + 8);
  int n = 0;
  for (uint64_t m = mask; m; m &= m - 1) val[n++] = blk[kZigzag[__builtin_ctzll(m)]];
  memcpy(rec, &mask, 8);
  for (int i = n; i & 3; ++i) val[i] = 0;
  return (8 + 2 * n + 7) & ~7;
}

inline int get_bits(Bits& b, int k) { return k ? b.get(k) : 0; }

// coefs: dense [blocks][64] natural order, zeroed by the caller; nzm[block] = the zigzag positions
// 1..63 that are nonzero once every scan is in (bit 0 is left to the caller: DC = coefs[b * 64])
int decode_progressive(Jpeg& j, int16_t* coefs, uint64_t* nzm) {
  int64_t base[3];
  int bw[3], nbx[3], nby[3];
  int64_t off = 0;
  for (int c = 0; c < j.ncomp; ++c) {
    const Comp& cc = j.comp[c];
    bw[c] = j.mcux * cc.h;
    base[c] = off;
    off += (int64_t)bw[c] * j.mcuy * cc.v;
    const int cw = (j.width * cc.h + j.hmax - 1) / j.hmax, ch = (j.height * cc.v + j.vmax - 1) / j.vmax;
    nbx[c] = (cw + 7) / 8;
    nby[c] = (ch + 7) / 8;
  }
  memset(nzm, 0, off * sizeof(uint64_t));
  const uint8_t* p = j.scan;
  const uint8_t* end = j.end;
  while (p + 4 <= end) {
    if (p[0] != 0xFF) {  // entropy data a scan did not consume (corrupt / padded): find the marker
      ++p;
      continue;
    }
    const int m = p[1];
    if (m == 0xFF) { ++p; continue; }
    if (m == 0x00 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) { p += 2; continue; }
    if (m == 0xD9) break;  // EOI
    p += 2;
    const int L = (p[0] << 8) | p[1];
    if (L < 2 || p + L > end) return MMF_EINVAL;
    const uint8_t* sg = p + 2;
    const int sl = L - 2;
    if (m == 0xC4) {
      int q = 0;
      while (q < sl) {
        if (q + 17 > sl) return MMF_EINVAL;
        const int tc = sg[q] >> 4, th = sg[q] & 3;
        int nv = 0;
        for (int i = 0; i < 16; ++i) nv += sg[q + 1 + i];
        if (nv > 256 || q + 17 + nv > sl) return MMF_EINVAL;
        if (!build_huff(tc ? j.ac[th] : j.dc[th], sg + q + 1, sg + q + 17, nv, !tc)) return MMF_EINVAL;
        q += 17 + nv;
      }
    } else if (m == 0xDD) {
      if (sl < 2) return MMF_EINVAL;
      j.restart = (sg[0] << 8) | sg[1];
    } else if (m == 0xDB) {
      return MMF_EUNSUPPORTED;  // a quantisation table redefined between scans: left to Pillow
    } else if (m == 0xDA) {
      if (sl < 1) return MMF_EINVAL;
      const int ns = sg[0];
      if (ns < 1 || ns > j.ncomp || sl < 4 + 2 * ns) return MMF_EINVAL;
      int sc[3], td[3], ta[3];
      for (int i = 0; i < ns; ++i) {
        const int cid = sg[1 + 2 * i], tt = sg[2 + 2 * i];
        sc[i] = -1;
        for (int c = 0; c < j.ncomp; ++c)
          if (j.comp[c].id == cid) sc[i] = c;
        if (sc[i] < 0) return MMF_EINVAL;
        td[i] = (tt >> 4) & 3;
        ta[i] = tt & 3;
      }
      const int Ss = sg[1 + 2 * ns], Se = sg[2 + 2 * ns], Ah = sg[3 + 2 * ns] >> 4, Al = sg[3 + 2 * ns] & 15;
      if (Ss > Se || Se > 63 || (Ss == 0 && Se != 0) || (Ss > 0 && ns != 1) || Al > 13) return MMF_EINVAL;
      for (int i = 0; i < ns; ++i) {
        if (Ss == 0 && Ah == 0 && !j.dc[td[i]].present) return MMF_EINVAL;
        if (Ss > 0 && !j.ac[ta[i]].present) return MMF_EINVAL;
      }
      Bits b{p + L, end};
      int pred[3] = {0, 0, 0};
      int eobrun = 0;
      const int ri = j.restart;
      int64_t unit = 0;
      const int p1 = 1 << Al, m1 = -(1 << Al);
      const uint64_t band = (Se == 63 ? ~0ull : (1ull << (Se + 1)) - 1) & (~0ull << Ss);
      // correction bits of the already-nonzero coefficients in `sel` (one bit each, in k order),
      // read up to 16 at a time
      auto refine = [&](int16_t* blk, uint64_t sel) {
        while (sel) {
          const int cnt = __builtin_popcountll(sel), take = cnt < 16 ? cnt : 16;
          const uint32_t bits = (uint32_t)b.get(take);
          for (int t = take - 1; t >= 0; --t) {
            const int kk = __builtin_ctzll(sel);
            sel &= sel - 1;
            int16_t& c = blk[kZigzag[kk]];
            if (((bits >> t) & 1) && (c & p1) == 0) c = (int16_t)(c >= 0 ? c + p1 : c + m1);
          }
        }
      };
      auto block = [&](int i, int64_t bi, int16_t* blk) {
        if (Ss == 0) {
          if (Ah == 0) {  // DC first
            int t = decode_sym(b, j.dc[td[i]]);
            if (t > 16) t = 16;
            const int diff = t ? extend(b.get(t), t) : 0;
            pred[i] = (int)((uint32_t)pred[i] + (uint32_t)diff);
            blk[0] = (int16_t)((uint32_t)pred[i] << Al);
          } else if (get_bits(b, 1)) {  // DC refine
            blk[0] = (int16_t)(blk[0] | p1);
          }
          return;
        }
        const Huff& ac = j.ac[ta[i]];
        uint64_t& nz = nzm[bi];  // zigzag positions already nonzero (earlier AC scans)
        if (Ah == 0) {  // AC first
          if (eobrun > 0) {
            --eobrun;
            return;
          }
          for (int k = Ss; k <= Se; ++k) {
            if (b.n < 16) b.fill();
            const int32_t f = ac.acfast[b.peek(kLook)];
            int v;
            if (f) {
              b.skip(f & 0xFF);
              if (f & 0x8000) break;  // EOB0: a run of one block (this one), eobrun stays 0
              k += (f >> 8) & 15;
              v = f >> 16;
            } else {
              const int rs = decode_sym(b, ac), r = rs >> 4, sz = rs & 15;
              if (!sz) {
                if (r == 15) {
                  k += 15;
                  continue;
                }
                eobrun = (1 << r) + get_bits(b, r) - 1;
                break;
              }
              k += r;
              v = extend(b.get(sz), sz);
            }
            if (k > 63) break;
            blk[kZigzag[k]] = (int16_t)(v * (1 << Al));
            nz |= 1ull << k;
          }
          return;
        }
        // AC refine (jdphuff.c decode_mcu_AC_refine) over bit masks: a run of r skips r still-zero
        // coefficients and corrects every nonzero one passed over; the (r + 1)-th zero gets the
        // newly nonzero value
        int k = Ss;
        if (eobrun == 0) {
          for (; k <= Se; ++k) {
            const int rs = decode_sym(b, ac);
            const int r = rs >> 4, sz = rs & 15;
            int v = 0;
            if (sz) {
              v = get_bits(b, 1) ? p1 : m1;
            } else if (r != 15) {
              eobrun = (1 << r) + get_bits(b, r);
              break;
            }
            const uint64_t from = ~0ull << k;
            uint64_t z = ~nz & band & from;
            for (int t = 0; t < r && z; ++t) z &= z - 1;
            const int tgt = z ? __builtin_ctzll(z) : Se + 1;
            refine(blk, nz & band & from & (tgt >= 64 ? ~0ull : (1ull << tgt) - 1));
            k = tgt;
            if (v && k <= Se) {
              blk[kZigzag[k]] = (int16_t)v;
              nz |= 1ull << k;
            }
          }
        }
        if (eobrun > 0) {
          if (k <= 63) refine(blk, nz & band & (~0ull << k));
          --eobrun;
        }
      };
      auto restart_check = [&]() {
        if (ri && unit && unit % ri == 0) {
          b.restart();
          pred[0] = pred[1] = pred[2] = 0;
          eobrun = 0;
        }
      };
      if (ns > 1) {
        for (int my = 0; my < j.mcuy; ++my)
          for (int mx = 0; mx < j.mcux; ++mx, ++unit) {
            restart_check();
            for (int i = 0; i < ns; ++i) {
              const Comp& c = j.comp[sc[i]];
              for (int yy = 0; yy < c.v; ++yy)
                for (int xx = 0; xx < c.h; ++xx)
                {
                  const int64_t bi = base[sc[i]] + (int64_t)(my * c.v + yy) * bw[sc[i]] + mx * c.h + xx;
                  block(i, bi, coefs + bi * 64);
                }
            }
          }
      } else {
        const int ci = sc[0];
        for (int by = 0; by < nby[ci]; ++by)
          for (int bx = 0; bx < nbx[ci]; ++bx, ++unit) {
            restart_check();
            const int64_t bi = base[ci] + (int64_t)by * bw[ci] + bx;
            block(0, bi, coefs + bi * 64);
          }
      }
      p = b.p;  // the bit reader stops at the next marker
      continue;
    }
    p += L;
  }
  return 0;
}

}  // namespace

extern "C" int mmf_jpeg_entropy(const uint8_t* data, int64_t nbytes, int16_t* coefs, uint16_t* qt) {
  if (!data || !coefs || !qt) return MMF_EINVAL;
  Jpeg j;
  const int rc = parse(data, nbytes, j);
  if (rc) return rc;
  for (int c = 0; c < j.ncomp; ++c) memcpy(qt + 64 * c, j.qt[j.comp[c].tq], 64 * sizeof(uint16_t));
  if (j.progressive) {
    int64_t blocks = 0;
    for (int c = 0; c < j.ncomp; ++c) blocks += (int64_t)j.mcux * j.comp[c].h * j.mcuy * j.comp[c].v;
    memset(coefs, 0, blocks * 128);
    thread_local std::vector<uint64_t> nzm;
    if ((int64_t)nzm.size() < blocks) nzm.resize(blocks);
    return decode_progressive(j, coefs, nzm.data());
  }
  return walk_blocks(
      j, [&](Bits& b, int64_t gb, const Huff& dc, const Huff& ac, int& pred) { decode_block(b, dc, ac, pred, coefs + gb * 64); },
      [&](int64_t gb) { memset(coefs + gb * 64, 0, 128); });
}

extern "C" int64_t mmf_jpeg_packed_bound(int32_t blocks) { return 8 + (int64_t)blocks * (8 + 128); }

extern "C" int mmf_jpeg_entropy_packed(const uint8_t* data, int64_t nbytes, uint8_t* out, int64_t cap,
                                       uint32_t* block_off, uint16_t* qt, int64_t* used) {
  if (!data || !out || !block_off || !qt || !used) return MMF_EINVAL;
  Jpeg j;
  const int rc = parse(data, nbytes, j);
  if (rc) return rc;
  int64_t blocks = 0;
  for (int c = 0; c < j.ncomp; ++c) {
    memcpy(qt + 64 * c, j.qt[j.comp[c].tq], 64 * sizeof(uint16_t));
    blocks += (int64_t)j.mcux * j.comp[c].h * j.mcuy * j.comp[c].v;
  }
  if (cap < mmf_jpeg_packed_bound((int32_t)blocks) || mmf_jpeg_packed_bound((int32_t)blocks) > 0xFFFFFFFFll)
    return MMF_ERANGE;
  memset(out, 0, 8);  // record 0: the all-zero block (padding blocks point here)
  int64_t cur = 8;
  if (j.progressive) {  // all scans into dense planes first, then one record per nonzero block
    thread_local std::vector<int16_t> dense;
    thread_local std::vector<uint64_t> nzm;
    if ((int64_t)dense.size() < blocks * 64) dense.resize(blocks * 64);
    if ((int64_t)nzm.size() < blocks) nzm.resize(blocks);
    memset(dense.data(), 0, blocks * 128);
    const int prc = decode_progressive(j, dense.data(), nzm.data());
    if (prc) return prc;
    for (int64_t b = 0; b < blocks; ++b) {
      const int16_t* blk = dense.data() + b * 64;
      const int sz = pack_block(blk, nzm[b] | (uint64_t)(blk[0] != 0), out + cur);
      block_off[b] = sz ? (uint32_t)cur : 0;
      cur += sz;
    }
    *used = cur;
    return 0;
  }
  walk_blocks(
      j,
      [&](Bits& b, int64_t gb, const Huff& dc, const Huff& ac, int& pred) {
        block_off[gb] = (uint32_t)cur;
        cur += decode_block_packed(b, dc, ac, pred, out + cur);
      },
      [&](int64_t gb) { block_off[gb] = 0; });
  *used = cur;
  return 0;
}

extern "C" int mmf_jpeg_stage_packed(const uint8_t* data, int64_t nbytes, uint8_t* dst, int64_t dst_cap,
                                     int64_t* cursor, uint32_t* block_off, uint16_t* qt, int64_t* rec_off) {
  if (!data || !dst || !cursor || !block_off || !qt || !rec_off) return MMF_EINVAL;
  Jpeg j;
  int rc = parse(data, nbytes, j);
  if (rc) return rc;
  int64_t blocks = 0;
  for (int c = 0; c < j.ncomp; ++c) blocks += (int64_t)j.mcux * j.comp[c].h * j.mcuy * j.comp[c].v;
  if (blocks > 0x7fffffff) return MMF_ERANGE;
  const int64_t bound = mmf_jpeg_packed_bound((int32_t)blocks);
  thread_local std::vector<uint8_t> scratch;  // per caller thread, reused: no page faults per image
  if ((int64_t)scratch.size() < bound) scratch.resize(bound + bound / 4);
  int64_t used = 0;
  rc = mmf_jpeg_entropy_packed(data, nbytes, scratch.data(), (int64_t)scratch.size(), block_off, qt, &used);
  if (rc) return rc;
  const int64_t off = __atomic_fetch_add(cursor, (used + 7) & ~7ll, __ATOMIC_RELAXED);
  *rec_off = off;
  if (off + used > dst_cap) return MMF_ERANGE;
  memcpy(dst + off, scratch.data(), used);
  return 0;
}

extern "C" int mmf_jpeg_stage_packed_batch(const uint8_t* const* datas, const int64_t* nbytes, int n, uint8_t* dst,
                                           int64_t dst_cap, int64_t* cursor, uint32_t* block_off,
                                           const int64_t* block_base, uint16_t* qt, int64_t* rec_off, int nthreads,
                                           int32_t* rcs) {
  if (n < 0 || (n > 0 && (!datas || !nbytes || !dst || !cursor || !block_off || !block_base || !qt || !rec_off || !rcs)))
    return MMF_EINVAL;
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int k = next.fetch_add(1); k < n; k = next.fetch_add(1))
      rcs[k] = mmf_jpeg_stage_packed(datas[k], nbytes[k], dst, dst_cap, cursor, block_off + block_base[k],
                                     qt + 192 * (int64_t)k, rec_off + k);
  };
  const int nt = nthreads < 1 ? 1 : (nthreads > n ? n : nthreads);
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}

extern "C" int mmf_jpeg_header_batch(const uint8_t* const* datas, const int64_t* nbytes, int n, int32_t* infos,
                                     int32_t* rcs, int nthreads) {
  if (n < 0 || (n > 0 && (!datas || !nbytes || !infos || !rcs))) return MMF_EINVAL;
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int k = next.fetch_add(1); k < n; k = next.fetch_add(1))
      rcs[k] = datas[k] ? mmf_jpeg_header(datas[k], nbytes[k], infos + (int64_t)k * MMF_JPEG_INFO_LEN) : MMF_EINVAL;
  };
  const int nt = nthreads < 1 ? 1 : (nthreads > (n + 15) / 16 ? (n + 15) / 16 : nthreads);  // >= 16 files a thread
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}
