// Host half of the device JPEG decode: marker parsing and baseline
// Huffman entropy decoding into quantised DCT coefficient planes -- the only inherently serial part
// of a JPEG decode.  Dequantisation, the islow IDCT, fancy chroma upsampling and YCbCr -> RGB run on
// the device (jpeg.hip); the pixels equal Pillow's decoder (libjpeg-turbo: jdhuff.c, jidctint.c,
// jdsample.c, jdcolor.c), which is what the reference's Image.open(...).convert("RGB")
// (misinfo_forensics.py:255-258) runs.  Restatement and pinning: oracle/jpeg_decode.py.
//
// Supported (mmf_jpeg_header returns 0): 8-bit baseline / extended sequential Huffman (SOF0/SOF1),
// one scan holding every component, 1 component or 3 YCbCr components with luma sampling h, v <= 2
// and chroma 1x1 (4:4:4, 4:2:2, 4:2:0); anything else returns MMF_EUNSUPPORTED and the caller decodes
// that file on the host (Pillow).
//
// Coefficient layout (mmf_jpeg_entropy): component c's blocks as [bh_c][bw_c][64] int16, natural
// (row-major) order, c = 0, 1, 2 back to back; bw_c = mcux * h_c, bh_c = mcuy * v_c (the MCU-padded
// block grid; blocks outside a single-component scan's extent stay zero, as in libjpeg).
#include <cstdint>
#include <cstring>
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
  // (value << 16) | (run << 8) | total bits; 0 = take the symbol path
  int32_t acfast[1 << kLook];
};

bool build_huff(Huff& t, const uint8_t* bits, const uint8_t* vals, int nvals) {
  int code = 0, k = 0;
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
    if (!sz || l + sz > kLook) continue;
    int v = (lk >> (kLook - l - sz)) & ((1 << sz) - 1);
    if (v < (1 << (sz - 1))) v -= (1 << sz) - 1;
    t.acfast[lk] = (int32_t)((uint32_t)v << 16) | (r << 8) | (l + sz);
  }
  t.present = true;
  return true;
}

struct Comp {
  int id, h, v, tq, td, ta;
};

struct Jpeg {
  int width = 0, height = 0, ncomp = 0, restart = 0, adobe = -1;
  Comp comp[4];
  int nscan = 0, scomp[4];
  uint16_t qt[4][64];
  bool qt_present[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  const uint8_t* scan = nullptr;  // entropy-coded segment start
  const uint8_t* end = nullptr;
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
    if (m == 0xC0 || m == 0xC1) {
      if (sl < 6 || s[0] != 8) return MMF_EUNSUPPORTED;  // 12-bit
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
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return MMF_EUNSUPPORTED;  // progressive, lossless, arithmetic
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
        if (!build_huff(tc ? j.ac[th] : j.dc[th], s + q + 1, s + q + 17, nv)) return MMF_EINVAL;
        q += 17 + nv;
      }
    } else if (m == 0xDD) {
      if (sl < 2) return MMF_EINVAL;
      j.restart = (s[0] << 8) | s[1];
    } else if (m == 0xEE) {
      if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) j.adobe = s[11];
    } else if (m == 0xDA) {
      if (!sof) return MMF_EINVAL;
      j.nscan = s[0];
      if (j.nscan != j.ncomp) return MMF_EUNSUPPORTED;  // multi-scan sequential
      for (int i = 0; i < j.nscan; ++i) {
        const int cid = s[1 + 2 * i], tt = s[2 + 2 * i];
        int ci = -1;
        for (int c = 0; c < j.ncomp; ++c)
          if (j.comp[c].id == cid) ci = c;
        if (ci < 0) return MMF_EINVAL;
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
  for (int c = 0; c < j.ncomp; ++c) {
    if (!j.qt_present[j.comp[c].tq] || !j.dc[j.comp[c].td].present || !j.ac[j.comp[c].ta].present) return MMF_EINVAL;
    j.hmax = j.hmax > j.comp[c].h ? j.hmax : j.comp[c].h;
    j.vmax = j.vmax > j.comp[c].v ? j.vmax : j.comp[c].v;
  }
  if (j.ncomp == 3) {
    if (j.adobe == 0) return MMF_EUNSUPPORTED;  // untransformed (RGB) JPEG
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
  pred += diff;
  blk[0] = (int16_t)pred;
  for (int k = 1; k < 64; ++k) {
    if (b.n < 16) b.fill();
    const int32_t f = ac.acfast[b.peek(kLook)];
    if (f) {
      k += (f >> 8) & 15;
      b.skip(f & 0xFF);
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
  pred += diff;
  if (pred) {
    mask = 1;
    val[n++] = (int16_t)pred;
  }
  for (int k = 1; k < 64; ++k) {
    if (b.n < 16) b.fill();
    const int32_t f = ac.acfast[b.peek(kLook)];
    int v;
    if (f) {
      k += (f >> 8) & 15;
      b.skip(f & 0xFF);
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

}  // namespace

extern "C" int mmf_jpeg_entropy(const uint8_t* data, int64_t nbytes, int16_t* coefs, uint16_t* qt) {
  if (!data || !coefs || !qt) return MMF_EINVAL;
  Jpeg j;
  const int rc = parse(data, nbytes, j);
  if (rc) return rc;
  for (int c = 0; c < j.ncomp; ++c) memcpy(qt + 64 * c, j.qt[j.comp[c].tq], 64 * sizeof(uint16_t));
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
