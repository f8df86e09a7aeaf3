// Device half of the JPEG decode (host half: jpeg_host.cpp).  Bit-exact with Pillow's libjpeg-turbo
// (restated in oracle/jpeg_decode.py): per 8x8 block the islow integer IDCT with dequantisation
// (jidctint.c: CONST_BITS 13, PASS1_BITS 2, DESCALE rounding, post-IDCT range limit), then per
// output pixel the fancy chroma upsampling (jdsample.c h2v1 / h2v2 triangle filters, edge samples
// replicated as jdmainct.c's context rows do) and YCbCr -> RGB (jdcolor.c tables, SCALEBITS 16),
// written as RGBX for mmf_resize_pil.
//   jpeg_idct_kernel : one thread per block; its packed record in (mask + nonzero values, ~48 B on
//                      photos instead of 128), 8 rows of 8 samples out (adjacent threads = adjacent
//                      blocks of a block row: coalesced row stores)
//   jpeg_color_kernel: one thread per output pixel, one 4-B RGBX store
// Both are HBM / latency-bound byte work (a 640x480 4:2:0 q90 image: 0.35 MB of packed coefficients
// -- 0.92 MB dense --, 0.46 MB of samples, 1.2 MB of RGBX).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int kInfoLen = 16;  // MMF_JPEG_INFO_LEN

// jidctint.c constants (FIX(x) at CONST_BITS = 13)
constexpr int kF0298 = 2446, kF0390 = 3196, kF0541 = 4433, kF0765 = 6270, kF0899 = 7373, kF1175 = 9633,
              kF1501 = 12299, kF1847 = 15137, kF1961 = 16069, kF2053 = 16819, kF2562 = 20995, kF3072 = 25172;

MMF_DEV void idct_1d(const int* d, int* o, int shift) {
  int z2 = d[2], z3 = d[6];
  int z1 = (z2 + z3) * kF0541;
  const int tmp2 = z1 + z3 * (-kF1847);
  const int tmp3 = z1 + z2 * kF0765;
  const int tmp0 = (d[0] + d[4]) * 8192;  // << CONST_BITS (as a multiply: defined for negatives)
  const int tmp1 = (d[0] - d[4]) * 8192;
  const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  int t0 = d[7], t1 = d[5], t2 = d[3], t3 = d[1];
  z1 = t0 + t3;
  z2 = t1 + t2;
  z3 = t0 + t2;
  int z4 = t1 + t3;
  const int z5 = (z3 + z4) * kF1175;
  t0 *= kF0298;
  t1 *= kF2053;
  t2 *= kF3072;
  t3 *= kF1501;
  z1 *= -kF0899;
  z2 *= -kF2562;
  z3 = z3 * (-kF1961) + z5;
  z4 = z4 * (-kF0390) + z5;
  t0 += z1 + z3;
  t1 += z2 + z4;
  t2 += z2 + z3;
  t3 += z1 + z4;
  const int r = 1 << (shift - 1);
  o[0] = (tmp10 + t3 + r) >> shift;
  o[7] = (tmp10 - t3 + r) >> shift;
  o[1] = (tmp11 + t2 + r) >> shift;
  o[6] = (tmp11 - t2 + r) >> shift;
  o[2] = (tmp12 + t1 + r) >> shift;
  o[5] = (tmp12 - t1 + r) >> shift;
  o[3] = (tmp13 + t0 + r) >> shift;
  o[4] = (tmp13 - t0 + r) >> shift;
}

// jdmaster.c post-IDCT range limit: idct_range_limit[v & 1023] (CENTERJSAMPLE folded in)
MMF_DEV uint32_t range_limit_idct(int v) {
  const int m = v & 1023;
  return (uint32_t)(m < 128 ? m + 128 : m < 512 ? 255 : m < 896 ? 0 : m - 896);
}

// zigzag position -> natural (row-major) index (ITU T.81 Figure A.6)
__constant__ constexpr uint8_t kZigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// grid (ceil(max blocks / 256), B); block 256.  Coefficients arrive packed (mmf_jpeg_entropy_packed):
// the block's record = uint64 mask of nonzero zigzag positions + their int16 values in zigzag order.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const uint8_t* __restrict__ packed,
                                                        const uint32_t* __restrict__ block_off,
                                                        const int64_t* __restrict__ pk_off, const uint16_t* __restrict__ qt,
                                                        const int64_t* __restrict__ coef_blocks,
                                                        const int32_t* __restrict__ infos, uint8_t* __restrict__ samples) {
  const int img = blockIdx.y;
  const int32_t* inf = infos + (size_t)img * kInfoLen;
  const int blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= inf[11]) return;
  const int ncomp = inf[2];
  int c = 0, rem = blk, cum = 0;
  while (c + 1 < ncomp && rem >= inf[5 + 2 * c] * inf[6 + 2 * c]) {
    rem -= inf[5 + 2 * c] * inf[6 + 2 * c];
    cum += inf[5 + 2 * c] * inf[6 + 2 * c];
    ++c;
  }
  const int bw = inf[5 + 2 * c];
  const int by = rem / bw, bx = rem - by * bw;
  const int64_t b0 = coef_blocks[img];
  const uint8_t* rec = packed + pk_off[img] + block_off[b0 + blk];
  const uint2 mw = *reinterpret_cast<const uint2*>(rec);
  const uint64_t mask = (uint64_t)mw.x | (uint64_t)mw.y << 32;
  const int16_t* val = reinterpret_cast<const int16_t*>(rec + 8);
  const uint16_t* q = qt + (size_t)img * 192 + c * 64;
  int qn[64];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 w0 = *reinterpret_cast<const uint4*>(q + i * 8);
    const uint32_t qv[4] = {w0.x, w0.y, w0.z, w0.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      qn[i * 8 + 2 * k] = (int)(qv[k] & 0xFFFF);
      qn[i * 8 + 2 * k + 1] = (int)(qv[k] >> 16);
    }
  }
  // dequantise: zigzag position k -> natural index kZigzag[k] (compile-time per unrolled k)
  int d[64];
  int n = 0;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const int nat = kZigzag[k];
    if ((mask >> k) & 1) {
      d[nat] = (int)val[n] * qn[nat];
      ++n;
    } else {
      d[nat] = 0;
    }
  }
  // pass 1: columns (d[v * 8 + u], inputs down a column) -> workspace, descaled by CONST_BITS - PASS1_BITS
  int ws[64];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    int in[8], o[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) in[v] = d[v * 8 + u];
    idct_1d(in, o, 11);
#pragma unroll
    for (int v = 0; v < 8; ++v) ws[v * 8 + u] = o[v];
  }
  // pass 2: rows -> samples, descaled by CONST_BITS + PASS1_BITS + 3, range-limited
  uint8_t* plane = samples + (b0 + cum) * 64;
  const int pitch = bw * 8;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int o[8];
    idct_1d(ws + r * 8, o, 18);
    const uint32_t lo = range_limit_idct(o[0]) | range_limit_idct(o[1]) << 8 | range_limit_idct(o[2]) << 16 |
                        range_limit_idct(o[3]) << 24;
    const uint32_t hi = range_limit_idct(o[4]) | range_limit_idct(o[5]) << 8 | range_limit_idct(o[6]) << 16 |
                        range_limit_idct(o[7]) << 24;
    *reinterpret_cast<uint2*>(plane + (size_t)(by * 8 + r) * pitch + bx * 8) = make_uint2(lo, hi);
  }
}

MMF_DEV int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// grid (ceil(max pixels / 256), B); block 256
__global__ __launch_bounds__(256) void jpeg_color_kernel(const int64_t* __restrict__ coef_blocks,
                                                         const int32_t* __restrict__ infos,
                                                         const uint8_t* __restrict__ samples,
                                                         uint8_t* __restrict__ out, const int64_t* __restrict__ out_off) {
  const int img = blockIdx.y;
  const int32_t* inf = infos + (size_t)img * kInfoLen;
  const int W = inf[0], H = inf[1];
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= W * H) return;
  const int y = p / W, x = p - y * W;
  const uint8_t* s0 = samples + coef_blocks[img] * 64;
  const int pitch0 = inf[5] * 8;
  const int Y = s0[(size_t)y * pitch0 + x];
  uint32_t px;
  if (inf[2] == 1) {
    px = (uint32_t)Y * 0x010101u | 0xFF000000u;
  } else {
    const int fh = inf[3], fv = inf[4];  // chroma is 1x1: the upsampling factors are luma's
    const uint8_t* s1 = s0 + (size_t)inf[5] * inf[6] * 64;
    const uint8_t* s2 = s1 + (size_t)inf[7] * inf[8] * 64;
    const int pc = inf[7] * 8;
    const int dw = (W + fh - 1) / fh, dh = (H + fv - 1) / fv;  // downsampled_width / _height
    int cb, cr;
    if (fh == 1 && fv == 1) {
      cb = s1[(size_t)y * pc + x];
      cr = s2[(size_t)y * pc + x];
    } else if (fv == 1) {  // h2v1: (3 in[j] + in[j -/+ 1] + 1 / 2) >> 2, edges replicated
      const int j = x >> 1, jn = (x & 1) ? min(j + 1, dw - 1) : max(j - 1, 0), bias = (x & 1) ? 2 : 1;
      const uint8_t* r1 = s1 + (size_t)y * pc;
      const uint8_t* r2 = s2 + (size_t)y * pc;
      cb = (3 * r1[j] + r1[jn] + bias) >> 2;
      cr = (3 * r2[j] + r2[jn] + bias) >> 2;
    } else {  // h2v2: column sums 3 in[i] + in[i -/+ 1], then (3 cs[j] + cs[j -/+ 1] + 8 / 7) >> 4
      const int i = y >> 1, iv = (y & 1) ? min(i + 1, dh - 1) : max(i - 1, 0);
      const int j = x >> 1, jn = (x & 1) ? min(j + 1, dw - 1) : max(j - 1, 0), bias = (x & 1) ? 7 : 8;
      const uint8_t *a1 = s1 + (size_t)i * pc, *b1 = s1 + (size_t)iv * pc;
      const uint8_t *a2 = s2 + (size_t)i * pc, *b2 = s2 + (size_t)iv * pc;
      cb = (3 * (3 * a1[j] + b1[j]) + (3 * a1[jn] + b1[jn]) + bias) >> 4;
      cr = (3 * (3 * a2[j] + b2[j]) + (3 * a2[jn] + b2[jn]) + bias) >> 4;
    }
    // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (FIX(x) = x * 65536 + 0.5)
    const int cbx = cb - 128, crx = cr - 128;
    const int R = clamp255(Y + ((91881 * crx + 32768) >> 16));
    const int G = clamp255(Y + ((-22554 * cbx + 32768 - 46802 * crx) >> 16));
    const int B = clamp255(Y + ((116130 * cbx + 32768) >> 16));
    px = (uint32_t)R | (uint32_t)G << 8 | (uint32_t)B << 16 | 0xFF000000u;
  }
  *reinterpret_cast<uint32_t*>(out + out_off[img] + (size_t)p * 4) = px;
}

}  // namespace

hipError_t launch_jpeg_reconstruct(const uint8_t* packed, const uint32_t* block_off, const int64_t* pk_off,
                                   const uint16_t* qt, const int64_t* coef_blocks, const int32_t* infos,
                                   const int64_t* out_offsets, int B, int max_blocks, int max_pixels, uint8_t* samples,
                                   uint8_t* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (max_blocks <= 0 || max_pixels <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((max_blocks + 255) / 256, B), dim3(256), 0, s, packed, block_off, pk_off, qt,
                     coef_blocks, infos, samples);
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((max_pixels + 255) / 256, B), dim3(256), 0, s, coef_blocks, infos,
                     samples, out, out_offsets);
  return hipGetLastError();
}
