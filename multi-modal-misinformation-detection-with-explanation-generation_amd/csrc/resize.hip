// Host-input geometry on the device: the two Pillow resamplings the reference's
// preprocessing applies to every decoded image, bit-exact with Pillow's Resample.c:
//   EfficientNet  Resize((224, 224)) on the PIL image = Image.resize((224, 224), BILINEAR)
//                 (misinfo_forensics.py:249-253)
//   CLIP          CLIPImageProcessor: shortest edge -> 224 with BICUBIC, centre crop 224x224
// Pillow's algorithm: per output coordinate xx, center = (xx + 0.5) * scale, support =
// filter_support * max(scale, 1), taps [xmin, xmin + n) with xmin = int(center - support + 0.5)
// clamped, weights filter((x + xmin - center + 0.5) / max(scale, 1)) normalised by their sum, all
// in double, then converted to 22-bit fixed point (round half away from zero); a horizontal pass
// over the rows the vertical pass needs into uint8 (rounded: acc starts at 2^21, clip8 = clamp of
// acc >> 22), then the vertical pass.  A pass whose size is unchanged is skipped (Pillow copies).
// Only the 224 x 224 window that survives the crop is computed; rows and columns are independent,
// so the window's values equal Pillow's.  oracle/pil_resample.py restates the same steps and
// tests pin both against Pillow itself.
// Source pixels are RGB (3 B) or RGBX (4 B: Pillow's in-memory layout, exported zero-copy).
// Kernels: coefficients in fp64 with contraction off (the same IEEE operations in the same order
// as Pillow's C on x86-64), integer MACs for the two passes.
#include "common.h"
#include "kernels.h"

namespace {

#pragma clang fp contract(off)

MMF_DEV double filt_eval(int f, double x) {
  if (x < 0.0) x = -x;
  if (f == 0) return x < 1.0 ? 1.0 - x : 0.0;  // bilinear (triangle), support 1
  const double a = -0.5;                      // bicubic, support 2
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// one thread per (job, axis, window coordinate o): bounds + fixed-point coefficients of output
// coordinate o + crop offset of a resize from in_size to out_size
__global__ __launch_bounds__(256) void resize_coef_kernel(const ResizeJob* __restrict__ jobs, int32_t* __restrict__ coef,
                                                          int32_t* __restrict__ bounds) {
  const ResizeJob& J = jobs[blockIdx.y];
  const int axis = blockIdx.z, o = blockIdx.x * 256 + threadIdx.x;
  if (o >= 224) return;
  const int in_size = axis ? J.h : J.w, out_size = axis ? J.oh : J.ow, ks = axis ? J.ksv : J.ksh;
  const int xx = o + (axis ? J.cy : J.cx);
  const double scale = (double)(float)in_size / out_size;
  const double fs = scale < 1.0 ? 1.0 : scale;
  const double support = (J.filt ? 2.0 : 1.0) * fs;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / fs;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[kResizeKMax];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    w[x] = filt_eval(J.filt, (x + xmin - center + 0.5) * ss);
    ww += w[x];
  }
  int32_t* k = coef + J.coef_off + (size_t)(axis ? 224 * J.ksh : 0) + (size_t)o * ks;
  for (int x = 0; x < ks; ++x) {
    double v = x < xmax ? w[x] : 0.0;
    if (x < xmax && ww != 0.0) v /= ww;
    k[x] = v < 0 ? (int)(-0.5 + v * (1 << 22)) : (int)(0.5 + v * (1 << 22));
  }
  int32_t* b = bounds + ((size_t)blockIdx.y * 2 + axis) * 224 * 2 + o * 2;
  b[0] = xmin;
  b[1] = xmax;
}

MMF_DEV uint8_t clip8(int v) {
  v >>= 22;  // arithmetic: floor
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// horizontal pass: tmp[r][o][c] for source rows y0 + r (r < y1 - y0) and window columns o
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ src, const ResizeJob* __restrict__ jobs,
                                                       const int32_t* __restrict__ coef, const int32_t* __restrict__ bounds,
                                                       uint8_t* __restrict__ tmp) {
  const ResizeJob& J = jobs[blockIdx.y];
  const int rows = J.y1 - J.y0;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * 224) return;
  const int r = idx / 224, o = idx - r * 224;
  const uint8_t* row = src + J.src_off + (size_t)(J.y0 + r) * J.w * J.ps;
  uint8_t* dst = tmp + J.tmp_off + ((size_t)r * 224 + o) * 3;
  if (!J.need_h) {  // unchanged width: Pillow skips the pass (columns map 1:1, crop offset cx)
    dst[0] = row[(o + J.cx) * J.ps];
    dst[1] = row[(o + J.cx) * J.ps + 1];
    dst[2] = row[(o + J.cx) * J.ps + 2];
    return;
  }
  const int32_t* b = bounds + ((size_t)blockIdx.y * 2 + 0) * 224 * 2 + o * 2;
  const int32_t* k = coef + J.coef_off + (size_t)o * J.ksh;
  const int xmin = b[0], n = b[1];
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int x = 0; x < n; ++x) {
    const uint8_t* p = row + (size_t)(xmin + x) * J.ps;
    s0 += p[0] * k[x];
    s1 += p[1] * k[x];
    s2 += p[2] * k[x];
  }
  dst[0] = clip8(s0);
  dst[1] = clip8(s1);
  dst[2] = clip8(s2);
}

// vertical pass: out[oy][ox][c] from tmp rows (bounds shifted by y0)
__global__ __launch_bounds__(256) void resize_v_kernel(const ResizeJob* __restrict__ jobs, const int32_t* __restrict__ coef,
                                                       const int32_t* __restrict__ bounds, const uint8_t* __restrict__ tmp,
                                                       uint8_t* const* __restrict__ outs) {
  const ResizeJob& J = jobs[blockIdx.y];
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= 224 * 224) return;
  const int oy = idx / 224, ox = idx - oy * 224;
  uint8_t* dst = outs[blockIdx.y] + (size_t)idx * 3;
  const uint8_t* t = tmp + J.tmp_off;
  if (!J.need_v) {  // unchanged height: window rows are tmp rows cy - y0 + oy
    const uint8_t* p = t + ((size_t)(oy + J.cy - J.y0) * 224 + ox) * 3;
    dst[0] = p[0];
    dst[1] = p[1];
    dst[2] = p[2];
    return;
  }
  const int32_t* b = bounds + ((size_t)blockIdx.y * 2 + 1) * 224 * 2 + oy * 2;
  const int32_t* k = coef + J.coef_off + (size_t)224 * J.ksh + (size_t)oy * J.ksv;
  const int ymin = b[0] - J.y0, n = b[1];
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int y = 0; y < n; ++y) {
    const uint8_t* p = t + ((size_t)(ymin + y) * 224 + ox) * 3;
    s0 += p[0] * k[y];
    s1 += p[1] * k[y];
    s2 += p[2] * k[y];
  }
  dst[0] = clip8(s0);
  dst[1] = clip8(s1);
  dst[2] = clip8(s2);
}

}  // namespace

hipError_t launch_resize_pil(const uint8_t* src, const ResizeJob* jobs, int njobs, int max_rows, int32_t* coef,
                             int32_t* bounds, uint8_t* tmp, uint8_t* const* outs, hipStream_t s) {
  if (njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(resize_coef_kernel, dim3(1, njobs, 2), dim3(256), 0, s, jobs, coef, bounds);
  hipLaunchKernelGGL(resize_h_kernel, dim3((max_rows * 224 + 255) / 256, njobs), dim3(256), 0, s, src, jobs, coef,
                     bounds, tmp);
  hipLaunchKernelGGL(resize_v_kernel, dim3((224 * 224 + 255) / 256, njobs), dim3(256), 0, s, jobs, coef, bounds, tmp,
                     outs);
  return hipGetLastError();
}
