// Row-wise kernels: LayerNorm, embeddings (+LN), CLIP patch im2col, EOS pooling, L2 norm.
// One 64-lane wave per row of width C in {512, 768}: every lane holds C/256 float4 in registers,
// so a row is read once, reduced with DPP/shuffle trees and written once (fp32 residual stream
// and/or fp16 GEMM operand).  Variance is the two-pass mean((x-mean)^2) in fp32 like torch.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

template <int NV>
MMF_DEV bool ln_row(float4 (&v)[NV], const float* g, const float* b, float eps, int C, int lane) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
    q += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    const float4 gg = *reinterpret_cast<const float4*>(g + c);
    const float4 bb = *reinterpret_cast<const float4*>(b + c);
    v[i].x = v[i].x * rstd * gg.x + bb.x;
    v[i].y = v[i].y * rstd * gg.y + bb.y;
    v[i].z = v[i].z * rstd * gg.z + bb.z;
    v[i].w = v[i].w * rstd * gg.w + bb.w;
  }
  // the row's statistics are finite iff every input was (an inf or NaN makes the mean or the
  // variance non-finite): wave-uniform
  return __builtin_isfinite(mean) && __builtin_isfinite(rstd);
}

template <int NV>
MMF_DEV void load_row(float4 (&v)[NV], const float* x, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(x + (i * 64 + lane) * 4);
}
template <int NV>
MMF_DEV void add_row(float4 (&v)[NV], const float* x, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 a = *reinterpret_cast<const float4*>(x + (i * 64 + lane) * 4);
    v[i].x += a.x; v[i].y += a.y; v[i].z += a.z; v[i].w += a.w;
  }
}
template <int NV>
MMF_DEV void store_row(const float4 (&v)[NV], float* y32, f16_t* y16, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (y32) *reinterpret_cast<float4*>(y32 + c) = v[i];
    if (y16) *reinterpret_cast<uint2*>(y16 + c) = make_uint2(pack2h(v[i].x, v[i].y), pack2h(v[i].z, v[i].w));
  }
}

// CLIP residual-stream rows: fp32, or fp16 (option clip_res16)
template <int NV, typename XT>
MMF_DEV void load_x(float4 (&v)[NV], const XT* x, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if constexpr (std::is_same_v<XT, float>) {
      v[i] = *reinterpret_cast<const float4*>(x + c);
    } else {
      const uint2 a = *reinterpret_cast<const uint2*>(x + c);
      v[i] = make_float4(lo_h(a.x), hi_h(a.x), lo_h(a.y), hi_h(a.y));
    }
  }
}
// stores v as XT and leaves v holding the stored (rounded) values
template <int NV, typename XT>
MMF_DEV void store_x(float4 (&v)[NV], XT* x, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if constexpr (std::is_same_v<XT, float>) {
      *reinterpret_cast<float4*>(x + c) = v[i];
    } else {
      const uint2 h = make_uint2(pack2h(v[i].x, v[i].y), pack2h(v[i].z, v[i].w));
      *reinterpret_cast<uint2*>(x + c) = h;
      v[i] = make_float4(lo_h(h.x), hi_h(h.x), lo_h(h.y), hi_h(h.y));
    }
  }
}

// (mean, M2) of a row held by one wave -- the single lazy-LN partial (P = 1, tn = C) of a row
// whose LayerNorm the next GEMM folds (gemm.hip)
template <int NV>
MMF_DEV float2 row_partial(const float4 (&v)[NV], int C) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q += (a * a + b * b) + (c * c + d * d);
  }
  return make_float2(mean, wave_sum(q));
}

template <int NV>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int ldx, const float* add, int ldadd,
                                                        const float* g, const float* b, float eps, float* y32,
                                                        int ldy32, f16_t* y16, int ldy16, int rows) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float4 v[NV];
  load_row<NV>(v, x + (size_t)row * ldx, lane);
  if (add) add_row<NV>(v, add + (size_t)row * ldadd, lane);
  ln_row<NV>(v, g, b, eps, NV * 256, lane);
  store_row<NV>(v, y32 ? y32 + (size_t)row * ldy32 : nullptr, y16 ? y16 + (size_t)row * ldy16 : nullptr, lane);
}

// RoBERTa precise mode (precise.hip / capi.cpp run_text_precise): x = LN(x + add) in place (fp32 stream)
// and the next GEMM's K-concatenated operand rows s3 = [hi | lo | hi] of the result (LO = false: hi
// alone, for a consumer on fp16 operands) -- the LayerNorm and the split3 pass in one
template <int NV, bool LO>
__global__ __launch_bounds__(256) void layernorm_split3_kernel(float* x, const float* add, const float* g,
                                                               const float* b, float eps, f16_t* s3, int rows) {
  constexpr int C = NV * 256;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float4 v[NV];
  load_row<NV>(v, x + (size_t)row * C, lane);
  add_row<NV>(v, add + (size_t)row * C, lane);
  ln_row<NV>(v, g, b, eps, C, lane);
  store_row<NV>(v, x + (size_t)row * C, nullptr, lane);
  f16_t* o = s3 + (size_t)row * 3 * C;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    const uint2 hi = make_uint2(pack2h(v[i].x, v[i].y), pack2h(v[i].z, v[i].w));
    *reinterpret_cast<uint2*>(o + c) = hi;
    if constexpr (LO) {
      *reinterpret_cast<uint2*>(o + C + c) = make_uint2(pack2h(v[i].x - lo_h(hi.x), v[i].y - hi_h(hi.x)),
                                                        pack2h(v[i].z - lo_h(hi.y), v[i].w - hi_h(hi.y)));
      *reinterpret_cast<uint2*>(o + 2 * C + c) = hi;
    }
  }
}

// Residual add + LayerNorm after an out-projection / FFN-2 GEMM whose fp16 output y is the
// residual branch: s = x + y in fp32 (x = fp32 residual stream), then
//   pre-LN (CLIP, TF clip:357-385):   s32 = s (the new residual stream), o16 = LN(s)
//   post-LN (RoBERTa, TF roberta:329-399): o32 = LN(s) (the new residual stream), o16 = LN(s)
// s32 / o32 may alias x (each wave reads its whole row before writing it).
// XT = f16_t: the CLIP residual stream held in fp16 (x and s32 fp16; o32 unused)
template <int NV, typename XT>
__global__ __launch_bounds__(256) void add_ln_kernel(const XT* x, int ldx, const f16_t* y, int ldy, const float* g,
                                                     const float* b, float eps, XT* s32, float* o32,
                                                     f16_t* o16, int ldo, int rows) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float4 v[NV];
  uint2 a[NV];
  const f16_t* yr = y + (size_t)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) a[i] = *reinterpret_cast<const uint2*>(yr + (i * 64 + lane) * 4);
  load_x<NV>(v, x + (size_t)row * ldx, lane);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i].x += lo_h(a[i].x); v[i].y += hi_h(a[i].x); v[i].z += lo_h(a[i].y); v[i].w += hi_h(a[i].y);
  }
  if (s32) store_x<NV>(v, s32 + (size_t)row * ldx, lane);
  ln_row<NV>(v, g, b, eps, NV * 256, lane);
  store_row<NV>(v, o32 ? o32 + (size_t)row * ldx : nullptr, o16 + (size_t)row * ldo, lane);
}

// RoBERTa's post-LN residual stream in split precision: x = hi + lo with hi = fp16(x) (the very
// tensor the next GEMM reads) and lo = fp16(x - hi) (|lo| <= 2^-11 |x|; ~22 significant bits for
// |x| >~ 0.03, vs 24 for fp32).  4 bytes per element like fp32, but hi doubles as the GEMM operand,
// so add+LN writes 4 instead of 6 bytes per element (12 -> 10 B/elem of HBM traffic).

template <int NV>
MMF_DEV void store_row_hilo(const float4 (&v)[NV], f16_t* hi, uint16_t* lo, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    const uint2 h = make_uint2(pack2h(v[i].x, v[i].y), pack2h(v[i].z, v[i].w));
    *reinterpret_cast<uint2*>(hi + c) = h;
    if (lo)  // lo = null: fp16-only stream (option text_hilo = 0)
      *reinterpret_cast<uint2*>(lo + c) = make_uint2(pack2h(v[i].x - lo_h(h.x), v[i].y - hi_h(h.x)),
                                                   pack2h(v[i].z - lo_h(h.y), v[i].w - hi_h(h.y)));
  }
}

// post-LN add+LayerNorm on the split stream: s = (hi + lo) + y; (hi, lo) = split(LN(s)), in place
// HILO = false: the stream is hi alone (fp16; option text_hilo = 0)
template <int NV, bool HILO>
__global__ __launch_bounds__(256) void add_ln_hilo_kernel(f16_t* hi, uint16_t* lo, int ld, const f16_t* y, int ldy,
                                                          const float* g, const float* b, float eps, int rows,
                                                          int* ovf, int L) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float4 v[NV];
  uint2 xh[NV], xl[NV], a[NV];
  f16_t* hr = hi + (size_t)row * ld;
  uint16_t* lr = lo + (size_t)row * ld;
  const f16_t* yr = y + (size_t)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    xh[i] = *reinterpret_cast<const uint2*>(hr + c);
    xl[i] = HILO ? *reinterpret_cast<const uint2*>(lr + c) : make_uint2(0, 0);
    a[i] = *reinterpret_cast<const uint2*>(yr + c);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i].x = (lo_h(xh[i].x) + lo_h(xl[i].x)) + lo_h(a[i].x);
    v[i].y = (hi_h(xh[i].x) + hi_h(xl[i].x)) + hi_h(a[i].x);
    v[i].z = (lo_h(xh[i].y) + lo_h(xl[i].y)) + lo_h(a[i].y);
    v[i].w = (hi_h(xh[i].y) + hi_h(xl[i].y)) + hi_h(a[i].y);
  }
  // overflow sentinel (ovf, per sequence of L rows): an fp16 branch output or stream row that
  // left fp16's range makes this row's statistics non-finite -- flagged, so that the text heads
  // return NaN scores for the sequence (the attention's masked softmax would otherwise hide a
  // non-finite key row behind finite outputs) and the API's run-time trap sees it
  if (!ln_row<NV>(v, g, b, eps, NV * 256, lane) && ovf && lane == 0) ovf[row / L] = 1;
  store_row_hilo<NV>(v, hr, HILO ? lr : nullptr, lane);
}

// fp32 rows (hi + lo) of the split stream, gathered with a row stride (the last layer's CLS rows)
__global__ __launch_bounds__(256) void hilo_rows_kernel(const f16_t* hi, const uint16_t* lo, int row_stride,
                                                        float* out, int B, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const f16_t* hr = hi + (size_t)row * row_stride;
  const uint16_t* lr = lo ? lo + (size_t)row * row_stride : nullptr;
  for (int c = lane * 4; c < C; c += 256) {
    const uint2 h = *reinterpret_cast<const uint2*>(hr + c);
    const uint2 l = lr ? *reinterpret_cast<const uint2*>(lr + c) : make_uint2(0, 0);
    *reinterpret_cast<float4*>(out + (size_t)row * C + c) =
        make_float4(lo_h(h.x) + lo_h(l.x), hi_h(h.x) + hi_h(l.x), lo_h(h.y) + lo_h(l.y), hi_h(h.y) + hi_h(l.y));
  }
}

// RoBERTa: position ids = cumsum(ids != pad) * (ids != pad) + pad (TF roberta:142-155);
// x = LN(word[id] + type[0] + pos[pid]).  One block per sequence.
template <int NV>
__global__ __launch_bounds__(256) void roberta_embed_kernel(const int32_t* ids, const float* word, const float* pos,
                                                            const float* type0, const float* g, const float* b,
                                                            float eps, uint16_t* xlo, f16_t* xb, float* x32, int L,
                                                            int pad, int* ovf) {
  __shared__ int s_ids[512];
  __shared__ int s_pos[512];
  const int bi = blockIdx.x, tid = threadIdx.x;
  for (int t = tid; t < L; t += 256) s_ids[t] = ids[(size_t)bi * L + t];
  __syncthreads();
  if (tid < 64) {  // wave-level inclusive scan of the non-pad flags, 64 positions per step
    int carry = 0;
    for (int base = 0; base < L; base += 64) {
      const int t = base + tid;
      int f = (t < L && s_ids[t] != pad) ? 1 : 0;
      int v = f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int n = __shfl_up(v, o, 64);
        if (tid >= o) v += n;
      }
      if (t < L) s_pos[t] = f ? (carry + v + pad) : pad;
      carry += __shfl(v, 63, 64);
    }
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int C = NV * 256;
  // blockIdx.y splits the sequence's rows over gridDim.y workgroups (each redoes the cheap scan)
  for (int t = blockIdx.y * 4 + wave; t < L; t += 4 * gridDim.y) {
    float4 v[NV];
    load_row<NV>(v, word + (size_t)s_ids[t] * C, lane);
    add_row<NV>(v, type0, lane);
    add_row<NV>(v, pos + (size_t)s_pos[t] * C, lane);
    const size_t r = (size_t)bi * L + t;
    if (!ln_row<NV>(v, g, b, eps, C, lane) && ovf && lane == 0) ovf[bi] = 1;
    if (x32) store_row<NV>(v, x32 + r * C, nullptr, lane);  // precise mode: the fp32 stream
    else store_row_hilo<NV>(v, xb + r * C, xlo ? xlo + r * C : nullptr, lane);
  }
}

// CLIP text: x = tok[id] + pos[t] (residual stream, fp32 or fp16); xb = LN1_layer0(x) (fp16)
template <int NV, typename XT>
__global__ __launch_bounds__(256) void clip_text_embed_kernel(const int32_t* ids, const float* tok, const float* pos,
                                                              const float* g, const float* b, float eps, XT* x,
                                                              f16_t* xb, float2* st, int rows, int L) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  constexpr int C = NV * 256;
  const int t = row % L;
  float4 v[NV];
  load_row<NV>(v, tok + (size_t)ids[row] * C, lane);
  add_row<NV>(v, pos + (size_t)t * C, lane);
  store_x<NV>(v, x + (size_t)row * C, lane);  // rounds v to XT: LN1 sees the stored stream
  if (st) {  // lazy LN: statistics of the stored stream (layer 0's QKV folds LN1)
    const float2 pm = row_partial<NV>(v, C);
    if (lane == 0) st[row] = pm;
    return;
  }
  ln_row<NV>(v, g, b, eps, C, lane);
  store_row<NV>(v, nullptr, xb + (size_t)row * C, lane);
}

// CLIP patch embedding operand: A[b*49 + p][c*1024 + ky*32 + kx] = (img/255 - mean_c)/std_c.
// One thread per (patch row, ky, 8-pixel group): the 24 interleaved RGB bytes arrive as three
// 8-B loads (was 8 single-byte loads per channel) and leave as one 16-B store per channel.
__global__ __launch_bounds__(256) void clip_im2col_kernel(const uint8_t* img, f16_t* A, int B) {
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)B * 49 * 128;
  if (gid >= total) return;
  const int g = gid % 128;
  const size_t rowp = gid / 128;
  const int p = rowp % 49, bi = rowp / 49;
  const int ky = g >> 2, kx0 = (g & 3) * 8;
  const int y = (p / 7) * 32 + ky, x0 = (p % 7) * 32 + kx0;
  const uint2* src = reinterpret_cast<const uint2*>(img + (((size_t)bi * 224 + y) * 224 + x0) * 3);  // 8-B aligned
  const uint2 w0 = src[0], w1 = src[1], w2 = src[2];
  const uint32_t wd[6] = {w0.x, w0.y, w1.x, w1.y, w2.x, w2.y};
  constexpr float kMean[3] = {0.48145466f, 0.4578275f, 0.40821073f};
  constexpr float kStd[3] = {0.26862954f, 0.26130258f, 0.27577711f};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float mean = kMean[c], istd = 1.0f / kStd[c];
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int byte = j * 3 + c;
      v[j] = ((float)((wd[byte >> 2] >> ((byte & 3) * 8)) & 0xffu) * (1.0f / 255.0f) - mean) * istd;
    }
    *reinterpret_cast<uint4*>(A + rowp * 3072 + c * 1024 + ky * 32 + kx0) =
        make_uint4(pack2h(v[0], v[1]), pack2h(v[2], v[3]), pack2h(v[4], v[5]), pack2h(v[6], v[7]));
  }
}

// CLIP vision: e = (t==0 ? class_emb : patch[b*49+t-1]) + pos[t]; x = pre_LN(e); xb = LN1(x)
template <typename XT>
__global__ __launch_bounds__(256) void clip_vision_assemble_kernel(const float* patches, const float* cls,
                                                                   const float* pos, const float* pg,
                                                                   const float* pb, const float* g1,
                                                                   const float* b1, float eps, XT* x,
                                                                   f16_t* xb, float2* st, int rows) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  constexpr int NV = 3, C = 768;
  const int t = row % 50, bi = row / 50;
  float4 v[NV];
  if (t == 0) load_row<NV>(v, cls, lane);
  else load_row<NV>(v, patches + ((size_t)bi * 49 + t - 1) * C, lane);
  add_row<NV>(v, pos + (size_t)t * C, lane);
  ln_row<NV>(v, pg, pb, eps, C, lane);
  store_x<NV>(v, x + (size_t)row * C, lane);  // rounds v to XT: LN1 sees the stored stream
  if (st) {
    const float2 pm = row_partial<NV>(v, C);
    if (lane == 0) st[row] = pm;
    return;
  }
  ln_row<NV>(v, g1, b1, eps, C, lane);
  store_row<NV>(v, nullptr, xb + (size_t)row * C, lane);
}

// EOS pooling index per sequence (TF clip:561-582): one wave per row, lanes stride the positions,
// one wave reduction (the sequential per-thread scan took ~21 us at B = 256 on one workgroup).
__global__ __launch_bounds__(256) void eos_index_kernel(const int32_t* ids, int32_t* out, int B, int L, int eos) {
  const int bi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (bi >= B) return;
  const int32_t* r = ids + (size_t)bi * L;
  int key = eos == 2 ? -1 : 0x7fffffff;
  for (int t = lane; t < L; t += 64) {
    const int v = r[t];
    if (eos == 2) key = max(key, v * 1024 + (1023 - t));  // argmax(ids), first maximal position (L <= 1024)
    else if (v == eos) key = min(key, t);                  // first EOS position
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int k2 = __shfl_xor(key, o, 64);
    key = eos == 2 ? max(key, k2) : min(key, k2);
  }
  if (lane == 0) out[bi] = eos == 2 ? 1023 - (key & 1023) : (key == 0x7fffffff ? 0 : key);
}

template <int NV>
__global__ __launch_bounds__(256) void gather_ln_kernel(const float* x, const int32_t* idx, int L, const float* g,
                                                        const float* b, float eps, f16_t* out, float* out32,
                                                        int B) {
  const int bi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (bi >= B) return;
  constexpr int C = NV * 256;
  const size_t row = (size_t)bi * L + (idx ? idx[bi] : 0);
  float4 v[NV];
  load_row<NV>(v, x + row * C, lane);
  ln_row<NV>(v, g, b, eps, C, lane);
  store_row<NV>(v, out32 ? out32 + (size_t)bi * C : nullptr, out ? out + (size_t)bi * C : nullptr, lane);
}

// rows b*L + (idx ? idx[b] : 0) of a fp16 [.,C] and an fp32 (or fp16: XT) [.,C] buffer -> compact
// [B,C] copies (o32 always fp32)
template <typename XT>
__global__ __launch_bounds__(256) void gather_rows2_kernel(const f16_t* a16, const XT* a32, const int32_t* idx,
                                                           int L, int C, f16_t* o16, float* o32, int B) {
  const int bi = blockIdx.x;
  if (bi >= B) return;
  const size_t row = (size_t)bi * L + (idx ? idx[bi] : 0);
  for (int c = threadIdx.x * 4; c < C; c += 256 * 4) {
    if (a16) *reinterpret_cast<uint2*>(o16 + (size_t)bi * C + c) = *reinterpret_cast<const uint2*>(a16 + row * C + c);
    if constexpr (std::is_same_v<XT, float>) {
      *reinterpret_cast<float4*>(o32 + (size_t)bi * C + c) = *reinterpret_cast<const float4*>(a32 + row * C + c);
    } else {
      const uint2 a = *reinterpret_cast<const uint2*>(a32 + row * C + c);
      *reinterpret_cast<float4*>(o32 + (size_t)bi * C + c) = make_float4(lo_h(a.x), hi_h(a.x), lo_h(a.y), hi_h(a.y));
    }
  }
}

__global__ __launch_bounds__(256) void l2norm_kernel(float* x, int B, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  float* r = x + (size_t)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += r[c] * r[c];
  const float inv = 1.0f / sqrtf(wave_sum(s));
  for (int c = lane; c < C; c += 64) r[c] *= inv;
}

}  // namespace

hipError_t launch_layernorm_split3(float* x, const float* add, const float* g, const float* b, float eps, f16_t* s3,
                                   int with_lo, int rows, int C, hipStream_t s) {
  if (C != 768) return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4);
  if (with_lo) hipLaunchKernelGGL((layernorm_split3_kernel<3, true>), grid, dim3(256), 0, s, x, add, g, b, eps, s3, rows);
  else hipLaunchKernelGGL((layernorm_split3_kernel<3, false>), grid, dim3(256), 0, s, x, add, g, b, eps, s3, rows);
  return hipGetLastError();
}

hipError_t launch_layernorm(const float* x, int ldx, const float* add, int ldadd, const float* g, const float* b,
                            float eps, float* y32, int ldy32, f16_t* y16, int ldy16, int rows, int C,
                            hipStream_t s) {
  const dim3 grid((rows + 3) / 4);
  if (C == 768)
    hipLaunchKernelGGL(layernorm_kernel<3>, grid, dim3(256), 0, s, x, ldx, add, ldadd, g, b, eps, y32, ldy32, y16,
                       ldy16, rows);
  else if (C == 512)
    hipLaunchKernelGGL(layernorm_kernel<2>, grid, dim3(256), 0, s, x, ldx, add, ldadd, g, b, eps, y32, ldy32, y16,
                       ldy16, rows);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

namespace {
template <typename XT>
hipError_t add_ln_any(const XT* x, int ldx, const f16_t* y, int ldy, const float* g, const float* b, float eps, XT* s32,
                      float* o32, f16_t* o16, int ldo, int rows, int C, hipStream_t s) {
  const dim3 grid((rows + 3) / 4);
  if (!o16) return hipErrorInvalidValue;
  if (C == 768)
    hipLaunchKernelGGL((add_ln_kernel<3, XT>), grid, dim3(256), 0, s, x, ldx, y, ldy, g, b, eps, s32, o32, o16, ldo,
                       rows);
  else if (C == 512)
    hipLaunchKernelGGL((add_ln_kernel<2, XT>), grid, dim3(256), 0, s, x, ldx, y, ldy, g, b, eps, s32, o32, o16, ldo,
                       rows);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
}  // namespace

hipError_t launch_add_ln(const float* x, int ldx, const f16_t* y, int ldy, const float* g, const float* b, float eps,
                         float* s32, float* o32, f16_t* o16, int ldo, int rows, int C, hipStream_t s) {
  return add_ln_any(x, ldx, y, ldy, g, b, eps, s32, o32, o16, ldo, rows, C, s);
}

hipError_t launch_add_ln(const f16_t* x, int ldx, const f16_t* y, int ldy, const float* g, const float* b, float eps,
                         f16_t* s16, f16_t* o16, int ldo, int rows, int C, hipStream_t s) {
  return add_ln_any(x, ldx, y, ldy, g, b, eps, s16, nullptr, o16, ldo, rows, C, s);
}

hipError_t launch_roberta_embed(const int32_t* ids, const float* word, const float* pos, const float* type0,
                                const float* g, const float* b, float eps, uint16_t* xlo, f16_t* xb, int B, int L,
                                int H, int pad_id, hipStream_t s, float* x32, int* ovf) {
  if (H != 768 || L > 512) return hipErrorInvalidValue;
  // 4 workgroups per sequence: one per sequence left the chip at 256 workgroups (~77 us at B = 256)
  hipLaunchKernelGGL(roberta_embed_kernel<3>, dim3(B, 4), dim3(256), 0, s, ids, word, pos, type0, g, b, eps, xlo, xb, x32,
                     L, pad_id, ovf);
  return hipGetLastError();
}

hipError_t launch_clip_text_embed(const int32_t* ids, const float* tok, const float* pos, const float* g,
                                  const float* b, float eps, float* x, f16_t* x16, f16_t* xb, float2* st, int B, int L,
                                  int H, hipStream_t s) {
  if (H != 512 || !x == !x16) return hipErrorInvalidValue;
  const int rows = B * L;
  if (x)
    hipLaunchKernelGGL((clip_text_embed_kernel<2, float>), dim3((rows + 3) / 4), dim3(256), 0, s, ids, tok, pos, g, b,
                       eps, x, xb, st, rows, L);
  else
    hipLaunchKernelGGL((clip_text_embed_kernel<2, f16_t>), dim3((rows + 3) / 4), dim3(256), 0, s, ids, tok, pos, g, b,
                       eps, x16, xb, st, rows, L);
  return hipGetLastError();
}

hipError_t launch_clip_im2col(const uint8_t* img, f16_t* A, int B, hipStream_t s) {
  if (reinterpret_cast<uintptr_t>(img) & 7) return hipErrorInvalidValue;  // 8-B pixel-row loads
  const size_t total = (size_t)B * 49 * 128;
  hipLaunchKernelGGL(clip_im2col_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, img, A, B);
  return hipGetLastError();
}

hipError_t launch_clip_vision_assemble(const float* patches, const float* cls, const float* pos,
                                       const float* pre_g, const float* pre_b, const float* ln1_g,
                                       const float* ln1_b, float eps, float* x, f16_t* x16, f16_t* xb, float2* st,
                                       int B, hipStream_t s) {
  if (!x == !x16) return hipErrorInvalidValue;
  const int rows = B * 50;
  if (x)
    hipLaunchKernelGGL(clip_vision_assemble_kernel<float>, dim3((rows + 3) / 4), dim3(256), 0, s, patches, cls, pos,
                       pre_g, pre_b, ln1_g, ln1_b, eps, x, xb, st, rows);
  else
    hipLaunchKernelGGL(clip_vision_assemble_kernel<f16_t>, dim3((rows + 3) / 4), dim3(256), 0, s, patches, cls, pos,
                       pre_g, pre_b, ln1_g, ln1_b, eps, x16, xb, st, rows);
  return hipGetLastError();
}

hipError_t launch_eos_index(const int32_t* ids, int32_t* out, int B, int L, int eos_id, hipStream_t s) {
  if (L > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(eos_index_kernel, dim3((B + 3) / 4), dim3(256), 0, s, ids, out, B, L, eos_id);
  return hipGetLastError();
}

hipError_t launch_gather_ln(const float* x, const int32_t* idx, int L, const float* g, const float* b, float eps,
                            f16_t* out, float* out32, int B, int C, hipStream_t s) {
  const dim3 grid((B + 3) / 4);
  if (C == 768)
    hipLaunchKernelGGL(gather_ln_kernel<3>, grid, dim3(256), 0, s, x, idx, L, g, b, eps, out, out32, B);
  else if (C == 512)
    hipLaunchKernelGGL(gather_ln_kernel<2>, grid, dim3(256), 0, s, x, idx, L, g, b, eps, out, out32, B);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_gather_rows2(const f16_t* a16, const float* a32, const f16_t* a32h, const int32_t* idx, int L,
                               int C, f16_t* o16, float* o32, int B, hipStream_t s) {
  if ((C & 3) || !a32 == !a32h) return hipErrorInvalidValue;
  if (a32)
    hipLaunchKernelGGL(gather_rows2_kernel<float>, dim3(B), dim3(256), 0, s, a16, a32, idx, L, C, o16, o32, B);
  else
    hipLaunchKernelGGL(gather_rows2_kernel<f16_t>, dim3(B), dim3(256), 0, s, a16, a32h, idx, L, C, o16, o32, B);
  return hipGetLastError();
}

hipError_t launch_l2norm(float* x, int B, int C, hipStream_t s) {
  hipLaunchKernelGGL(l2norm_kernel, dim3((B + 3) / 4), dim3(256), 0, s, x, B, C);
  return hipGetLastError();
}

hipError_t launch_add_ln_hilo(f16_t* hi, uint16_t* lo, int ld, const f16_t* y, int ldy, const float* g,
                              const float* b, float eps, int rows, int C, hipStream_t s, int* ovf, int L) {
  if (C != 768 || (ld & 3) || (ldy & 3) || (ovf && L <= 0)) return hipErrorInvalidValue;
  if (lo)
    hipLaunchKernelGGL((add_ln_hilo_kernel<3, true>), dim3((rows + 3) / 4), dim3(256), 0, s, hi, lo, ld, y, ldy, g, b, eps,
                       rows, ovf, L);
  else
    hipLaunchKernelGGL((add_ln_hilo_kernel<3, false>), dim3((rows + 3) / 4), dim3(256), 0, s, hi, lo, ld, y, ldy, g, b,
                       eps, rows, ovf, L);
  return hipGetLastError();
}

hipError_t launch_hilo_rows(const f16_t* hi, const uint16_t* lo, int row_stride, float* out, int B, int C,
                            hipStream_t s) {
  if ((C & 3) || (row_stride & 3)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(hilo_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, s, hi, lo, row_stride, out, B, C);
  return hipGetLastError();
}
