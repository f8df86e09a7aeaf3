// EfficientNet-B0 (torchvision spec, eval) pieces that are not 1x1 convolutions.  Activations are
// NHWC fp16 so channels are the contiguous, coalesced axis; every BatchNorm is folded into the
// preceding convolution's weights/bias at load time (mmf_finalize).  These kernels are HBM-bound
// (SURVEY.md §8d): each reads its input once and writes its output once.
//   stem      uint8 HWC -> ImageNet normalise -> conv3x3 s2 (3->32) + BN + SiLU
//   dwconv    depthwise kxk (k=3,5; s=1,2) + BN + SiLU, with the SE global-average-pool partial
//             sums of the fp32 outputs (deterministic per-chunk partials, no atomics)
//   se        mean -> fc1 + SiLU -> fc2 + sigmoid -> per-(image, channel) scale (applied inside
//             the project GEMM's A load)
//   gap_cls   global average pool of the head conv + Linear(1280, 2) + softmax[:, 1]
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

// per-image base pointer (workgroup-uniform -> SGPRs) + 32-bit byte offset: global loads / stores
// use the saddr + 32-bit voffset form instead of per-lane 64-bit address arithmetic
template <typename T>
MMF_DEV T* at_bytes(T* base, uint32_t byte_off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(const_cast<typename std::remove_const<T>::type*>(base)) + byte_off);
}

// Diagnostic build only (-DMMF_EFF_STAMP, tools/effnet_stamps.py): per-block phase stamps of the
// depthwise / fused-front kernels into a buffer of their own (slots [region][block][32]: 0 / 1 =
// s_memrealtime at start / end, 2.. = s_memtime after each phase, 31 = the number of stamps).  In
// the production build every EST_* macro is empty.
#ifdef MMF_EFF_STAMP
constexpr int kStampBlocks = 16384, kStampSlots = 32;
__device__ unsigned long long* g_eff_stamp;
MMF_DEV unsigned long long est_time() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define EST_BEGIN(REGION)                                                                                   \
  unsigned long long* est_ = nullptr;                                                                        \
  int est_n_ = 2;                                                                                            \
  {                                                                                                          \
    const unsigned est_b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                   \
    if (g_eff_stamp && est_b < (unsigned)kStampBlocks)                                                       \
      est_ = g_eff_stamp + ((size_t)(REGION) * kStampBlocks + est_b) * kStampSlots;                         \
    const unsigned long long est_r = __builtin_amdgcn_s_memrealtime();                                       \
    const unsigned long long est_t = est_time();                                                             \
    if (est_ && threadIdx.x == 0) { est_[0] = est_r; est_[2] = est_t; }                                      \
  }
#define EST()                                                                                                \
  {                                                                                                          \
    const unsigned long long est_t = est_time();                                                             \
    ++est_n_;                                                                                                \
    if (est_ && threadIdx.x == 0 && est_n_ < kStampSlots - 1) est_[est_n_] = est_t;                          \
  }
#define EST_END()                                                                                            \
  {                                                                                                          \
    const unsigned long long est_r = __builtin_amdgcn_s_memrealtime();                                       \
    if (est_ && threadIdx.x == 0) { est_[1] = est_r; est_[kStampSlots - 1] = (unsigned long long)est_n_; }   \
  }
#else
#define EST_BEGIN(REGION)
#define EST()
#define EST_END()
#endif

// One thread per output pixel, all 32 channels; weights transposed in LDS to [tap][channel] so
// every tap is 8 broadcast float4 reads.  ToTensor + Normalize folded into one FMA per input.
// F32 = true: input is an already-normalised fp32 NCHW tensor (detector.forward_image signature,
// misinfo_forensics.py:102-104) instead of uint8 HWC pixels.  OT = float: fp32 output for the
// fp32 tower (option effnet_fp32, effnet_f32.hip).
__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

template <bool F32, typename OT = f16_t>
__global__ __launch_bounds__(256) void stem_kernel(const void* src, const float* w, const float* bias, OT* out,
                                                   int B) {
  const uint8_t* img = (const uint8_t*)src;
  const float* xf = (const float*)src;
  __shared__ __attribute__((aligned(16))) float sw[27 * 32];
  __shared__ __attribute__((aligned(16))) float sb[32];
  for (int i = threadIdx.x; i < 32 * 27; i += 256) sw[(i % 27) * 32 + i / 27] = w[i];
  if (threadIdx.x < 32) sb[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  const size_t pix = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (size_t)B * 112 * 112) return;
  const int ox = pix % 112, oy = (pix / 112) % 112, bi = pix / (112 * 112);
  // (u/255 - mean)/std == u * (1/(255 std)) + (-mean/std)
  const float sc[3] = {1.0f / (255.0f * 0.229f), 1.0f / (255.0f * 0.224f), 1.0f / (255.0f * 0.225f)};
  const float of[3] = {-0.485f / 0.229f, -0.456f / 0.224f, -0.406f / 0.225f};
  float acc[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) acc[j] = sb[j];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * 2 - 1 + ky;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * 2 - 1 + kx;
      if (iy < 0 || iy >= 224 || ix < 0 || ix >= 224) continue;  // zero padding (normalised space)
      const uint8_t* p = img + (((size_t)bi * 224 + iy) * 224 + ix) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        // fp32 tower: ToTensor / Normalize evaluated as torchvision does ((u / 255 - mean) / std)
        const float v = F32 ? xf[(((size_t)bi * 3 + c) * 224 + iy) * 224 + ix]
                        : sizeof(OT) == 4 ? ((float)p[c] / 255.0f - kMean[c]) / kStd[c]
                                          : fmaf((float)p[c], sc[c], of[c]);
        const float4* wr = reinterpret_cast<const float4*>(sw + (c * 9 + ky * 3 + kx) * 32);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 ww = wr[q];
          acc[q * 4 + 0] = fmaf(ww.x, v, acc[q * 4 + 0]);
          acc[q * 4 + 1] = fmaf(ww.y, v, acc[q * 4 + 1]);
          acc[q * 4 + 2] = fmaf(ww.z, v, acc[q * 4 + 2]);
          acc[q * 4 + 3] = fmaf(ww.w, v, acc[q * 4 + 3]);
        }
      }
    }
  }
  if constexpr (sizeof(OT) == 4) {
    float4* dst = reinterpret_cast<float4*>(out + pix * 32);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      dst[q] = make_float4(silu_precise(acc[q * 4]), silu_precise(acc[q * 4 + 1]), silu_precise(acc[q * 4 + 2]),
                           silu_precise(acc[q * 4 + 3]));
    return;
  }
  uint4* dst = reinterpret_cast<uint4*>(out + pix * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_apply(acc[q * 8 + j], ACT_SILU);
    dst[q] = make_uint4(pack2h(o[0], o[1]), pack2h(o[2], o[3]), pack2h(o[4], o[5]), pack2h(o[6], o[7]));
  }
}

// Depthwise kxk + BN + SiLU + SE pool partial from an LDS input tile [IT][IT][CW] (zero padding
// already materialised): thread (px, g) computes output pixels px, px + PX, ... of channel group g,
// so the pool partial of a channel stays in one thread and is reduced across px in a fixed order
// (deterministic, no atomics): one partial per (image, tile, channel).
template <int K, int S>
MMF_DEV void dw_compute(const f16_t* tile, const float* sw, const float* sb, float* red, f16_t* __restrict__ out,
                        float* __restrict__ pool_part, int bi, int c0, int oy0, int ox0, int Ho, int Wo, int C,
                        int CW, int T, int IT) {
  const int tid = threadIdx.x, NG = CW / 8;
  const int PX = 256 / NG;
  const int g = tid % NG, px = tid / NG;
  float psum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (px < PX) {
    for (int p = px; p < T * T; p += PX) {
      const int oy = p / T, ox = p - oy * T;
      if (oy0 + oy >= Ho || ox0 + ox >= Wo) continue;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = sb[g * 8 + j];
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const uint4 v = *reinterpret_cast<const uint4*>(tile + ((size_t)((oy * S + ky) * IT + ox * S + kx) * NG + g) * 8);
          const float4 w0 = *reinterpret_cast<const float4*>(sw + (ky * K + kx) * CW + g * 8);
          const float4 w1 = *reinterpret_cast<const float4*>(sw + (ky * K + kx) * CW + g * 8 + 4);
          acc[0] = fmaf(lo_h(v.x), w0.x, acc[0]); acc[1] = fmaf(hi_h(v.x), w0.y, acc[1]);
          acc[2] = fmaf(lo_h(v.y), w0.z, acc[2]); acc[3] = fmaf(hi_h(v.y), w0.w, acc[3]);
          acc[4] = fmaf(lo_h(v.z), w1.x, acc[4]); acc[5] = fmaf(hi_h(v.z), w1.y, acc[5]);
          acc[6] = fmaf(lo_h(v.w), w1.z, acc[6]); acc[7] = fmaf(hi_h(v.w), w1.w, acc[7]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j] = act_apply(acc[j], ACT_SILU);
        psum[j] += acc[j];
      }
      *reinterpret_cast<uint4*>(at_bytes(out + (size_t)bi * Ho * Wo * C,
                                         (uint32_t)(((oy0 + oy) * Wo + ox0 + ox) * C + c0 + g * 8) * 2u)) =
          make_uint4(pack2h(acc[0], acc[1]), pack2h(acc[2], acc[3]), pack2h(acc[4], acc[5]),
                     pack2h(acc[6], acc[7]));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[px * CW + g * 8 + j] = psum[j];
  }
  __syncthreads();
  // fixed-order reduction over pixel lanes -> one partial per (image, tile, channel)
  const int ntiles = gridDim.x;
  for (int c = tid; c < CW; c += 256) {
    float sum = 0.f;
    for (int q = 0; q < PX; ++q) sum += red[q * CW + c];
    *at_bytes(pool_part + (size_t)bi * ntiles * C, (uint32_t)(blockIdx.x * C + c0 + c) * 4u) = sum;
  }
}

// acc + (float)half * w in one v_fma_mix_f32 (the half selected from a packed pair, converted exactly
// in the multiplier: the same single-rounding fmaf as converting first, so outputs are bit-identical),
// so the depthwise taps need no separate f16 -> f32 conversions.  Build with -DMMF_DW_MIX=0 for the
// convert-once + packed-FMA form (measured: depthwise / fused-front kernels 1-11 % slower).
#ifndef MMF_DW_MIX
#define MMF_DW_MIX 1
#endif
template <bool HI>
MMF_DEV float fma_mix(uint32_t h2, float w, float acc) {
  float d;
  if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h2), "v"(w), "v"(acc));
  else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h2), "v"(w), "v"(acc));
  return d;
}

// Compile-time-geometry variant of dw_compute: T x T output tile, CW channels, and each work item
// (channel group g, output row oy, run of R consecutive outputs) walks the input row segment of a
// kernel row once -- ((R-1)S + K) LDS reads / fp16 unpacks per kernel row instead of R*K -- and
// reuses the kernel row's weights for all R outputs (K reads instead of R*K).  Per output the
// VALU work drops by ~30 % at K = 5, R = 7, and every tile offset is an immediate.
// Items = NG * T * (T / R) over the first (256 / NG) * NG threads (each keeps its channel group).
// PS: halfs per tile pixel (CW, or CW + a pad that spreads a wave's 16-B tap reads over more LDS banks).
template <int K, int S, int T, int CW, int R, int PS = CW>
MMF_DEV void dw_compute_ct(const f16_t* tile, const float* sw, const float* sb, float* red, f16_t* __restrict__ out,
                           float* __restrict__ pool_part, int bi, int c0, int oy0, int ox0, int Ho, int Wo, int C,
                           int tix, int ntiles) {
  constexpr int NG = CW / 8, IT = (T - 1) * S + K, NR = T / R, ITEMS = NG * T * NR, IC = (R - 1) * S + K;
  constexpr int STRIDE = (256 / NG) * NG;  // active threads: a thread's channel group g never changes
  constexpr int NRED = STRIDE / NG;         // partial-sum slots per channel (<= the caller's red rows)
  static_assert(T % R == 0, "runs tile the row");
  static_assert(PS >= CW && PS % 8 == 0, "16-B aligned pixels");
  const int tid = threadIdx.x;
  const int g = tid % NG;
  float psum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (tid < STRIDE) {
    for (int item = tid; item < ITEMS; item += STRIDE) {
      const int rest = item / NG;
      const int run = rest % NR, oy = rest / NR, ox = run * R;
      if (oy0 + oy >= Ho) continue;
      float acc[R][8];
#pragma unroll
      for (int o = 0; o < R; ++o)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[o][j] = sb[g * 8 + j];
#pragma unroll 1
      for (int ky = 0; ky < K; ++ky) {
        float wk[K][8];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float4 w0 = *reinterpret_cast<const float4*>(sw + (ky * K + kx) * CW + g * 8);
          const float4 w1 = *reinterpret_cast<const float4*>(sw + (ky * K + kx) * CW + g * 8 + 4);
          wk[kx][0] = w0.x; wk[kx][1] = w0.y; wk[kx][2] = w0.z; wk[kx][3] = w0.w;
          wk[kx][4] = w1.x; wk[kx][5] = w1.y; wk[kx][6] = w1.z; wk[kx][7] = w1.w;
        }
        const f16_t* row = tile + (size_t)((oy * S + ky) * IT + ox * S) * PS + g * 8;
#pragma unroll
        for (int col = 0; col < IC; ++col) {
          const uint4 v = *reinterpret_cast<const uint4*>(row + col * PS);
          if constexpr (MMF_DW_MIX) {
            const uint32_t hv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int o = 0; o < R; ++o) {
              const int kx = col - o * S;
              if (kx >= 0 && kx < K) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  acc[o][2 * q] = fma_mix<false>(hv[q], wk[kx][2 * q], acc[o][2 * q]);
                  acc[o][2 * q + 1] = fma_mix<true>(hv[q], wk[kx][2 * q + 1], acc[o][2 * q + 1]);
                }
              }
            }
          } else {
            const float f[8] = {lo_h(v.x), hi_h(v.x), lo_h(v.y), hi_h(v.y),
                                lo_h(v.z), hi_h(v.z), lo_h(v.w), hi_h(v.w)};
#pragma unroll
            for (int o = 0; o < R; ++o) {
              const int kx = col - o * S;
              if (kx >= 0 && kx < K) {
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[o][j] = fmaf(f[j], wk[kx][j], acc[o][j]);
              }
            }
          }
        }
      }
#pragma unroll
      for (int o = 0; o < R; ++o) {
        if (ox0 + ox + o < Wo) {
          act4<ACT_SILU, true>(acc[o]);
          act4<ACT_SILU, true>(acc[o] + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) psum[j] += acc[o][j];
          *reinterpret_cast<uint4*>(at_bytes(out + (size_t)bi * Ho * Wo * C,
                                             (uint32_t)(((oy0 + oy) * Wo + ox0 + ox + o) * C + c0 + g * 8) * 2u)) =
              make_uint4(pack2h(acc[o][0], acc[o][1]), pack2h(acc[o][2], acc[o][3]), pack2h(acc[o][4], acc[o][5]),
                         pack2h(acc[o][6], acc[o][7]));
        }
      }
    }
  }
  __syncthreads();  // `red` aliases the input tile: every tap read is done before it is overwritten
  if (tid < STRIDE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(tid / NG) * CW + g * 8 + j] = psum[j];
  }
  __syncthreads();
  // fixed-order reduction over the thread slots of each channel -> one partial per (image, tile, channel)
  for (int c = tid; c < CW; c += 256) {
    float sum = 0.f;
    for (int q = 0; q < NRED; ++q) sum += red[q * CW + c];
    *at_bytes(pool_part + (size_t)bi * ntiles * C, (uint32_t)(tix * C + c0 + c) * 4u) = sum;
  }
}

// LDS bytes of the input tile region.  Compile-time-geometry kernels (dw_compute_ct) reuse it for
// the pool-partial slots `red` once the taps are done (fewer LDS bytes -> one more block per CU).
MMF_DEV_HOST_INLINE int dw_tile_bytes(int IT, int CW, bool alias_red, int PS = 0) {
  const int t = IT * IT * (PS ? PS : CW) * 2, r = (256 / (CW / 8)) * CW * 4;
  return ((alias_red && r > t ? r : t) + 15) & ~15;
}

// Depthwise kxk conv, LDS-tiled: a block owns a T x T output tile of one image and CW channels
// (CW = 32 or 48, i.e. NG = 4 or 6 groups of 8).  The input tile with its halo
// ((T-1)S + K)^2 x CW is read from HBM once, coalesced (zero padding written as zeros), and every
// tap is then served from LDS; weights sit in LDS as [tap][CW] fp32.  Thread (px, g) computes
// output pixels px, px + PX, ... for channel group g, so the SE pool partial of a channel stays in
// one thread and is reduced across px in a fixed order (deterministic, no atomics): one partial
// per (image, tile, channel).
// grid (tiles_y * tiles_x, C / CW, B); block 256 threads (PX * NG of them active in phase 2)
// TT / CWT / R > 0: compile-time tile edge, channel width and output run (dw_compute_ct); 0: runtime
template <int K, int S, int TT, int CWT, int R>
__global__ __launch_bounds__(256, 3) void dwconv_kernel(const f16_t* __restrict__ in, const float* __restrict__ w,
                                                     const float* __restrict__ bias, f16_t* __restrict__ out,
                                                     float* __restrict__ pool_part, int H, int W, int C, int CW_,
                                                     int T_, int tiles_x) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dw_smem[];
  constexpr int PAD = (K - 1) / 2;
  const int T = TT ? TT : T_, CW = CWT ? CWT : CW_;
  const int NG = CW / 8, IT = (T - 1) * S + K;  // input tile edge
  const int tid = threadIdx.x;
  const int bi = blockIdx.z, c0 = blockIdx.y * CW;
  const int ty0 = blockIdx.x / tiles_x, tx0 = blockIdx.x - ty0 * tiles_x;
  const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
  const int oy0 = ty0 * T, ox0 = tx0 * T;
  f16_t* tile = (f16_t*)dw_smem;                                 // [IT][IT][CW]
  float* sw = (float*)(dw_smem + dw_tile_bytes(IT, CW, TT > 0));  // [K*K][CW]
  float* sb = sw + K * K * CW;                                     // [CW]
  float* red = TT > 0 ? (float*)dw_smem : sb + CW;                 // [PX][CW]
  EST_BEGIN(8 + ((K == 5) * 2 + (S == 2)) * 4 + (TT == 14 ? 1 : TT == 7 ? 2 : TT == 16 ? 3 : 0))

  // ---- input tile (+halo) -> LDS ----
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  auto tile_src = [&](int idx, uint4& v) {
    const int g = idx % NG, pix = idx / NG;
    const int ty = pix / IT, tx = pix - ty * IT;
    const int iy = iy0 + ty, ix = ix0 + tx;
    v = make_uint4(0, 0, 0, 0);
    if (idx < IT * IT * NG && iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(at_bytes(in + (size_t)bi * H * W * C, (uint32_t)((iy * W + ix) * C + c0 + g * 8) * 2u));
  };
  if constexpr (TT > 0) {
    // compile-time tile: every thread's loads are issued before its first LDS store, so the
    // block pays one HBM latency for the tile instead of one per loop trip
    constexpr int NL = ((((TT - 1) * S + K) * ((TT - 1) * S + K) * (CWT / 8)) + 255) / 256;
    uint4 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) tile_src(tid + i * 256, v[i]);
#pragma unroll
    for (int i = 0; i < NL; ++i)
      if (tid + i * 256 < IT * IT * NG) *reinterpret_cast<uint4*>(tile + (size_t)(tid + i * 256) * 8) = v[i];
  } else {
    for (int idx = tid; idx < IT * IT * NG; idx += 256) {
      uint4 v;
      tile_src(idx, v);
      *reinterpret_cast<uint4*>(tile + (size_t)idx * 8) = v;
    }
  }
  if constexpr (TT > 0) {
    constexpr int NW = (K * K * CWT + 255) / 256;
    float wv[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int i = tid + j * 256, t = i / CWT, c = i - t * CWT;
      wv[j] = i < K * K * CWT ? w[(size_t)(c0 + c) * K * K + t] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NW; ++j)
      if (tid + j * 256 < K * K * CWT) sw[tid + j * 256] = wv[j];
  } else {
    for (int i = tid; i < K * K * CW; i += 256) {
      const int t = i / CW, c = i - t * CW;
      sw[i] = w[(size_t)(c0 + c) * K * K + t];
    }
  }
  for (int i = tid; i < CW; i += 256) sb[i] = bias[c0 + i];
  __syncthreads();
  EST()

  if constexpr (TT > 0)
    dw_compute_ct<K, S, TT, CWT, R>(tile, sw, sb, red, out, pool_part, bi, c0, oy0, ox0, Ho, Wo, C, blockIdx.x, gridDim.x);
  else dw_compute<K, S>(tile, sw, sb, red, out, pool_part, bi, c0, oy0, ox0, Ho, Wo, C, CW, T, IT);
  EST()
  EST_END()
}

// MBConv front, fused: 1x1 expand (BN folded) + SiLU computed per input tile on the MFMA, straight
// into the depthwise conv's LDS tile, then the depthwise conv of dwconv_kernel.  The expanded
// activation (6x the block's input channels, the largest tensor of the block) never touches HBM:
// the block reads its Cin-channel input (once per 48-channel group, plus the halo) instead of
// writing and re-reading Cexp channels.  Used where Cin <= 64 (the high-resolution stages 2-4,
// where that tensor dominates the image tower's traffic); elsewhere expand is its own launch.
//  expand: E[pix][c] = SiLU(be[c] + sum_k X[pix][k] We[c][k]) as D = We . X^T on
//          v_mfma_f32_16x16x32_f16 (A = We rows of this channel group, B = 16 tile pixels), each
//          lane ends with 4 consecutive channels of one pixel -> 8-B LDS writes; pixels outside the
//          image are written as 0 (the depthwise conv zero-pads E, not X).
// grid (tiles, Cexp / CW, B); block 256 threads; KS = ceil(Cin / 32) <= 2
// MMF_EDW_PF = 1: the next group's weights are fetched into registers under the current group
#ifndef MMF_EDW_PF
#define MMF_EDW_PF 1
#endif
// MMF_EDW_PADSKIP = 1: fragment rows wholly in the zero padding skip their expand MFMAs and SiLU
#ifndef MMF_EDW_PADSKIP
#define MMF_EDW_PADSKIP 1
#endif
template <int K, int S, int KS, int TT, int R, int TPAD>
#ifndef MMF_EDW_MINB1
#define MMF_EDW_MINB1 4  // resident blocks per CU hipcc budgets registers for (KS = 1: stage 3.1 148 -> 128 VGPRs, 4 blocks/CU; -0.9 %)
#endif
__global__ __launch_bounds__(256, KS == 1 ? MMF_EDW_MINB1 : KS == 2 ? 3 : 2) void expand_dw_kernel(const f16_t* __restrict__ x, int Cin,
                                                        const f16_t* __restrict__ we, const float* __restrict__ be,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        f16_t* __restrict__ out, float* __restrict__ pool_part, int H,
                                                        int W, int C, int CW_, int T_, int tiles_x, int gpb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dw_smem[];
  constexpr int PAD = (K - 1) / 2, KP = KS * 32;
  constexpr int CW = 48, NF = CW / 16;  // the host launches 48-channel groups only
  constexpr int PS = CW + (TT ? TPAD : 0);  // halfs per tile pixel (the runtime-geometry dw_compute: CW)
  constexpr int NRF_CT = TT ? ((((TT - 1) * S + K) * ((TT - 1) * S + K)) + 15) / 16 : 0;
  const int T = TT ? TT : T_;
  const int NG = CW / 8, IT = (T - 1) * S + K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int bi = blockIdx.z;
  const int ty0 = blockIdx.x / tiles_x, tx0 = blockIdx.x - ty0 * tiles_x;
  const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
  const int oy0 = ty0 * T, ox0 = tx0 * T;
  f16_t* tile = (f16_t*)dw_smem;                                     // [IT][IT][PS]
  float* sw = (float*)(dw_smem + dw_tile_bytes(IT, CW, TT > 0, PS));  // [K*K][CW]
  float* sb = sw + K * K * CW;                                         // [CW]
  float* red = TT > 0 ? (float*)dw_smem : sb + CW;                     // [PX][CW]
  float* sbe = TT > 0 ? sb + CW : red + (256 / NG) * CW;           // [CW] expand bias
  f16_t* swe = (f16_t*)(sbe + CW);                        // [CW][KP] expand weights (zero-padded K)

  EST_BEGIN((K == 5) * 4 + (S == 2) * 2 + (KS == 2))
  // this wave's input-pixel fragments first: their HBM latency overlaps the weight staging
  constexpr int MAXRF = 6;  // ceil(ceil(IT^2 / 16) / 4) for IT <= 19 (host-checked)
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int npix = IT * IT, nrf = (npix + 15) / 16;
  uint4 xr[MAXRF][KS];
#pragma unroll
  for (int it = 0; it < MAXRF; ++it) {
    const int pix = (wave + 4 * it) * 16 + fr;
    const int ty = pix / IT, tx = pix - ty * IT;
    const int iy = iy0 + ty, ix = ix0 + tx;
    const bool inimg = pix < npix && iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + fg * 8;
      xr[it][ks] = (inimg && k < Cin) ? *reinterpret_cast<const uint4*>(at_bytes(x + (size_t)bi * H * W * Cin,
                                                                                 (uint32_t)((iy * W + ix) * Cin + k) * 2u))
                                      : make_uint4(0, 0, 0, 0);
    }
  }
  // every 48-channel group of the block's Cexp channels, reusing the input fragments above.  The
  // group's weights are fetched into registers one group ahead (issued under the previous group's
  // expand + depthwise phases) and written to LDS after that group's trailing barrier.
  constexpr int NPE = (CW * (KP / 8) + 255) / 256, NPD = (K * K * CW + 255) / 256;
  uint4 pe[NPE];
  float pd[NPD], pbias = 0.f, pbe = 0.f;
  auto fetch_w = [&](int c0) {
#pragma unroll
    for (int j = 0; j < NPE; ++j) {
      const int i = tid + j * 256, r = i / (KP / 8), kc = i - r * (KP / 8);
      pe[j] = (i < CW * (KP / 8) && kc * 8 < Cin) ? *reinterpret_cast<const uint4*>(we + (size_t)(c0 + r) * Cin + kc * 8)
                                                   : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NPD; ++j) {
      const int i = tid + j * 256, t = i / CW, c = i - t * CW;
      pd[j] = i < K * K * CW ? w[(size_t)(c0 + c) * K * K + t] : 0.f;
    }
    if (tid < CW) {
      pbias = bias[c0 + tid];
      pbe = be[c0 + tid];
    }
  };
  // this block's channel groups: gpb of them from blockIdx.y * gpb (launch_expand_dw splits the groups
  // over blocks when the launch has too few tiles to fill the chip)
  const int cbeg = blockIdx.y * gpb * CW, cend = min(C, cbeg + gpb * CW);
  if (MMF_EDW_PF) fetch_w(cbeg);
  for (int c0 = cbeg; c0 < cend; c0 += CW) {
    if (!MMF_EDW_PF) fetch_w(c0);
#pragma unroll
    for (int j = 0; j < NPE; ++j) {
      const int i = tid + j * 256, r = i / (KP / 8), kc = i - r * (KP / 8);
      if (i < CW * (KP / 8)) *reinterpret_cast<uint4*>(swe + r * KP + kc * 8) = pe[j];
    }
#pragma unroll
    for (int j = 0; j < NPD; ++j)
      if (tid + j * 256 < K * K * CW) sw[tid + j * 256] = pd[j];
    if (tid < CW) {
      sb[tid] = pbias;
      sbe[tid] = pbe;
    }
    __syncthreads();
    EST()
    if (MMF_EDW_PF && c0 + CW < cend) fetch_w(c0 + CW);

    // ---- expand the input tile (+halo) into LDS: every MFMA of a fragment row issued before its
    // epilogues (the group's weight fragments and bias held in registers) ----
    {
      f16x8 wf[NF][KS];
      float4 bev[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          wf[nf][ks] = as_f16x8(*reinterpret_cast<const uint4*>(swe + (nf * 16 + fr) * KP + ks * 32 + fg * 8));
        bev[nf] = *reinterpret_cast<const float4*>(sbe + nf * 16 + fg * 4);
      }
#pragma unroll
      for (int it = 0; it < MAXRF; ++it) {
        const int rf = wave + 4 * it;
        if ((TT > 0 && 4 * it + 3 < NRF_CT) || rf < nrf) {
          const int pix = rf * 16 + fr;
          const int ty = pix / IT, tx = pix - ty * IT;
          const int iy = iy0 + ty, ix = ix0 + tx;
          const bool inimg = pix < npix && iy >= 0 && iy < H && ix >= 0 && ix < W;
          if (MMF_EDW_PADSKIP && __builtin_amdgcn_ballot_w64(inimg) == 0) {
            // all 16 pixels of the fragment row lie in the zero padding (tile rows above / below the
            // image): their expanded values are the depthwise conv's zero padding, no MFMA or SiLU
#pragma unroll
            for (int nf = 0; nf < NF; ++nf)
              if (pix < npix) *reinterpret_cast<uint2*>(tile + (size_t)pix * PS + nf * 16 + fg * 4) = make_uint2(0u, 0u);
            continue;
          }
          f32x4 acc[NF];
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) acc[nf] = mfma16x16x32(wf[nf][ks], as_f16x8(xr[it][ks]), acc[nf]);
          }
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            float e[4] = {acc[nf][0] + bev[nf].x, acc[nf][1] + bev[nf].y, acc[nf][2] + bev[nf].z, acc[nf][3] + bev[nf].w};
            act4<ACT_SILU, true>(e);
            // zero padding masked on the packed halves (2 ANDs instead of 4 selects; fp16 +0 either way)
            const uint32_t keep = 0u - (uint32_t)inimg;
            const uint2 hv = make_uint2(pack2h(e[0], e[1]) & keep, pack2h(e[2], e[3]) & keep);
            if (pix < npix) *reinterpret_cast<uint2*>(tile + (size_t)pix * PS + nf * 16 + fg * 4) = hv;
          }
        }
      }
    }
    __syncthreads();
    EST()
    if constexpr (TT > 0)
      dw_compute_ct<K, S, TT, CW, R, PS>(tile, sw, sb, red, out, pool_part, bi, c0, oy0, ox0, Ho, Wo, C, blockIdx.x, gridDim.x);
    else dw_compute<K, S>(tile, sw, sb, red, out, pool_part, bi, c0, oy0, ox0, Ho, Wo, C, CW, T, IT);
    EST()
    __syncthreads();  // the next group restages sw / sb / swe / tile and rewrites red
    EST()
  }
  EST_END()
}

// Stem + stage-1 depthwise, fused: the stem (ImageNet normalise -> conv3x3 s2 3->32 + BN + SiLU)
// is computed per 16x16 depthwise tile straight into the depthwise conv's LDS tile (its 18x18
// halo recomputed, 1.27x the stem work), so the 112x112x32 stem activation -- the largest tensor
// of the image tower -- never touches HBM: the block reads a 37x37x3 uint8 image patch instead.
//  stem on the MFMA as a K = 27 (padded to 32) GEMM: D[ch][pix] = W[ch][k] . P[k][pix] with
//  k = (ky, kx, c) so that each ky contributes 9 CONTIGUOUS floats of one patch row (HWC);
//  operands split as fp16 hi + lo (x = xh + xl, w = wh + wl; wl.xh + wh.xl + wh.xh, fp32
//  accumulation) so the conv keeps ~20 mantissa bits, well under the fp16 rounding of its output.
// grid (49, 1, B); block 256
constexpr int SD_T = 16, SD_IT = 18, SD_PR = 2 * SD_IT + 1, SD_PW = SD_PR * 3;
#ifndef MMF_SD_PAD
#define MMF_SD_PAD 0  // halfs of pad per stem-tile pixel; 16 halves the tap reads' LDS cycles but costs a block per CU: +0.4 % tower
#endif
constexpr int SD_PS = 32 + MMF_SD_PAD;

template <bool F32>
__global__ __launch_bounds__(256, 3) void stem_dw_kernel(const void* src, const float* __restrict__ ws,
                                                      const float* __restrict__ bs, const float* __restrict__ wd,
                                                      const float* __restrict__ bd, f16_t* __restrict__ out,
                                                      float* __restrict__ pool_part) {
  constexpr int CW = 32, NPIX = SD_IT * SD_IT, NMT = (NPIX + 15) / 16;
  __shared__ __attribute__((aligned(16))) float patch[(SD_PR * SD_PW + 255) / 256 * 256];  // image patch, HWC
  __shared__ __attribute__((aligned(16))) f16_t tile[NPIX * SD_PS];  // stem tile (+halo), SD_PS halfs per pixel
  __shared__ __attribute__((aligned(16))) float sw[9 * CW];
  __shared__ __attribute__((aligned(16))) float sb[CW];
  float* red = patch;  // pool-partial slots [64][32]: the patch is dead once the stem tile is built
  static_assert((SD_PR * SD_PW + 255) / 256 * 256 >= (256 / (CW / 8)) * CW, "red fits in the patch");
  const uint8_t* img = (const uint8_t*)src;
  const float* xf = (const float*)src;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int bi = blockIdx.z;
  const int ty0 = blockIdx.x / 7, tx0 = blockIdx.x - ty0 * 7;
  const int oy0 = ty0 * SD_T, ox0 = tx0 * SD_T;
  const int py0 = 2 * oy0 - 3, px0 = 2 * ox0 - 3;  // image coords of patch (0, 0)
  EST_BEGIN(24)

  // depthwise weights [C][9] transposed into LDS
  const float wd0 = wd[(tid % CW) * 9 + tid / CW];
  const float wd1 = tid + 256 < 9 * CW ? wd[((tid + 256) % CW) * 9 + (tid + 256) / CW] : 0.f;
  const float bd0 = tid < CW ? bd[tid] : 0.f;
  // stem weight fragments (A operand: row = output channel nt*16 + fr, k = fg*8 + e), split hi/lo
  int offk[8];
  f16x8 whi[2], wlo[2];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = fg * 8 + e, ky = k / 9, r9 = k - ky * 9;
    offk[e] = k < 27 ? ky * SD_PW + r9 : -1;
  }
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    float wv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = fg * 8 + e, ky = k / 9, r9 = k - ky * 9, kx = r9 / 3, c = r9 - kx * 3;
      wv[e] = k < 27 ? ws[(nt * 16 + fr) * 27 + c * 9 + ky * 3 + kx] : 0.f;
    }
    uint32_t h[4], l[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      h[q] = pack2h(wv[2 * q], wv[2 * q + 1]);
      l[q] = pack2h(wv[2 * q] - lo_h(h[q]), wv[2 * q + 1] - hi_h(h[q]));
    }
    whi[nt] = as_f16x8(make_uint4(h[0], h[1], h[2], h[3]));
    wlo[nt] = as_f16x8(make_uint4(l[0], l[1], l[2], l[3]));
  }
  float4 sbias[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) sbias[nt] = *reinterpret_cast<const float4*>(bs + nt * 16 + fg * 4);
  // ---- normalised patch -> LDS (zero outside the image: the stem pads after Normalize) ----
  constexpr int NP = SD_PR * SD_PW, NL = (NP + 255) / 256;
  float raw[NL];  // all of this thread's loads in flight before the first LDS store
  int chan[NL];   // channel of the element, -1 outside the image (zero padding)
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int idx = tid + i * 256;
    const int pr = idx / SD_PW, rem = idx - pr * SD_PW;
    const int pc = rem / 3, c = rem - pc * 3;
    const int iy = py0 + pr, ix = px0 + pc;
    // unconditional load from a clamped address (no divergent region around the load, so the
    // compiler does not drain vmcnt per element); out-of-image elements are zeroed below
    const bool ok = idx < NP && iy >= 0 && iy < 224 && ix >= 0 && ix < 224;
    const int iyc = min(max(iy, 0), 223), ixc = min(max(ix, 0), 223);
    chan[i] = ok ? c : -1;
    if constexpr (F32) raw[i] = xf[(((size_t)bi * 3 + c) * 224 + iyc) * 224 + ixc];
    else raw[i] = __builtin_bit_cast(float, (uint32_t)*at_bytes(img + (size_t)bi * 224 * 224 * 3,
                                                                (uint32_t)((iyc * 224 + ixc) * 3 + c)));
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {  // (the array is padded to NL * 256: no branch around the stores)
    const int c = chan[i];
    float v = raw[i];
    if constexpr (!F32) {  // ToTensor + Normalize: u / (255 std) - mean / std
      const float sc = c == 0 ? 1.0f / (255.0f * 0.229f) : c == 1 ? 1.0f / (255.0f * 0.224f) : 1.0f / (255.0f * 0.225f);
      const float of = c == 0 ? -0.485f / 0.229f : c == 1 ? -0.456f / 0.224f : -0.406f / 0.225f;
      v = fmaf((float)__builtin_bit_cast(uint32_t, v), sc, of);
    }
    patch[tid + i * 256] = c < 0 ? 0.f : v;
  }
  sw[tid] = wd0;
  if (tid + 256 < 9 * CW) sw[tid + 256] = wd1;
  if (tid < CW) sb[tid] = bd0;
  __syncthreads();
  EST()

  // ---- stem: 16 tile pixels per MFMA column block ----
  for (int mt = wave; mt < NMT; mt += 4) {
    const int p = mt * 16 + fr;
    const int pc = p < NPIX ? p : NPIX - 1;
    const int sy = pc / SD_IT, sx = pc - sy * SD_IT;
    const int base = sy * 2 * SD_PW + sx * 6;
    float xv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = offk[e] >= 0 ? patch[base + offk[e]] : 0.f;
    uint32_t h[4], l[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      h[q] = pack2h(xv[2 * q], xv[2 * q + 1]);
      l[q] = pack2h(xv[2 * q] - lo_h(h[q]), xv[2 * q + 1] - hi_h(h[q]));
    }
    const f16x8 xhi = as_f16x8(make_uint4(h[0], h[1], h[2], h[3]));
    const f16x8 xlo = as_f16x8(make_uint4(l[0], l[1], l[2], l[3]));
    const int gy = oy0 - 1 + sy, gx = ox0 - 1 + sx;  // stem output coords of this pixel
    const bool inimg = gy >= 0 && gy < 112 && gx >= 0 && gx < 112;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      acc = mfma16x16x32(wlo[nt], xhi, acc);
      acc = mfma16x16x32(whi[nt], xlo, acc);
      acc = mfma16x16x32(whi[nt], xhi, acc);
      float e4[4] = {acc[0] + sbias[nt].x, acc[1] + sbias[nt].y, acc[2] + sbias[nt].z, acc[3] + sbias[nt].w};
      act4<ACT_SILU, true>(e4);
      const int ch = nt * 16 + fg * 4;
      f16_t* dst = tile + p * SD_PS + ch;
      if (p < NPIX)
        *reinterpret_cast<uint2*>(dst) = inimg ? make_uint2(pack2h(e4[0], e4[1]), pack2h(e4[2], e4[3])) : make_uint2(0, 0);
    }
  }
  __syncthreads();
  EST()
  dw_compute_ct<3, 1, SD_T, CW, 4, SD_PS>(tile, sw, sb, red, out, pool_part, bi, 0, oy0, ox0, 112, 112, CW, blockIdx.x, 49);
  EST()
  EST_END()
}

// Squeeze-excitation, one 1024-thread block per image.  The three phases are each a few dependent
// L2 round trips, so the kernel is latency-bound: every phase keeps many independent loads in
// flight (unrolled partial sums) instead of walking dependent chains.
//   pool : pooled[c] = sum over the dwconv's per-tile partials (fixed order) / HW
//   fc1  : s1[o] = SiLU(b1[o] + w1[o,:] . pooled)  -- each of the 16 waves owns <= 4 outputs and
//          accumulates them together (lanes stride over C), then one wave reduction per output
//   fc2  : scale[c] = sigmoid(b2[c] + sum_j w2t[j][c] s1[j])  (w2t = fc2 weight transposed at load,
//          so consecutive threads read consecutive addresses)
constexpr int SE_THREADS = 1024;
#ifndef SE_FC1_U
#define SE_FC1_U 8
#endif

template <bool PRECISE>
__global__ __launch_bounds__(SE_THREADS) void se_kernel(const float* pool_part, int nchunks, float inv_hw,
                                                        const float* w1, const float* b1, const float* w2t,
                                                        const float* b2, float* scale, int C, int Csq) {
  __shared__ float pooled[1280];
  __shared__ float s1[64];
  const int bi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* pp = pool_part + (size_t)bi * nchunks * C;
  for (int c = tid; c < C; c += SE_THREADS) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int k = 0;
    for (; k + 16 <= nchunks; k += 16) {  // 16 partials in flight (the 49- / 16-tile early stages)
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = pp[(size_t)(k + u) * C + c];
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        a0 += v[u];
        a1 += v[u + 1];
        a2 += v[u + 2];
        a3 += v[u + 3];
      }
    }
    for (; k + 4 <= nchunks; k += 4) {
      a0 += pp[(size_t)k * C + c];
      a1 += pp[(size_t)(k + 1) * C + c];
      a2 += pp[(size_t)(k + 2) * C + c];
      a3 += pp[(size_t)(k + 3) * C + c];
    }
    for (; k < nchunks; ++k) a0 += pp[(size_t)k * C + c];
    pooled[c] = ((a0 + a1) + (a2 + a3)) * inv_hw;
  }
  __syncthreads();
  {
    constexpr int OPW = 4;  // outputs per wave (Csq <= 64 = 16 waves x 4)
    float acc[OPW] = {0.f, 0.f, 0.f, 0.f};
    // the wave's outputs walk C together: per step SE_FC1_U weights of every output in flight (4 x U
    // loads, one L2 round trip per step for all outputs); each output's FMAs stay in ascending c
    // (lane, lane + 64, ...).  U = 8: the C = 672 / 1152 blocks in 2 - 3 steps instead of 3 - 5
    constexpr int U = SE_FC1_U;
    for (int c = lane; c < C; c += 64 * U) {
      float wv[OPW][U];
#pragma unroll
      for (int t = 0; t < OPW; ++t) {
        const int o = wave + 16 * t;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int cc = c + 64 * u;
          wv[t][u] = (o < Csq && cc < C) ? w1[(size_t)o * C + cc] : 0.f;
        }
      }
#pragma unroll
      for (int t = 0; t < OPW; ++t)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (wave + 16 * t < Csq && c + 64 * u < C) acc[t] = fmaf(wv[t][u], pooled[c + 64 * u], acc[t]);
    }
#pragma unroll
    for (int t = 0; t < OPW; ++t) {
      const int o = wave + 16 * t;
      const float a = wave_sum(acc[t]);
      if (o < Csq && lane == 0) s1[o] = PRECISE ? silu_precise(a + b1[o]) : act_apply(a + b1[o], ACT_SILU);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += SE_THREADS) {
    float a0 = b2[c], a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int j = 0;
    // 32 weight loads in flight per step (one L2 round trip per 32 inputs: Csq <= 64 in two); the
    // accumulation order is unchanged (input j -> accumulator j % 4, ascending j)
    for (; j + 32 <= Csq; j += 32) {
      float wv[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) wv[u] = w2t[(size_t)(j + u) * C + c];
#pragma unroll
      for (int u = 0; u < 32; u += 4) {
        a0 = fmaf(wv[u], s1[j + u], a0);
        a1 = fmaf(wv[u + 1], s1[j + u + 1], a1);
        a2 = fmaf(wv[u + 2], s1[j + u + 2], a2);
        a3 = fmaf(wv[u + 3], s1[j + u + 3], a3);
      }
    }
    for (; j + 16 <= Csq; j += 16) {
      float wv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) wv[u] = w2t[(size_t)(j + u) * C + c];
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        a0 = fmaf(wv[u], s1[j + u], a0);
        a1 = fmaf(wv[u + 1], s1[j + u + 1], a1);
        a2 = fmaf(wv[u + 2], s1[j + u + 2], a2);
        a3 = fmaf(wv[u + 3], s1[j + u + 3], a3);
      }
    }
    for (; j + 4 <= Csq; j += 4) {
      a0 = fmaf(w2t[(size_t)j * C + c], s1[j], a0);
      a1 = fmaf(w2t[(size_t)(j + 1) * C + c], s1[j + 1], a1);
      a2 = fmaf(w2t[(size_t)(j + 2) * C + c], s1[j + 2], a2);
      a3 = fmaf(w2t[(size_t)(j + 3) * C + c], s1[j + 3], a3);
    }
    for (; j < Csq; ++j) a0 = fmaf(w2t[(size_t)j * C + c], s1[j], a0);
    const float a = (a0 + a1) + (a2 + a3);
    scale[(size_t)bi * C + c] = 1.0f / (1.0f + expf(-a));
  }
}

__global__ __launch_bounds__(256) void gap_classifier_kernel(const f16_t* x, int HW, int C, const float* w,
                                                             const float* b, float* logits, float* score,
                                                             int score_stride) {
  __shared__ float red[2][4];
  const int bi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float l0 = 0.f, l1 = 0.f;
  const float inv = 1.0f / (float)HW;
  // 8 channels per thread (16-B loads), pixels summed in order; 7 rows of loads in flight
  for (int c8 = tid * 8; c8 < C; c8 += 256 * 8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const f16_t* xp = x + (size_t)bi * HW * C + c8;
    int p = 0;
    for (; p + 7 <= HW; p += 7) {
      uint4 v[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) v[u] = *reinterpret_cast<const uint4*>(xp + (size_t)(p + u) * C);
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        s[0] += lo_h(v[u].x); s[1] += hi_h(v[u].x); s[2] += lo_h(v[u].y); s[3] += hi_h(v[u].y);
        s[4] += lo_h(v[u].z); s[5] += hi_h(v[u].z); s[6] += lo_h(v[u].w); s[7] += hi_h(v[u].w);
      }
    }
    for (; p < HW; ++p) {
      const uint4 v = *reinterpret_cast<const uint4*>(xp + (size_t)p * C);
      s[0] += lo_h(v.x); s[1] += hi_h(v.x); s[2] += lo_h(v.y); s[3] += hi_h(v.y);
      s[4] += lo_h(v.z); s[5] += hi_h(v.z); s[6] += lo_h(v.w); s[7] += hi_h(v.w);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      l0 = fmaf(w[c8 + j], s[j] * inv, l0);
      l1 = fmaf(w[C + c8 + j], s[j] * inv, l1);
    }
  }
  l0 = wave_sum(l0);
  l1 = wave_sum(l1);
  if (lane == 0) { red[0][wave] = l0; red[1][wave] = l1; }
  __syncthreads();
  if (tid == 0) {
    const float a = red[0][0] + red[0][1] + red[0][2] + red[0][3] + b[0];
    const float c1 = red[1][0] + red[1][1] + red[1][2] + red[1][3] + b[1];
    if (logits) { logits[bi * 2] = a; logits[bi * 2 + 1] = c1; }
    if (score) {
      const float m = fmaxf(a, c1), e0 = expf(a - m), e1 = expf(c1 - m);
      score[(size_t)bi * score_stride] = e1 / (e0 + e1);
    }
  }
}

}  // namespace

#ifdef MMF_EFF_STAMP
// diagnostic build: where the stamping kernels write (nullptr = off)
extern "C" int mmf_debug_eff_stamp(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_eff_stamp), &buf, sizeof(buf));
}
#endif

hipError_t launch_effnet_stem(const uint8_t* img, const float* w, const float* bias, f16_t* out, int B,
                              hipStream_t s) {
  const size_t total = (size_t)B * 112 * 112;
  hipLaunchKernelGGL(stem_kernel<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const void*)img, w,
                     bias, out, B);
  return hipGetLastError();
}

hipError_t launch_effnet_stem_dw(const uint8_t* img, const float* xf32, const float* ws, const float* bs,
                                 const float* wd, const float* bd, f16_t* out, float* pool_part, int B,
                                 int* nchunks_out, hipStream_t s) {
  *nchunks_out = 49;  // = dwconv_nchunks(112, 112, 32, 1): the SE reads the same partial layout
  const dim3 grid(49, 1, B), blk(256);
  if (xf32) hipLaunchKernelGGL((stem_dw_kernel<true>), grid, blk, 0, s, (const void*)xf32, ws, bs, wd, bd, out, pool_part);
  else hipLaunchKernelGGL((stem_dw_kernel<false>), grid, blk, 0, s, (const void*)img, ws, bs, wd, bd, out, pool_part);
  return hipGetLastError();
}

hipError_t launch_effnet_stem_f32(const float* x, const float* w, const float* bias, f16_t* out, int B,
                                  hipStream_t s) {
  const size_t total = (size_t)B * 112 * 112;
  hipLaunchKernelGGL(stem_kernel<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const void*)x, w,
                     bias, out, B);
  return hipGetLastError();
}

hipError_t launch_effnet_stem32(const uint8_t* img, const float* x, const float* w, const float* bias, float* out,
                                int B, hipStream_t s) {
  const dim3 grid((unsigned)(((size_t)B * 112 * 112 + 255) / 256)), blk(256);
  if (x) hipLaunchKernelGGL((stem_kernel<true, float>), grid, blk, 0, s, (const void*)x, w, bias, out, B);
  else hipLaunchKernelGGL((stem_kernel<false, float>), grid, blk, 0, s, (const void*)img, w, bias, out, B);
  return hipGetLastError();
}

// depthwise output runs R of the compile-time geometries (dw_compute_ct; -D overrides for A/B builds)
#ifndef MMF_R_D16
#define MMF_R_D16 4
#endif
#ifndef MMF_R_D14
#define MMF_R_D14 2
#endif
#ifndef MMF_R_D8
#define MMF_R_D8 2
#endif
#ifndef MMF_R_D7
#define MMF_R_D7 1
#endif
#ifndef MMF_R_E21
#define MMF_R_E21 2
#endif
#ifndef MMF_R_E22
#define MMF_R_E22 2
#endif
#ifndef MMF_R_E32
#define MMF_R_E32 2
#endif
#ifndef MMF_R_E31
#define MMF_R_E31 1
#endif
#ifndef MMF_R_E41
#define MMF_R_E41 1
#endif

// tile edge: the largest divisor of the output edge up to 16 (stride 1) / 8 (stride 2)
// narrow = true (standalone depthwise launches, option dw_cw32): 32-channel groups where C allows, for
// 24 KB instead of 36 KB of LDS per 14x14 k5 block (more resident blocks); the tile count is unchanged
static void dw_geometry(int H, int W, int C, int stride, int* T_, int* CW_, int* tiles_x_, int* ntiles_,
                        bool narrow = false) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int cap = stride == 1 ? 16 : 8;
  int T = 1;
  for (int t = cap; t >= 1; --t)
    if (Ho % t == 0) { T = t; break; }
  const int tx = (Wo + T - 1) / T, ty = (Ho + T - 1) / T;
  *T_ = T;
  *CW_ = (C % 48 == 0 && !(narrow && C % 32 == 0)) ? 48 : 32;
  *tiles_x_ = tx;
  *ntiles_ = tx * ty;
}

int dwconv_nchunks(int H, int W, int C, int stride) {
  int T, CW, tx, n;
  dw_geometry(H, W, C, stride, &T, &CW, &tx, &n);
  return n;
}

hipError_t launch_dwconv(const f16_t* in, const float* w, const float* bias, f16_t* out, float* pool_part, int B,
                         int H, int W, int C, int k, int stride, int* nchunks_out, hipStream_t s, int ct) {
  int T, CW, tiles_x, ntiles;
  dw_geometry(H, W, C, stride, &T, &CW, &tiles_x, &ntiles, (ct & 8) != 0);
  if (C % CW) return hipErrorInvalidValue;
  *nchunks_out = ntiles;
  const int IT = (T - 1) * stride + k, PX = 256 / (CW / 8);
  const size_t smem = (size_t)dw_tile_bytes(IT, CW, false) + (size_t)(k * k * CW + CW + PX * CW) * 4;
  const size_t smem_ct = (size_t)dw_tile_bytes(IT, CW, true) + (size_t)(k * k * CW + CW) * 4;
  const dim3 grid(ntiles, C / CW, B), blk(256);
  // compile-time geometries of EfficientNet-B0 at 224^2 (output runs R chosen so that items <= 256)
#define MMF_DWCT(KK, SS, TT, CC, RR)                                                                          \
  if (k == KK && stride == SS && T == TT && CW == CC) {                                                        \
    hipLaunchKernelGGL((dwconv_kernel<KK, SS, TT, CC, RR>), grid, blk, smem_ct, s, in, w, bias, out, pool_part, H,   \
                       W, C, CW, T, tiles_x);                                                                 \
    return hipGetLastError();                                                                                 \
  }
  if (ct & 1) {  // bit 0 clear: runtime-geometry kernels only (parity tests)
    MMF_DWCT(3, 1, 16, 32, MMF_R_D16)
    MMF_DWCT(3, 1, 14, 32, MMF_R_D14)
    MMF_DWCT(5, 1, 14, 32, MMF_R_D14)
    MMF_DWCT(5, 1, 7, 32, MMF_R_D7)
    MMF_DWCT(3, 1, 7, 32, MMF_R_D7)
    MMF_DWCT(5, 2, 7, 32, MMF_R_D7)
    MMF_DWCT(3, 1, 14, 48, MMF_R_D14)
    MMF_DWCT(5, 1, 14, 48, MMF_R_D14)
    MMF_DWCT(3, 2, 8, 48, MMF_R_D8)
    MMF_DWCT(5, 1, 7, 48, MMF_R_D7)
    MMF_DWCT(3, 1, 7, 48, MMF_R_D7)
    MMF_DWCT(5, 2, 7, 48, MMF_R_D7)
    MMF_DWCT(3, 2, 7, 48, MMF_R_D7)
  }
#undef MMF_DWCT
#define MMF_DW(KK, SS)                                                                                        \
  if (k == KK && stride == SS) {                                                                              \
    hipLaunchKernelGGL((dwconv_kernel<KK, SS, 0, 0, 1>), grid, blk, smem, s, in, w, bias, out, pool_part, H, W, C, \
                       CW, T, tiles_x);                                                                       \
    return hipGetLastError();                                                                                 \
  }
  MMF_DW(3, 1)
  MMF_DW(3, 2)
  MMF_DW(5, 1)
  MMF_DW(5, 2)
#undef MMF_DW
  return hipErrorInvalidValue;
}

#ifndef MMF_EDW_PAD
#define MMF_EDW_PAD 8
#endif
#ifndef MMF_EDW_PAD52
#define MMF_EDW_PAD52 MMF_EDW_PAD  // stage 3.1 (5 x 5, stride 2; 40.6 KB per block at pad 8: still 4 per CU)
#endif
#ifndef MMF_EDW_SPLIT_BELOW
#define MMF_EDW_SPLIT_BELOW 8192  // fused fronts with fewer (tile, image) blocks split their channel groups (0: never; B = 512: 3.502 -> 3.475 ms)
#endif

// Cin <= 64 (stages 2 - 4.1, KS <= 2), and 3 x 3 blocks of Cin <= 96 (stages 4.2 / 4.3: Cin 80, KS = 3;
// their two launches 28 + 33 -> 45 us per 256 images).  The 5 x 5 blocks of Cin 80 / 112 (stages 5.1 -
// 6.1, KS = 3 / 4) measured a tie or slower fused (230-256 VGPRs: two waves per SIMD).
bool expand_dw_applicable(int cin, int cexp, int k) {
  const bool ok_cin = cin <= 64 || (k == 3 && cin <= 96);
  return ok_cin && (cin % 8) == 0 && (cexp % 48) == 0;
}

hipError_t launch_expand_dw(const f16_t* x, int cin, const f16_t* we, const float* be, const float* w,
                            const float* bias, f16_t* out, float* pool_part, int B, int H, int W, int C, int k,
                            int stride, int* nchunks_out, hipStream_t s, int ct) {
  int T, CW, tiles_x, ntiles;
  dw_geometry(H, W, C, stride, &T, &CW, &tiles_x, &ntiles);
  if (!expand_dw_applicable(cin, C, k) || CW != 48) return hipErrorInvalidValue;
  *nchunks_out = ntiles;
  const int IT = (T - 1) * stride + k, PX = 256 / (CW / 8), KS = (cin + 31) / 32;
  if (IT > 19) return hipErrorInvalidValue;  // the kernel's MAXRF prefetch depth
  const size_t smem =
      (size_t)dw_tile_bytes(IT, CW, false) + (size_t)(k * k * CW + CW + PX * CW + CW) * 4 + (size_t)CW * KS * 32 * 2;
  auto smem_ct = [&](int pad) {
    return (size_t)dw_tile_bytes(IT, CW, true, CW + pad) + (size_t)(k * k * CW + CW + CW) * 4 + (size_t)CW * KS * 32 * 2;
  };
  // launches with few tiles (the 28^2 / 14^2 stages) split their channel groups over blocks: one
  // block per (tile, group) instead of a block walking every group, so the chip fills (each block
  // re-reads its Cin-channel input tile from L2; every output and pool partial is computed as before)
  const int groups = C / CW;
  const long blocks = (long)ntiles * B;
  const int split = blocks < MMF_EDW_SPLIT_BELOW ? groups : 1;
  const int gpb = (groups + split - 1) / split;
  const dim3 grid(ntiles, (groups + gpb - 1) / gpb, B), blk(256);
#define MMF_EDWCT(KK, SS, QS, TT, RR, PP)                                                                    \
  if (k == KK && stride == SS && KS == QS && T == TT) {                                                        \
    hipLaunchKernelGGL((expand_dw_kernel<KK, SS, QS, TT, RR, PP>), grid, blk, smem_ct(PP), s, x, cin, we, be, w, bias, \
                       out, pool_part, H, W, C, CW, T, tiles_x, gpb);                                          \
    return hipGetLastError();                                                                                  \
  }
  // PP: tile-pixel pad in halfs (tools/dw_bank_model.py: 112-B pixels cut the tap reads' LDS cycles 10-21 %)
  if (ct) {
    MMF_EDWCT(3, 2, 1, 8, MMF_R_E21, MMF_EDW_PAD)
    MMF_EDWCT(3, 1, 1, 14, MMF_R_E22, MMF_EDW_PAD)
    MMF_EDWCT(5, 1, 2, 14, MMF_R_E32, MMF_EDW_PAD)
    MMF_EDWCT(5, 2, 1, 7, MMF_R_E31, MMF_EDW_PAD52)
    MMF_EDWCT(3, 2, 2, 7, MMF_R_E41, MMF_EDW_PAD)
    MMF_EDWCT(3, 1, 3, 14, MMF_R_D14, MMF_EDW_PAD)  // stages 4.2 / 4.3 (Cin 80)
  }
#undef MMF_EDWCT
#define MMF_EDW(KK, SS, QS)                                                                                      \
  if (k == KK && stride == SS && KS == QS) {                                                                     \
    hipLaunchKernelGGL((expand_dw_kernel<KK, SS, QS, 0, 1, 0>), grid, blk, smem, s, x, cin, we, be, w, bias, out,    \
                       pool_part, H, W, C, CW, T, tiles_x, gpb);                                                 \
    return hipGetLastError();                                                                                    \
  }
  // runtime-geometry kernels (shapes past B0's, or ct = 0)
  MMF_EDW(3, 2, 1) MMF_EDW(3, 1, 1) MMF_EDW(5, 2, 1) MMF_EDW(5, 1, 2) MMF_EDW(3, 2, 2)
  MMF_EDW(3, 1, 3)
#undef MMF_EDW
  return hipErrorInvalidValue;
}

hipError_t launch_se(const float* pool_part, int nchunks, float inv_hw, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* scale, int B, int C, int Csq, hipStream_t s,
                     bool precise) {
  if (C > 1280 || Csq > 64) return hipErrorInvalidValue;
  if (precise)
    hipLaunchKernelGGL(se_kernel<true>, dim3(B), dim3(SE_THREADS), 0, s, pool_part, nchunks, inv_hw, w1, b1, w2, b2,
                       scale, C, Csq);
  else
    hipLaunchKernelGGL(se_kernel<false>, dim3(B), dim3(SE_THREADS), 0, s, pool_part, nchunks, inv_hw, w1, b1, w2, b2,
                       scale, C, Csq);
  return hipGetLastError();
}

hipError_t launch_gap_classifier(const f16_t* x, int HW, int C, const float* w, const float* b, float* logits,
                                 float* score, int score_stride, int B, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;  // 16-B channel groups
  hipLaunchKernelGGL(gap_classifier_kernel, dim3(B), dim3(256), 0, s, x, HW, C, w, b, logits, score, score_stride);
  return hipGetLastError();
}
