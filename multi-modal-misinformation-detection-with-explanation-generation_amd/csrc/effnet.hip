// EfficientNet-B0 (torchvision spec, eval) pieces that are not 1x1 convolutions.  Activations are
// NHWC bf16 so channels are the contiguous, coalesced axis; every BatchNorm is folded into the
// preceding convolution's weights/bias at load time (mmf_finalize).  These kernels are HBM-bound
// (SURVEY.md §8d): each reads its input once and writes its output once.
//   stem      uint8 HWC -> ImageNet normalise -> conv3x3 s2 (3->32) + BN + SiLU
//   dwconv    depthwise kxk (k=3,5; s=1,2) + BN + SiLU, with the SE global-average-pool partial
//             sums of the fp32 outputs (deterministic per-chunk partials, no atomics)
//   se        mean -> fc1 + SiLU -> fc2 + sigmoid -> per-(image, channel) scale (applied inside
//             the project GEMM's A load)
//   gap_cls   global average pool of the head conv + Linear(1280, 2) + softmax[:, 1]
#include "common.h"
#include "kernels.h"

namespace {

// One thread per output pixel, all 32 channels; weights transposed in LDS to [tap][channel] so
// every tap is 8 broadcast float4 reads.  ToTensor + Normalize folded into one FMA per input.
// F32 = true: input is an already-normalised fp32 NCHW tensor (detector.forward_image signature,
// misinfo_forensics.py:102-104) instead of uint8 HWC pixels.
template <bool F32>
__global__ __launch_bounds__(256) void stem_kernel(const void* src, const float* w, const float* bias, bf16_t* out,
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
        const float v = F32 ? xf[(((size_t)bi * 3 + c) * 224 + iy) * 224 + ix] : fmaf((float)p[c], sc[c], of[c]);
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
  uint4* dst = reinterpret_cast<uint4*>(out + pix * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_apply(acc[q * 8 + j], ACT_SILU);
    dst[q] = make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]), pack2bf(o[6], o[7]));
  }
}

// grid (chunks, C/8/CGT, B); block = PL pixel lanes x CGT channel groups of 8
template <int K>
__global__ __launch_bounds__(256) void dwconv_kernel(const bf16_t* in, const float* w, const float* bias,
                                                     bf16_t* out, float* pool_part, int H, int W, int C,
                                                     int stride, int CGT, int PL, int pix_per_chunk) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sw = smem;                    // [K*K][CGT*8]
  float* sb = sw + K * K * CGT * 8;    // [CGT*8]
  float* red = sb + CGT * 8;           // [PL][CGT*8]
  const int tid = threadIdx.x;
  const int ncw = CGT * 8, c0 = blockIdx.y * ncw;
  const int bi = blockIdx.z;
  for (int i = tid; i < K * K * ncw; i += blockDim.x) {
    const int t = i / ncw, c = i % ncw;
    sw[i] = w[(size_t)(c0 + c) * K * K + t];
  }
  for (int i = tid; i < ncw; i += blockDim.x) sb[i] = bias[c0 + i];
  __syncthreads();
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;  // pad = (K-1)/2
  const int pad = (K - 1) / 2;
  const int cgl = tid % CGT, pl = tid / CGT;
  const int cl = cgl * 8;
  float psum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int p_begin = blockIdx.x * pix_per_chunk;
  const int p_end = min(p_begin + pix_per_chunk, Ho * Wo);
  if (pl < PL) {
    for (int p = p_begin + pl; p < p_end; p += PL) {
      const int oy = p / Wo, ox = p - oy * Wo;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = sb[cl + j];
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int iy = oy * stride - pad + ky;
        if (iy < 0 || iy >= H) continue;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int ix = ox * stride - pad + kx;
          if (ix < 0 || ix >= W) continue;
          const uint4 v = *reinterpret_cast<const uint4*>(in + (((size_t)bi * H + iy) * W + ix) * C + c0 + cl);
          const float* ww = sw + (ky * K + kx) * ncw + cl;
          acc[0] = fmaf(lo_bf(v.x), ww[0], acc[0]); acc[1] = fmaf(hi_bf(v.x), ww[1], acc[1]);
          acc[2] = fmaf(lo_bf(v.y), ww[2], acc[2]); acc[3] = fmaf(hi_bf(v.y), ww[3], acc[3]);
          acc[4] = fmaf(lo_bf(v.z), ww[4], acc[4]); acc[5] = fmaf(hi_bf(v.z), ww[5], acc[5]);
          acc[6] = fmaf(lo_bf(v.w), ww[6], acc[6]); acc[7] = fmaf(hi_bf(v.w), ww[7], acc[7]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j] = act_apply(acc[j], ACT_SILU);
        psum[j] += acc[j];
      }
      *reinterpret_cast<uint4*>(out + (((size_t)bi * Ho + oy) * Wo + ox) * C + c0 + cl) =
          make_uint4(pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3]), pack2bf(acc[4], acc[5]),
                     pack2bf(acc[6], acc[7]));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[pl * ncw + cl + j] = psum[j];
  }
  __syncthreads();
  // fixed-order reduction over pixel lanes -> one partial per (image, chunk, channel)
  for (int c = tid; c < ncw; c += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < PL; ++q) s += red[q * ncw + c];
    pool_part[((size_t)bi * gridDim.x + blockIdx.x) * C + c0 + c] = s;
  }
}

// One block per image.  w2t is fc2's weight transposed to [Csq][C] (packed at load) so every
// k-step of both matvecs is one coalesced row read; fc1 partial dots are spread over all waves.
__global__ __launch_bounds__(256) void se_kernel(const float* pool_part, int nchunks, float inv_hw, const float* w1,
                                                 const float* b1, const float* w2t, const float* b2, float* scale,
                                                 int C, int Csq) {
  __shared__ float pooled[1280];
  __shared__ float s1[64];
  const int bi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* pp = pool_part + (size_t)bi * nchunks * C;
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < nchunks; ++k) s += pp[(size_t)k * C + c];
    pooled[c] = s * inv_hw;
  }
  __syncthreads();
  for (int o = wave; o < Csq; o += 4) {
    const float* wr = w1 + (size_t)o * C;
    float a0 = 0.f, a1 = 0.f;
    int c = lane;
    for (; c + 64 < C; c += 128) {
      a0 = fmaf(wr[c], pooled[c], a0);
      a1 = fmaf(wr[c + 64], pooled[c + 64], a1);
    }
    if (c < C) a0 = fmaf(wr[c], pooled[c], a0);
    const float a = wave_sum(a0 + a1);
    if (lane == 0) s1[o] = act_apply(a + b1[o], ACT_SILU);
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float a = b2[c];
    for (int j = 0; j < Csq; ++j) a = fmaf(w2t[(size_t)j * C + c], s1[j], a);
    scale[(size_t)bi * C + c] = 1.0f / (1.0f + expf(-a));
  }
}

__global__ __launch_bounds__(256) void gap_classifier_kernel(const bf16_t* x, int HW, int C, const float* w,
                                                             const float* b, float* logits, float* score,
                                                             int score_stride) {
  __shared__ float red[2][4];
  const int bi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float l0 = 0.f, l1 = 0.f;
  const float inv = 1.0f / (float)HW;
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += bf2f(x[((size_t)bi * HW + p) * C + c]);
    s *= inv;
    l0 = fmaf(w[c], s, l0);
    l1 = fmaf(w[C + c], s, l1);
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

hipError_t launch_effnet_stem(const uint8_t* img, const float* w, const float* bias, bf16_t* out, int B,
                              hipStream_t s) {
  const size_t total = (size_t)B * 112 * 112;
  hipLaunchKernelGGL(stem_kernel<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const void*)img, w,
                     bias, out, B);
  return hipGetLastError();
}

hipError_t launch_effnet_stem_f32(const float* x, const float* w, const float* bias, bf16_t* out, int B,
                                  hipStream_t s) {
  const size_t total = (size_t)B * 112 * 112;
  hipLaunchKernelGGL(stem_kernel<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const void*)x, w,
                     bias, out, B);
  return hipGetLastError();
}

static void dw_geometry(int H, int W, int C, int stride, int* CGT_, int* PL_, int* ppc_, int* nchunks_) {
  const int CG = C / 8;
  int CGT = 1;
  for (int cand : {8, 6, 4, 3, 2, 1})
    if (CG % cand == 0) { CGT = cand; break; }
  const int PL = 256 / CGT;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int ppc = PL * 8;  // ~8 output pixels per thread per chunk
  *CGT_ = CGT; *PL_ = PL; *ppc_ = ppc; *nchunks_ = (Ho * Wo + ppc - 1) / ppc;
}

int dwconv_nchunks(int H, int W, int C, int stride) {
  int a, b, c, n;
  dw_geometry(H, W, C, stride, &a, &b, &c, &n);
  return n;
}

hipError_t launch_dwconv(const bf16_t* in, const float* w, const float* bias, bf16_t* out, float* pool_part, int B,
                         int H, int W, int C, int k, int stride, int* nchunks_out, hipStream_t s) {
  if (C & 7) return hipErrorInvalidValue;
  const int CG = C / 8;
  int CGT, PL, ppc, nchunks;
  dw_geometry(H, W, C, stride, &CGT, &PL, &ppc, &nchunks);
  *nchunks_out = nchunks;
  const size_t smem = (size_t)(k * k * CGT * 8 + CGT * 8 + PL * CGT * 8) * sizeof(float);
  const dim3 grid(nchunks, CG / CGT, B), blk(PL * CGT);
  if (k == 3)
    hipLaunchKernelGGL(dwconv_kernel<3>, grid, blk, smem, s, in, w, bias, out, pool_part, H, W, C, stride, CGT, PL, ppc);
  else if (k == 5)
    hipLaunchKernelGGL(dwconv_kernel<5>, grid, blk, smem, s, in, w, bias, out, pool_part, H, W, C, stride, CGT, PL, ppc);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_se(const float* pool_part, int nchunks, float inv_hw, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* scale, int B, int C, int Csq, hipStream_t s) {
  if (C > 1280 || Csq > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(se_kernel, dim3(B), dim3(256), 0, s, pool_part, nchunks, inv_hw, w1, b1, w2, b2, scale, C, Csq);
  return hipGetLastError();
}

hipError_t launch_gap_classifier(const bf16_t* x, int HW, int C, const float* w, const float* b, float* logits,
                                 float* score, int score_stride, int B, hipStream_t s) {
  hipLaunchKernelGGL(gap_classifier_kernel, dim3(B), dim3(256), 0, s, x, HW, C, w, b, logits, score, score_stride);
  return hipGetLastError();
}
