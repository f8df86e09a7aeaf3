// RoBERTa precise mode (option text_hilo = 2): the text tower for checkpoints
// whose LayerNorms amplify the fp16 rounding of the GEMM operands themselves (one channel
// dominating every LayerNorm, gamma ~7: DESIGN.md §4), where no stream layout holds 1e-3.
//
// Every GEMM runs on the production fp16 MFMA kernel with ~22-bit operands, by concatenating along K:
//   A3 = [A_hi | A_lo | A_hi]  (hi = fp16(a), lo = fp16(a - hi)),  W3 = [W_hi | W_hi | W_lo]
//   A3 . W3^T = A_hi W_hi^T + A_lo W_hi^T + A_hi W_lo^T   (the lo . lo term, ~2^-22, dropped)
// with fp32 accumulation -- three fp16 products per MAC, 3x the K loop, no new GEMM kernel.  The
// residual stream, the branch outputs, LayerNorm and the attention stay fp32 (this file's kernels):
//   split3_kernel      fp32 rows -> A3 rows (the GEMM operand of the stream, ctx and the FFN hidden)
//   attention32_kernel fp32 q / k / v -> fp32 ctx, exact softmax (expf), keys in chunks of 32
#include "common.h"
#include "kernels.h"

namespace {

// out[r][0:C] = hi, out[r][C:2C] = lo, out[r][2C:3C] = hi; one thread per 4 consecutive columns.
// LO = false: hi alone (the consumer GEMM reads the first third: text_prec_mask bit clear)
template <bool LO>
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, int ldx, f16_t* __restrict__ out,
                                                     int rows, int C) {
  const int q = C >> 2;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (size_t)rows * q) return;
  const int r = (int)(idx / q), c = (int)(idx - (size_t)r * q) * 4;
  const float4 v = *reinterpret_cast<const float4*>(x + (size_t)r * ldx + c);
  const uint2 hi = make_uint2(pack2h(v.x, v.y), pack2h(v.z, v.w));
  const uint2 lo = make_uint2(pack2h(v.x - lo_h(hi.x), v.y - hi_h(hi.x)), pack2h(v.z - lo_h(hi.y), v.w - hi_h(hi.y)));
  f16_t* o = out + (size_t)r * 3 * C + c;
  *reinterpret_cast<uint2*>(o) = hi;
  if constexpr (LO) {
    *reinterpret_cast<uint2*>(o + C) = lo;
    *reinterpret_cast<uint2*>(o + 2 * C) = hi;
  }
}

// fp32 multi-head attention, head dim 64, any L (RoBERTa <= 512): one thread per query, 128 queries
// per block; the block walks the keys in chunks of 32 (K and V of the chunk in LDS, read as
// broadcasts) with an online softmax: per chunk the scores s_j = (q . k_j) / 8 + mask_j, the
// running max m, o and l rescaled by exp(m_old - m_new), then o += exp(s_j - m) v_j.  qkv: fp32
// [B*L][ld] with q at column h*64, k at koff + h*64, v at voff + h*64; out fp32 [B*L][ldo].
constexpr int A32_Q = 128, A32_K = 32;
__global__ __launch_bounds__(A32_Q) void attention32_kernel(const float* __restrict__ qkv, int ld, int koff, int voff,
                                                            const int32_t* __restrict__ mask, float* __restrict__ out,
                                                            int ldo, int L, int H, f16_t* __restrict__ out3, int with_lo) {
  __shared__ __attribute__((aligned(16))) float Ks[A32_K][64];
  __shared__ __attribute__((aligned(16))) float Vs[A32_K][64];
  __shared__ float kb[A32_K];
  const int bh = blockIdx.x, bi = bh / H, h = bh - bi * H;
  const int tid = threadIdx.x;
  const int qi = blockIdx.y * A32_Q + tid;
  const int qc = qi < L ? qi : L - 1;  // (threads past L compute a clamped row, never stored)
  const float* base = qkv + (size_t)bi * L * ld;
  // q and o as 32 pairs: every dot-product / accumulation step is one packed fp32 FMA (v_pk_fma_f32,
  // two lanes' worth of fp32 FMAs per issue; the even / odd columns of the q.k dot product in two
  // accumulators, added at the end)
  f32x2_t q[32], o[32];
  {
    const float4* qp = reinterpret_cast<const float4*>(base + (size_t)qc * ld + h * 64);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float4 v = qp[c];
      q[2 * c] = (f32x2_t){v.x, v.y} * 0.125f;  // 1 / sqrt(64): exact
      q[2 * c + 1] = (f32x2_t){v.z, v.w} * 0.125f;
    }
  }
#pragma unroll
  for (int d = 0; d < 32; ++d) o[d] = (f32x2_t){0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += A32_K) {
    __syncthreads();  // the previous chunk's readers are done
    for (int e = tid; e < A32_K * 16; e += A32_Q) {  // 32 keys x 16 float4 of K and of V
      const int j = e >> 4, c = (e & 15) * 4, key = k0 + j;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (key < L) {
        kv = *reinterpret_cast<const float4*>(base + (size_t)key * ld + koff + h * 64 + c);
        vv = *reinterpret_cast<const float4*>(base + (size_t)key * ld + voff + h * 64 + c);
      }
      *reinterpret_cast<float4*>(&Ks[j][c]) = kv;
      *reinterpret_cast<float4*>(&Vs[j][c]) = vv;
    }
    if (tid < A32_K) {
      const int key = k0 + tid;
      kb[tid] = (key < L && (!mask || mask[(size_t)bi * L + key] != 0)) ? 0.f : -INFINITY;
    }
    __syncthreads();
    float s[A32_K];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < A32_K; ++j) {
      f32x2_t a2 = {0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float4 kv = *reinterpret_cast<const float4*>(&Ks[j][4 * c]);
        a2 = __builtin_elementwise_fma(q[2 * c], (f32x2_t){kv.x, kv.y}, a2);
        a2 = __builtin_elementwise_fma(q[2 * c + 1], (f32x2_t){kv.z, kv.w}, a2);
      }
      s[j] = (a2.x + a2.y) + kb[j];
      cm = fmaxf(cm, s[j]);
    }
    const float mn = fmaxf(m, cm);
    if (mn == -INFINITY) continue;  // every key so far masked (a later chunk may hold valid ones)
    const float sc = expf(m - mn);  // (m = -inf: 0)
    l *= sc;
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = o[d] * sc;
#pragma unroll
    for (int j = 0; j < A32_K; ++j) {
      const float p = expf(s[j] - mn);  // masked: exp(-inf) = 0
      l += p;
      const f32x2_t pp = {p, p};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float4 vv = *reinterpret_cast<const float4*>(&Vs[j][4 * c]);
        o[2 * c] = __builtin_elementwise_fma(pp, (f32x2_t){vv.x, vv.y}, o[2 * c]);
        o[2 * c + 1] = __builtin_elementwise_fma(pp, (f32x2_t){vv.z, vv.w}, o[2 * c + 1]);
      }
    }
    m = mn;
  }
  if (qi >= L) return;
  const float inv = l == 0.f ? 0.f : 1.0f / l;  // (a non-finite sum propagates)
  if (out3) {  // the out-projection's operand row, split as split3_kernel does (fused: no fp32 ctx pass)
    const int D = H * 64;
    f16_t* o3 = out3 + ((size_t)bi * L + qi) * 3 * D + h * 64;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float v0 = o[2 * c].x * inv, v1 = o[2 * c].y * inv, v2 = o[2 * c + 1].x * inv, v3 = o[2 * c + 1].y * inv;
      const uint2 hi = make_uint2(pack2h(v0, v1), pack2h(v2, v3));
      *reinterpret_cast<uint2*>(o3 + 4 * c) = hi;
      if (with_lo) {
        *reinterpret_cast<uint2*>(o3 + D + 4 * c) =
            make_uint2(pack2h(v0 - lo_h(hi.x), v1 - hi_h(hi.x)), pack2h(v2 - lo_h(hi.y), v3 - hi_h(hi.y)));
        *reinterpret_cast<uint2*>(o3 + 2 * D + 4 * c) = hi;
      }
    }
    return;
  }
  float4* op = reinterpret_cast<float4*>(out + ((size_t)bi * L + qi) * ldo + h * 64);
#pragma unroll
  for (int c = 0; c < 16; ++c)
    op[c] = make_float4(o[2 * c].x * inv, o[2 * c].y * inv, o[2 * c + 1].x * inv, o[2 * c + 1].y * inv);
}

}  // namespace

hipError_t launch_split3(const float* x, int ldx, f16_t* out, int rows, int C, hipStream_t s, int with_lo) {
  if (rows <= 0) return hipSuccess;
  if ((C & 3) || (ldx & 3)) return hipErrorInvalidValue;
  const size_t n = (size_t)rows * (C / 4);
  if (with_lo)
    hipLaunchKernelGGL(split3_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, out, rows, C);
  else
    hipLaunchKernelGGL(split3_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, out, rows, C);
  return hipGetLastError();
}

hipError_t launch_attention32(const float* qkv, int ld, int koff, int voff, const int32_t* mask, float* out, int ldo,
                              int B, int L, int H, hipStream_t s, f16_t* out3, int with_lo) {
  if (B <= 0 || L <= 0) return hipSuccess;
  if ((ld & 3) || (koff & 3) || (voff & 3) || (ldo & 3)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(attention32_kernel, dim3(B * H, (L + A32_Q - 1) / A32_Q), dim3(A32_Q), 0, s, qkv, ld, koff, voff,
                     mask, out, ldo, L, H, out3, with_lo);
  return hipGetLastError();
}
