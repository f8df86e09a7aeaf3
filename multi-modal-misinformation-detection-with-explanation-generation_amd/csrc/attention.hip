// Fused multi-head attention for the three encoders (head_dim 64, sequence <= 128; RoBERTa up to 512
// by attention_long_kernel below):
//   RoBERTa  L=128, 12 heads, key-padding mask          (TF roberta:158-251)
//   CLIP ViT L=50,  12 heads, no mask                    (TF clip:280-333)
//   CLIP txt L=77,   8 heads, causal + key-padding mask  (TF clip:494-590)
// One workgroup (4 waves) per (sequence, head).  K and V of the whole head live in LDS row-major
// ([key][64], 16-B chunks XOR-swizzled by key & 7, both staged with 16-B stores); each wave takes
// 16-query tiles:
//   S^T = K Q^T (v_mfma_f32_16x16x32_f16 with K as the A operand, Q fragments straight from
//         global/L2): each lane ends with 4 consecutive KEYS of one query
//   fp32 masked softmax in registers (a query's keys sit in 4 lanes -> 2 xor-shuffles)
//   O^T = V^T P^T with P^T taken straight from the softmax registers as the MFMA B operand: the
//         lane's 4 + 4 keys of a 32-key block are its two key tiles' values, so the contraction
//         runs over keys in that permuted order and V^T is read with the same permutation by
//         two ds_read_b64_tr_b16 (4 keys x 16 dims, transposed in the LDS read path) -- P never
//         round-trips through LDS, V is never transposed by scalar stores.  Each lane ends with 4 consecutive head
//         dims of one query (8-B stores).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int LMAX = 128;
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

MMF_DEV int kv_swz(int key, int kc) { return key * 64 + ((kc ^ (key & 7)) << 3); }

// LK = keys padded to the 32-deep PV k-step, a compile-time constant (32 / 64 / 96 / 128) so the
// key-tile loops carry no runtime bounds: the K-fragment reads of a query tile batch up ahead of
// its MFMAs instead of sitting in one basic block per key tile.
// CAUSAL (CLIP text) is compile-time too: the bidirectional encoders carry no per-score compare.
template <int LK, bool CAUSAL>
__global__ __launch_bounds__(256, 4) void attention_kernel(const f16_t* __restrict__ qkv, int ld,
                                                        const int32_t* __restrict__ mask, f16_t* __restrict__ out,
                                                        int ldo, int L, int H) {
  __shared__ __attribute__((aligned(16))) f16_t Ks[LK * 64];
  __shared__ __attribute__((aligned(16))) f16_t Vs[LK * 64];
  __shared__ __attribute__((aligned(16))) float kbias[256];  // (LK used; every thread stores its slot)

  const int bh = blockIdx.x, bi = bh / H, h = bh - bi * H;
  const int D = H * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const f16_t* base = qkv + (size_t)bi * L * ld;

  const int fr = lane & 15, fg = lane >> 4;
  const int nqt = (L + 15) >> 4;
  constexpr int NKT = LK / 16;
  // stage K and V (swizzled rows); zero the padded keys so 0 * pad stays finite.  All global loads
  // (K, V and this wave's Q fragments for both of its query tiles) are issued before the first
  // LDS store so the whole workgroup has its 48 KB in flight at once.
  constexpr int NIT = LK * 8 / 256, NQT = LMAX / 64;
  // Every load goes through buffer descriptors bounded at the sequence's L rows (and the mask's L
  // words): rows past L read as 0 with no branch or select around a load, so hipcc places no vmcnt
  // wait between them -- the workgroup pays one HBM round trip for K, V, Q and the mask together.
  const rsrc_t rseq = make_rsrc(base, (uint32_t)L * (uint32_t)ld * 2u);
  const rsrc_t rmask = make_rsrc(mask ? mask + (size_t)bi * L : nullptr, (uint32_t)L * 4u);
  const uint32_t mraw = __builtin_amdgcn_raw_buffer_load_b32(rmask, (uint32_t)tid * 4u, 0, 0);
  auto ld16 = [&](int row, int col) -> uint4 {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rseq, ((uint32_t)row * (uint32_t)ld + (uint32_t)col) * 2u, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  uint4 kr[NIT], vr[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int c = tid + i * 256, key = c >> 3, kc = c & 7;
    kr[i] = ld16(key, D + h * 64 + kc * 8);
    vr[i] = ld16(key, 2 * D + h * 64 + kc * 8);
  }
  // Q fragments: row q = qt*16 + fr, dims 32*ks + 8*fg .. +7, for qt = wave + 4*it
  f16x8 qfa[NQT][2];
#pragma unroll
  for (int it = 0; it < NQT; ++it)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qfa[it][ks] = as_f16x8(ld16((wave + 4 * it) * 16 + fr, h * 64 + ks * 32 + fg * 8));
  static_assert(LK <= 256, "one key-bias entry per thread");
  const bool kvalid = tid < L && (!mask || mraw != 0);
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int c = tid + i * 256, key = c >> 3, kc = c & 7;  // key < LK always
    *reinterpret_cast<uint4*>(Ks + kv_swz(key, kc)) = kr[i];
    *reinterpret_cast<uint4*>(Vs + kv_swz(key, kc)) = vr[i];
  }
  kbias[tid] = kvalid ? 0.f : -INFINITY;  // (no branch: the mask load stays with the others)
  __syncthreads();

  static_assert(NQT == 2, "two query tiles per wave");
  f16x8 qf[2] = {qfa[0][0], qfa[0][1]};
#pragma unroll 1
  for (int it = 0; it < NQT; ++it) {
    const int qt = wave + 4 * it;
    if (qt >= nqt) break;
    // S^T[key][q]: lane holds keys j*16 + fg*4 + r (r = 0..3) of query q = qt*16 + fr
    f32x4 s[NKT];
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int key = j * 16 + fr, kc = ks * 4 + fg;
        const f16x8 kf = as_f16x8(*reinterpret_cast<const uint4*>(Ks + kv_swz(key, kc)));
        s[j] = mfma16x16x32(kf, qf[ks], s[j]);
      }
    }
    // masked softmax over keys (fp32), scale 1/sqrt(64), in the exp2 domain: one FMA per score
    // (scale * log2 e and the mask bias) and one v_exp_f32 per exponential.  P stays unnormalised
    // (<= 1, rounded to fp16 for the PV MFMA) and O is divided by the row sum at the store.
    constexpr float kScaleLog2e = 0.125f * 1.44269504088896341f;
    const int qq = qt * 16 + fr;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
      const float4 kb = *reinterpret_cast<const float4*>(kbias + j * 16 + fg * 4);
      const float kbr[4] = {kb.x, kb.y, kb.z, kb.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = fmaf(s[j][r], kScaleLog2e, kbr[r]);
        if (CAUSAL && j * 16 + fg * 4 + r > qq) v = -INFINITY;
        s[j][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (mx == -INFINITY) mx = 0.f;  // every key masked: all exponentials 0, sum 0, output 0
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[j][r] - mx);
        s[j][r] = e;
        sum += e;
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = sum == 0.f ? 0.f : 1.0f / sum;
    // O^T[d][q] = sum_key V^T[d][key] P^T[key][q] over 32-key blocks; B operand of lane (fr, fg):
    // k-index 8fg + i <-> key 32kb + 4fg + i (i < 4, tile 2kb) / 32kb + 16 + 4fg + (i - 4) (tile 2kb+1)
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < LK / 32; ++kb) {
      {
        const uint4 pk = make_uint4(pack2h(s[2 * kb][0], s[2 * kb][1]), pack2h(s[2 * kb][2], s[2 * kb][3]),
                                    pack2h(s[2 * kb + 1][0], s[2 * kb + 1][1]),
                                    pack2h(s[2 * kb + 1][2], s[2 * kb + 1][3]));
        const f16x8 pf = as_f16x8(pk);
        // A operand V^T[d = dt*16 + fr][keys 32kb + 4fg + 0..3 | 32kb + 16 + 4fg + 0..3]: lane
        // 4q + p of each 16-lane group addresses key row (.. + q), dims dt*16 + 4p .. +3
        const int key0 = kb * 32 + fg * 4 + (fr >> 2), p = fr & 3;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int c = dt * 2 + (p >> 1), e = (p & 1) * 4;
          const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + kv_swz(key0, c) + e));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + kv_swz(key0 + 16, c) + e));
          const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
          o[dt] = mfma16x16x32(as_f16x8(make_uint4(l2.x, l2.y, h2.x, h2.y)), pf, o[dt]);
        }
      }
    }
    if (qq < L) {
      f16_t* dst = out + ((size_t)bi * L + qq) * ldo + h * 64 + fg * 4;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<uint2*>(dst + dt * 16) =
            make_uint2(pack2h(o[dt][0] * inv, o[dt][1] * inv), pack2h(o[dt][2] * inv, o[dt][3] * inv));
    }
    qf[0] = qfa[1][0];
    qf[1] = qfa[1][1];
  }
}

// Sequences of 129..512 tokens (RoBERTa truncates at 512, misinfo_forensics.py:327-333): the whole
// head's K and V (up to 2 x 64 KB) stay resident in LDS (one workgroup per CU) and each 16-query
// tile walks the keys in 128-key chunks with an online softmax (running max / sum per query, O
// rescaled when the max grows).  The S^T / P^T-in-registers / transposed-V formulation is the one
// of attention_kernel above; P is rounded to fp16 unnormalised (<= 1) and O divided by the sum at
// the end.
constexpr int LLONG = 512, KCH = 128;

__global__ __launch_bounds__(256) void attention_long_kernel(const f16_t* __restrict__ qkv, int ld,
                                                             const int32_t* __restrict__ mask,
                                                             f16_t* __restrict__ out, int ldo, int L, int H,
                                                             int causal) {
  __shared__ __attribute__((aligned(16))) f16_t Ks[LLONG * 64];
  __shared__ __attribute__((aligned(16))) f16_t Vs[LLONG * 64];
  __shared__ __attribute__((aligned(16))) float kbias[LLONG];

  const int bh = blockIdx.x, bi = bh / H, h = bh - bi * H;
  const int D = H * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Lk = (L + 31) & ~31;
  const f16_t* base = qkv + (size_t)bi * L * ld;
  const int fr = lane & 15, fg = lane >> 4;
  const int nqt = (L + 15) >> 4;

  // stage K and V in batches of 4 x 16 B per thread (loads of a batch issued before its stores)
  for (int c0 = 0; c0 < Lk * 8; c0 += 4 * 256) {
    uint4 kr[4], vr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + tid + i * 256, key = c >> 3, kc = c & 7;
      kr[i] = make_uint4(0, 0, 0, 0);
      vr[i] = make_uint4(0, 0, 0, 0);
      if (key < L) {
        kr[i] = *reinterpret_cast<const uint4*>(base + (size_t)key * ld + D + h * 64 + kc * 8);
        vr[i] = *reinterpret_cast<const uint4*>(base + (size_t)key * ld + 2 * D + h * 64 + kc * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + tid + i * 256, key = c >> 3, kc = c & 7;
      if (key < Lk) {
        *reinterpret_cast<uint4*>(Ks + kv_swz(key, kc)) = kr[i];
        *reinterpret_cast<uint4*>(Vs + kv_swz(key, kc)) = vr[i];
      }
    }
  }
  for (int k = tid; k < Lk; k += 256)
    kbias[k] = (k < L && (!mask || mask[(size_t)bi * L + k])) ? 0.f : -INFINITY;
  __syncthreads();

#pragma unroll 1
  for (int qt = wave; qt < nqt; qt += 4) {
    const int qq = qt * 16 + fr;
    f16x8 qf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qq < L) v = *reinterpret_cast<const uint4*>(base + (size_t)qq * ld + h * 64 + ks * 32 + fg * 8);
      qf[ks] = as_f16x8(v);
    }
    float m = -INFINITY, sum = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k0 = 0; k0 < Lk; k0 += KCH) {
      const int nkt = min(KCH, Lk - k0) >> 4;  // 16-key tiles in this chunk (even: Lk % 32 == 0)
      f32x4 s[KCH / 16];
#pragma unroll
      for (int j = 0; j < KCH / 16; ++j) {
        s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (j < nkt) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const int key = k0 + j * 16 + fr, kc = ks * 4 + fg;
            const f16x8 kf = as_f16x8(*reinterpret_cast<const uint4*>(Ks + kv_swz(key, kc)));
            s[j] = mfma16x16x32(kf, qf[ks], s[j]);
          }
        }
      }
      float mc = -INFINITY;
#pragma unroll
      for (int j = 0; j < KCH / 16; ++j) {
        if (j < nkt) {
          const float4 kb = *reinterpret_cast<const float4*>(kbias + k0 + j * 16 + fg * 4);
          const float kbr[4] = {kb.x, kb.y, kb.z, kb.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = s[j][r] * 0.125f + kbr[r];
            if (causal && k0 + j * 16 + fg * 4 + r > qq) v = -INFINITY;
            s[j][r] = v;
            mc = fmaxf(mc, v);
          }
        }
      }
      mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m, mc);
      const float alpha = (m == -INFINITY) ? 0.f : __expf(m - mn);  // m == -inf: nothing accumulated yet
      m = mn;
      float cs = 0.f;
#pragma unroll
      for (int j = 0; j < KCH / 16; ++j) {
        if (j < nkt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = (mn == -INFINITY) ? 0.f : __expf(s[j][r] - mn);
            s[j][r] = e;
            cs += e;
          }
        }
      }
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      sum = sum * alpha + cs;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
#pragma unroll
      for (int kb = 0; kb < KCH / 32; ++kb) {
        if (2 * kb < nkt) {
          const uint4 pk = make_uint4(pack2h(s[2 * kb][0], s[2 * kb][1]), pack2h(s[2 * kb][2], s[2 * kb][3]),
                                      pack2h(s[2 * kb + 1][0], s[2 * kb + 1][1]),
                                      pack2h(s[2 * kb + 1][2], s[2 * kb + 1][3]));
          const f16x8 pf = as_f16x8(pk);
          const int key0 = k0 + kb * 32 + fg * 4 + (fr >> 2), p = fr & 3;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const int c = dt * 2 + (p >> 1), e = (p & 1) * 4;
            const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + kv_swz(key0, c) + e));
            const i16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + kv_swz(key0 + 16, c) + e));
            const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
            o[dt] = mfma16x16x32(as_f16x8(make_uint4(l2.x, l2.y, h2.x, h2.y)), pf, o[dt]);
          }
        }
      }
    }
    if (qq < L) {
      const float inv = sum == 0.f ? 0.f : 1.0f / sum;
      f16_t* dst = out + ((size_t)bi * L + qq) * ldo + h * 64 + fg * 4;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<uint2*>(dst + dt * 16) =
            make_uint2(pack2h(o[dt][0] * inv, o[dt][1] * inv), pack2h(o[dt][2] * inv, o[dt][3] * inv));
    }
  }
}


// One query per sequence (the last encoder layer: only the RoBERTa CLS row / the CLIP CLS or EOS row
// is consumed after it, so the other queries of that layer are dead work).  One wave per (sequence,
// head): lanes over keys for the scores (fp32 dot products of 64 dims, ascending), wave max / sum,
// then lanes over the 64 head dims for O = sum_j p_j v_j (keys ascending, fp32), stored fp16.
// q: [B][ldq] fp32 (head h at h * 64); K / V: the QKV rows of the sequence (row b * L + j, columns
// koff + h * 64 / voff + h * 64); a masked key (mask 0, or past qpos[b] when causal) is excluded.
__global__ __launch_bounds__(256) void attention_q1_kernel(const float* __restrict__ q, int ldq,
                                                           const f16_t* __restrict__ qkv, int ld, int koff, int voff,
                                                           const int32_t* __restrict__ mask,
                                                           const int32_t* __restrict__ qpos, f16_t* __restrict__ out,
                                                           int ldo, int B, int L, int H) {
  __shared__ float ps[4][LLONG];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + wave;
  if (wid >= B * H) return;  // wave-uniform
  const int bi = wid / H, h = wid - bi * H;
  float qf[64];  // the query in fp32 (the skinny Q GEMM's fp32 output: no fp16 rounding of q)
  {
    const float4* qp = reinterpret_cast<const float4*>(q + (size_t)bi * ldq + h * 64);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float4 v = qp[c];
      qf[c * 4] = v.x;
      qf[c * 4 + 1] = v.y;
      qf[c * 4 + 2] = v.z;
      qf[c * 4 + 3] = v.w;
    }
  }
  const int last = qpos ? qpos[bi] : L - 1;  // causal: keys <= the query position
  float m = -INFINITY;
  // two keys per lane per trip (j, j + 64): both K rows' loads in flight before either dot product
  for (int j0 = lane; j0 < L; j0 += 128) {
    uint4 kv[2][8];
    bool valid[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = j0 + 64 * t;
      valid[t] = j < L && (!mask || mask[(size_t)bi * L + j] != 0) && j <= last;
      const uint4* kp = reinterpret_cast<const uint4*>(qkv + ((size_t)bi * L + min(j, L - 1)) * ld + koff + h * 64);
#pragma unroll
      for (int c = 0; c < 8; ++c) kv[t][c] = kp[c];
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = j0 + 64 * t;
      if (j >= L) break;
      float sdot = -INFINITY;
      if (valid[t]) {
        float a = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const uint32_t w[4] = {kv[t][c].x, kv[t][c].y, kv[t][c].z, kv[t][c].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a = fmaf(qf[c * 8 + e * 2], lo_h(w[e]), a);
            a = fmaf(qf[c * 8 + e * 2 + 1], hi_h(w[e]), a);
          }
        }
        sdot = a * 0.125f;  // 1 / sqrt(64)
      }
      ps[wave][j] = sdot;
      m = fmaxf(m, sdot);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float sum = 0.f;
  for (int j = lane; j < L; j += 64) {
    const float sv = ps[wave][j];
    const float e = sv == -INFINITY ? 0.f : __expf(sv - m);
    ps[wave][j] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const f16_t* vp = qkv + (size_t)bi * L * ld + voff + h * 64 + lane;
  float o = 0.f;
  // keys in chunks of 32: the chunk's V loads all in flight, then the same ascending-j fmaf chain
  const int jend = min(last + 1, L);
  for (int jb = 0; jb < jend; jb += 32) {
    f16_t vv[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) vv[u] = vp[(size_t)min(jb + u, jend - 1) * ld];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (jb + u < jend) o = fmaf(ps[wave][jb + u], h2f(vv[u]), o);
  }
  out[(size_t)bi * ldo + h * 64 + lane] = f2h(sum == 0.f ? 0.f : o / sum);  // (non-finite sum: propagates)
}

}  // namespace

hipError_t launch_attention_q1(const float* q, int ldq, const f16_t* qkv, int ld, int koff, int voff,
                               const int32_t* mask, const int32_t* qpos, f16_t* out, int ldo, int B, int L, int H,
                               hipStream_t s) {
  if (L <= 0 || L > LLONG || (ldq & 3) || (ld & 7) || (koff & 7) || (voff & 7)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(attention_q1_kernel, dim3((B * H + 3) / 4), dim3(256), 0, s, q, ldq, qkv, ld, koff, voff, mask,
                     qpos, out, ldo, B, L, H);
  return hipGetLastError();
}

hipError_t launch_attention(const f16_t* qkv, int ldqkv, const int32_t* mask, f16_t* out, int ldo, int B, int L,
                            int H, int causal, hipStream_t s) {
  if (L <= 0 || L > LLONG || (ldqkv & 7) || (ldo & 3)) return hipErrorInvalidValue;
  if (L > LMAX) {
    hipLaunchKernelGGL(attention_long_kernel, dim3(B * H), dim3(256), 0, s, qkv, ldqkv, mask, out, ldo, L, H,
                       causal);
    return hipGetLastError();
  }
#define MMF_ATTN(LK)                                                                                              \
  if (causal) hipLaunchKernelGGL((attention_kernel<LK, true>), dim3(B * H), dim3(256), 0, s, qkv, ldqkv, mask, out, ldo, L, H); \
  else hipLaunchKernelGGL((attention_kernel<LK, false>), dim3(B * H), dim3(256), 0, s, qkv, ldqkv, mask, out, ldo, L, H)
  switch ((L + 31) >> 5) {  // keys padded to 32
    case 1: MMF_ATTN(32); break;
    case 2: MMF_ATTN(64); break;
    case 3: MMF_ATTN(96); break;
    default: MMF_ATTN(128);
  }
#undef MMF_ATTN
  return hipGetLastError();
}
