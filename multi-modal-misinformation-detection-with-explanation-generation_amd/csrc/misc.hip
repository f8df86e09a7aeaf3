// Small fp32 kernels at the ends of the path: the RoBERTa dual heads, the FusionJudge MLP with
// verdict / explanation rule, cosine rows, and the Truth-Vault search (similarities + top-k).
// These are latency/L2-bound: they run in exact fp32 like the reference.
#include "common.h"
#include "kernels.h"

namespace {

// misinfo_forensics.py:57-69, 97-98, 342-347: two Linear(768,256)-ReLU-Linear(256,2) heads on the
// CLS row, softmax[:, 1].  Block = 4 rows x ONE head (blockIdx.y: 0 = ai, 1 = misinfo), so a block
// streams 0.75 MB of W1 instead of 1.5 MB (the per-block L2 stream is what bounds this kernel at
// the end of the RoBERTa tower); W1 stored transposed [768][256] so a k-step of the 256 hidden
// units reads one coalesced 1-KB row.  Per head the arithmetic order is unchanged.
__global__ __launch_bounds__(1024) void text_heads_kernel(const float* x, int row_stride, const float* w1a,
                                                         const float* b1a, const float* w2a, const float* b2a,
                                                         const float* w1m, const float* b1m, const float* w2m,
                                                         const float* b2m, float* ai_logits, float* mi_logits,
                                                         float* scores, int score_stride, int B, const int* ovf) {
  // 1024 threads: hidden unit h = tid % 256 of K-slice ks = tid / 256 (192 inputs each), so each
  // thread's dependent load/FMA chain is a quarter of the 768; slices combined in fixed order.
  constexpr int KS = 4, KL = 768 / KS;
  __shared__ float xs[4][768];
  __shared__ float hp[KS][4][256];  // [slice][row][hidden] partial sums
  __shared__ float red[4][4][2];    // [wave][row][o]
  const int tid = threadIdx.x, r0 = blockIdx.x * 4, h = tid & 255, ks = tid >> 8, head = blockIdx.y;
  const float* w1h = head ? w1m : w1a;
  const float* b1 = head ? b1m : b1a;
  const float* w2 = head ? w2m : w2a;
  const float* b2 = head ? b2m : b2a;
  float* logits = head ? mi_logits : ai_logits;
  for (int i = tid; i < 4 * 768; i += 1024) {
    const int r = i / 768, c = i % 768;
    xs[r][c] = (r0 + r < B) ? x[(size_t)(r0 + r) * row_stride + c] : 0.f;
  }
  __syncthreads();
  {
    const float* w1 = w1h + (size_t)ks * KL * 256 + h;
    float hsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k = 0; k < KL; ++k) {
      const float w = w1[(size_t)k * 256];
#pragma unroll
      for (int r = 0; r < 4; ++r) hsum[r] = fmaf(w, xs[r][ks * KL + k], hsum[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) hp[ks][r][h] = hsum[r];
  }
  __syncthreads();
  if (tid < 256) {  // waves 0-3: hidden units -> ReLU -> the 2 output logits per row
    float part[4][2];
    const float w20 = w2[h], w21 = w2[256 + h], bb = b1[h];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float hs = hp[0][r][h];
#pragma unroll
      for (int q = 1; q < KS; ++q) hs += hp[q][r][h];
      const float hv = fmaxf(hs + bb, 0.f);
      part[r][0] = hv * w20;
      part[r][1] = hv * w21;
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        const float v = wave_sum(part[r][o]);
        if (lane == 0) red[wave][r][o] = v;
      }
  }
  __syncthreads();
  if (tid < 4 && r0 + tid < B) {
    const int r = tid, row = r0 + r;
    float l[2];
#pragma unroll
    for (int o = 0; o < 2; ++o) l[o] = red[0][r][o] + red[1][r][o] + red[2][r][o] + red[3][r][o];
    l[0] += b2[0]; l[1] += b2[1];
    if (ovf && ovf[row]) l[0] = l[1] = __builtin_nanf("");  // the sequence's fp16 stream overflowed (norm.hip)
    if (logits) { logits[row * 2] = l[0]; logits[row * 2 + 1] = l[1]; }
    if (scores) {  // softmax(l)[1] = exp(l1 - m) / (exp(l0 - m) + exp(l1 - m))
      const float m = fmaxf(l[0], l[1]);
      const float e0 = expf(l[0] - m), e1 = expf(l[1] - m);
      scores[(size_t)row * score_stride + head] = e1 / (e0 + e1);
    }
  }
}

// misinfo_forensics.py:575-615 (fusion_verdict) + 742-765 (fallback explanation rule cascade).
// One wave per row (it sits at the very end of the step, after the towers join, so its latency is
// fully exposed: a thread per row walked ~2.4k dependent FMAs, ~17 us).  Lane o computes hidden
// unit o of Linear(5,64), lanes < 32 the units of Linear(64,32) from the wave's LDS row, lane 0
// the two logits; every dot product keeps the ascending-index fmaf order of the scalar form.
__global__ __launch_bounds__(256) void fusion_kernel(const float* x5, const float* w0, const float* b0,
                                                     const float* w3, const float* b3, const float* w5,
                                                     const float* b5, float* probs, int32_t* verdict, float* conf,
                                                     int32_t* rule, int B) {
  __shared__ float sw0[64 * 5], sb0[64], sw3[32 * 65], sb3[32], sw5[64], sb5[2];
  __shared__ float hs[4][64], h2[4][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = blockIdx.x * 4 + wave;
  const bool live = row < B;
  float x[5];  // (issued before the weight staging: one load latency for both)
#pragma unroll
  for (int i = 0; i < 5; ++i) x[i] = live ? x5[(size_t)row * 5 + i] : 0.f;
  for (int i = tid; i < 320; i += 256) sw0[i] = w0[i];
  for (int i = tid; i < 2048; i += 256) sw3[(i >> 6) * 65 + (i & 63)] = w3[i];  // padded rows: no bank conflicts
  if (tid < 64) { sb0[tid] = b0[tid]; sw5[tid] = w5[tid]; }
  if (tid < 32) sb3[tid] = b3[tid];
  if (tid < 2) sb5[tid] = b5[tid];
  __syncthreads();
  {
    float a = sb0[lane];
#pragma unroll
    for (int i = 0; i < 5; ++i) a = fmaf(sw0[lane * 5 + i], x[i], a);
    hs[wave][lane] = fmaxf(a, 0.f);
  }
  __syncthreads();
  if (lane < 32) {
    float a = sb3[lane];
#pragma unroll 16
    for (int i = 0; i < 64; ++i) a = fmaf(sw3[lane * 65 + i], hs[wave][i], a);
    h2[wave][lane] = fmaxf(a, 0.f);
  }
  __syncthreads();
  if (!live || lane != 0) return;
  float l0 = sb5[0], l1 = sb5[1];
  for (int o = 0; o < 32; ++o) {
    l0 = fmaf(sw5[o], h2[wave][o], l0);
    l1 = fmaf(sw5[32 + o], h2[wave][o], l1);
  }
  const float m = fmaxf(l0, l1);
  const float e0 = expf(l0 - m), e1 = expf(l1 - m);
  const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
  probs[(size_t)row * 2] = p0;
  probs[(size_t)row * 2 + 1] = p1;
  const int v = p1 > 0.5f ? 1 : 0;
  if (verdict) verdict[row] = v;
  if (conf) conf[row] = v ? p1 : p0;
  if (rule) {
    int rr = 5;
    if (x[4] > 0.7f) rr = 0;
    else if (x[2] > 0.7f) rr = 1;
    else if (x[0] > 0.7f) rr = 2;
    else if (x[1] > 0.7f) rr = 3;
    else if (x[3] < 0.3f) rr = 4;
    rule[row] = rr;
  }
}

__global__ __launch_bounds__(256) void rowdot_kernel(const float* a, const float* c, float* out, int ostride, int B,
                                                     int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  float s = 0.f;
  for (int i0 = lane; i0 < C; i0 += 512) {  // 8 columns per lane in flight, then the ascending-i chain
    float ta[8], tc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 64 * u;
      ta[u] = i < C ? a[(size_t)row * C + i] : 0.f;
      tc[u] = i < C ? c[(size_t)row * C + i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + 64 * u < C) s = fmaf(ta[u], tc[u], s);
  }
  s = wave_sum(s);
  if (lane == 0) out[(size_t)row * ostride] = s;
}

// S[B][N] = Q[B][D] . V[N][D]^T, fp32 (misinfo_forensics.py:446).  Tile 16 queries x 64 rows,
// 64-deep K chunks staged through LDS with 16-B loads; the next chunk's loads (clamped rows,
// no divergent region) are in flight while the current one is consumed.  Every output is one
// fp32 FMA chain over k = 0 .. D-1 in order.  D % 64 == 0 (host-checked).
__global__ __launch_bounds__(256) void vault_sims_kernel(const float* q, const float* v, float* S, int B, int N,
                                                         int D) {
  constexpr int KC = 64, LD = KC + 4;  // row stride 68 floats: 16-B aligned, rows 4 banks apart
  __shared__ __attribute__((aligned(16))) float qs[16 * LD];
  __shared__ __attribute__((aligned(16))) float vs[64 * LD];
  const int tid = threadIdx.x, tq = tid >> 4, tv = tid & 15;
  const int q0 = blockIdx.y * 16, v0 = blockIdx.x * 64;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // this thread's chunk pieces: one float4 of Q (row tid / 16, col 4 (tid % 16)), four of V
  const int qr = tid >> 4, qc = (tid & 15) * 4;
  const float* qp = q + (size_t)min(q0 + qr, B - 1) * D + qc;
  const float* vp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) vp[i] = v + (size_t)min(v0 + qr + 16 * i, N - 1) * D + qc;
  float4 rq, rv[4];
  auto load = [&](int k0) {
    rq = *reinterpret_cast<const float4*>(qp + k0);
#pragma unroll
    for (int i = 0; i < 4; ++i) rv[i] = *reinterpret_cast<const float4*>(vp[i] + k0);
  };
  load(0);
  for (int k0 = 0; k0 < D; k0 += KC) {
    *reinterpret_cast<float4*>(qs + qr * LD + qc) = rq;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(vs + (qr + 16 * i) * LD + qc) = rv[i];
    __syncthreads();
    if (k0 + KC < D) load(k0 + KC);
#pragma unroll 16
    for (int k = 0; k < KC; ++k) {
      const float a = qs[tq * LD + k];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(a, vs[(tv + 16 * j) * LD + k], acc[j]);
    }
    __syncthreads();
  }
  if (q0 + tq < B) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (v0 + tv + 16 * j < N) S[(size_t)(q0 + tq) * N + v0 + tv + 16 * j] = acc[j];
  }
}

// The same similarities on the fp32-input MFMA (v_mfma_f32_16x16x4_f32: bit-for-bit a k-ordered fmaf
// chain, as effnet_f32.hip's pw32m): BIT-IDENTICAL to vault_sims_kernel (every output the chain over
// k = 0 .. D-1 in order from 0) at the MFMA rate -- the launch sits on the step's serial tail.  Block
// = 64 vault rows x 16 queries, wave w = vault rows 16 w .. 16 w + 15; K in 16-deep chunks staged
// through LDS k-transposed ([row][g][s] = X[row][4 s + g]: a lane of group g reads its four steps'
// operands k = g, 4 + g, 8 + g, 12 + g with one ds_read_b128; step s covers k = 4 s .. 4 s + 3 in
// lane-group order), the next chunk's loads in flight under the current one's MFMAs.  Vault rows are
// the MFMA's A operand, so each lane ends with 4 consecutive vault rows of one query: 16-B stores.
__device__ __forceinline__ int vq_off(int row, int g) { return row * 16 + ((g ^ (((row >> 3) & 1) << 1)) << 2); }

// CH 16-deep chunks per LDS stage (one barrier per 16 CH of K; D % (16 CH) == 0, host-checked): the
// same chunk images and MFMA order as CH = 1, so the same ascending-k chains
template <int CH>
__global__ __launch_bounds__(256) void vault_sims_mfma_kernel(const float* __restrict__ q, const float* __restrict__ v,
                                                              float* __restrict__ S, int B, int N, int D) {
  __shared__ __attribute__((aligned(16))) float qs[2][CH][16 * 16];
  __shared__ __attribute__((aligned(16))) float vs[2][CH][64 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 16;
  // loaders: V chunk 64 x 16 = one float4 per thread (row lr, k quad lc); Q chunk 16 x 16 = threads 0-63
  const int lr = tid >> 2, lc = tid & 3;
  const float* vp = v + (size_t)min(n0 + lr, N - 1) * D + lc * 4;  // clamped rows: loaded, never stored
  const float* qp = q + (size_t)min(b0 + (lr & 15), B - 1) * D + lc * 4;
  float4 rv[CH], rq[CH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      rv[h] = *reinterpret_cast<const float4*>(vp + k0 + 16 * h);
      rq[h] = *reinterpret_cast<const float4*>(qp + k0 + 16 * h);
    }
  };
  auto lstore = [&](int buf) {  // k = 4 lc + e -> [row][g = e][s = lc]
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      const float av[4] = {rv[h].x, rv[h].y, rv[h].z, rv[h].w}, bv[4] = {rq[h].x, rq[h].y, rq[h].z, rq[h].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) vs[buf][h][vq_off(lr, e) + lc] = av[e];
      if (tid < 64) {
#pragma unroll
        for (int e = 0; e < 4; ++e) qs[buf][h][vq_off(lr, e) + lc] = bv[e];
      }
    }
  };
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = D / (16 * CH);
  gload(0);
  lstore(0);
  __syncthreads();
  for (int c = 0; c < nst; ++c) {
    const int buf = c & 1;
    if (c + 1 < nst) gload((c + 1) * 16 * CH);
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      const float4 wf = *reinterpret_cast<const float4*>(&vs[buf][h][vq_off(wave * 16 + fr, fg)]);
      const float4 xf = *reinterpret_cast<const float4*>(&qs[buf][h][vq_off(fr, fg)]);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.x, xf.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.y, xf.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.z, xf.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.w, xf.w, acc, 0, 0, 0);
    }
    if (c + 1 < nst) lstore(buf ^ 1);
    __syncthreads();
  }
  // lane: S[query b0 + fr][vault rows n .. n + 3], n = n0 + 16 wave + 4 fg
  const int b = b0 + fr, n = n0 + wave * 16 + fg * 4;
  if (b < B) {
    float* dst = S + (size_t)b * N + n;
    if (n + 3 < N && ((N & 3) == 0)) {
      *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < N) dst[r] = acc[r];
    }
  }
}

// Ranking of the reference's np.argsort(sims)[-k:][::-1] (misinfo_forensics.py:449): value
// descending; numpy sorts NaN (a zero-norm vault row: 0/0 in the renormalisation, :443-445) after
// every number, so the reversed tail puts NaN rows FIRST.  The scans rank by a key: the similarity,
// with NaN mapped to +inf (a cosine of unit rows is never +inf) and mapped back on output; empty
// slots hold -inf with index -1.  Exact ties: numpy's default sort is not stable (its tie order is
// data- and platform-dependent); ties are ordered here by descending index = what a
// stable argsort would give.
MMF_DEV float rank_key(float v) { return v != v ? INFINITY : v; }
MMF_DEV float unkey(float k) { return k == INFINITY ? NAN : k; }
MMF_DEV bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia > ib); }

// One 256-thread block per query row: each wave keeps per-lane top-K lists over its share of the
// columns (columns w * 64 + lane + 256 i, 8 loads in flight per lane), reduces them to the wave's
// top-K, and wave 0 merges the four waves' 4K candidates.  `better` is a strict total order (value,
// then index), so the K selected (value, index) pairs do not depend on how the columns were split.
template <int K>
__global__ __launch_bounds__(256) void vault_topk_kernel(const float* S, int B, int N, float thresh, float* sims,
                                                         int32_t* idx, float* disc, int disc_stride,
                                                         const float* temb, const float* title, int D,
                                                         float* tsim) {
  static_assert(4 * K <= 64, "wave 0 holds the 4K candidates one per lane");
  __shared__ float cv[4 * K];
  __shared__ int ci[4 * K];
  const int row = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (row >= B) return;  // (uniform per block)
  float tv[K];
  int ti[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { tv[i] = -INFINITY; ti[i] = -1; }
  const float* s = S + (size_t)row * N;
  for (int j0 = wave * 64 + lane; j0 < N; j0 += 256 * 8) {
    float vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) vv[u] = (j0 + 256 * u < N) ? rank_key(s[j0 + 256 * u]) : -INFINITY;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float v = vv[u];
      const int vi = j0 + 256 * u;
      if (vi < N && better(v, vi, tv[K - 1], ti[K - 1])) {
        tv[K - 1] = v; ti[K - 1] = vi;
#pragma unroll
        for (int i = K - 1; i > 0; --i) {
          if (better(tv[i], ti[i], tv[i - 1], ti[i - 1])) {
            const float a = tv[i]; tv[i] = tv[i - 1]; tv[i - 1] = a;
            const int b = ti[i]; ti[i] = ti[i - 1]; ti[i - 1] = b;
          }
        }
      }
    }
  }
  // the wave's top K: K rounds of a wave arg-max over the lists' heads, the winning lane pops
#pragma unroll
  for (int t = 0; t < K; ++t) {
    float bv = tv[0];
    int bi = ti[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { cv[wave * K + t] = bv; ci[wave * K + t] = bi; }
    if (ti[0] == bi) {
#pragma unroll
      for (int i = 0; i < K - 1; ++i) { tv[i] = tv[i + 1]; ti[i] = ti[i + 1]; }
      tv[K - 1] = -INFINITY; ti[K - 1] = -1;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  // merge: lane l < 4K holds candidate l
  float mv = lane < 4 * K ? cv[lane] : -INFINITY;
  int mi = lane < 4 * K ? ci[lane] : -1;
  float outv[K];
  int outi[K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    float bv = mv;
    int bi = mi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    outv[t] = bv; outi[t] = bi;
    if (mi == bi) { mv = -INFINITY; mi = -1; }
  }
  const bool hit = outv[0] > thresh && outv[0] != INFINITY;  // NaN > thresh is false
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < K; ++t) {
      if (sims) sims[(size_t)row * K + t] = unkey(outv[t]);
      if (idx) idx[(size_t)row * K + t] = outi[t];
    }
    if (disc) disc[(size_t)row * disc_stride] = hit ? outv[0] : 0.f;
  }
  if (tsim) {
    float d = 0.f;
    if (hit && temb && title) {
      // 8 columns per lane in flight at once (D <= 512), then the same ascending-c fmaf chain
      for (int c0 = lane; c0 < D; c0 += 512) {
        float ta[8], tb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + 64 * u;
          ta[u] = c < D ? temb[(size_t)row * D + c] : 0.f;
          tb[u] = c < D ? title[(size_t)outi[0] * D + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (c0 + 64 * u < D) d = fmaf(ta[u], tb[u], d);
      }
      d = wave_sum(d);
    }
    if (lane == 0) tsim[row] = d;
  }
}

// top-k for k > 8 (search_vault's top_k is a free parameter): one 1024-thread block per query
// row sorts all N similarities (padded to P, a power of two) in LDS with a bitonic network under
// the same `better` order, then writes the first k.  N <= P <= 16384 (128 KB of LDS).
template <int P>
__global__ __launch_bounds__(1024) void vault_sort_topk_kernel(const float* S, int B, int N, int k, float thresh,
                                                               float* sims, int32_t* idx, float* disc,
                                                               int disc_stride, const float* temb,
                                                               const float* title, int D, float* tsim) {
  __shared__ float key[P];
  __shared__ int id[P];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* s = S + (size_t)row * N;
  for (int i = tid; i < P; i += 1024) {
    key[i] = i < N ? rank_key(s[i]) : -INFINITY;
    id[i] = i < N ? i : -1;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P / 2; i += 1024) {
        const int lo = 2 * stride * (i / stride) + (i % stride), hi = lo + stride;
        const bool desc = (lo & size) == 0;  // descending segments; the final pass is all-descending
        const float a = key[lo], b = key[hi];
        const int ia = id[lo], ib = id[hi];
        if (desc ? better(b, ib, a, ia) : better(a, ia, b, ib)) {
          key[lo] = b; key[hi] = a;
          id[lo] = ib; id[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  const bool hit = key[0] > thresh && key[0] != INFINITY;
  for (int t = tid; t < k; t += 1024) {
    if (sims) sims[(size_t)row * k + t] = unkey(key[t]);
    if (idx) idx[(size_t)row * k + t] = id[t];
  }
  if (tid == 0 && disc) disc[(size_t)row * disc_stride] = hit ? key[0] : 0.f;  // (a hit is finite)
  if (tsim && tid < 64) {
    float d = 0.f;
    if (hit && temb && title) {
      for (int c = tid; c < D; c += 64) d = fmaf(temb[(size_t)row * D + c], title[(size_t)id[0] * D + c], d);
      d = wave_sum(d);
    }
    if (tid == 0) tsim[row] = d;
  }
}

}  // namespace

hipError_t launch_text_heads(const float* x, int row_stride, const float* w1a, const float* b1a, const float* w2a,
                             const float* b2a, const float* w1m, const float* b1m, const float* w2m,
                             const float* b2m, float* ai_logits, float* mi_logits, float* scores, int score_stride,
                             int B, hipStream_t s, const int* ovf) {
  hipLaunchKernelGGL(text_heads_kernel, dim3((B + 3) / 4, 2), dim3(1024), 0, s, x, row_stride, w1a, b1a, w2a, b2a, w1m,
                     b1m, w2m, b2m, ai_logits, mi_logits, scores, score_stride, B, ovf);
  return hipGetLastError();
}

hipError_t launch_fusion(const float* x5, const float* w0, const float* b0, const float* w3, const float* b3,
                         const float* w5, const float* b5, float* probs, int32_t* verdict, float* conf,
                         int32_t* rule, int B, hipStream_t s) {
  hipLaunchKernelGGL(fusion_kernel, dim3((B + 3) / 4), dim3(256), 0, s, x5, w0, b0, w3, b3, w5, b5, probs,
                     verdict, conf, rule, B);
  return hipGetLastError();
}

hipError_t launch_rowdot(const float* a, const float* c, float* out, int ostride, int B, int C, hipStream_t s) {
  hipLaunchKernelGGL(rowdot_kernel, dim3((B + 3) / 4), dim3(256), 0, s, a, c, out, ostride, B, C);
  return hipGetLastError();
}

#ifndef MMF_VAULT_CH
#define MMF_VAULT_CH 4  // 16-deep K chunks per LDS stage / barrier
#endif
hipError_t launch_vault_sims(const float* q, const float* v, float* S, int B, int N, int D, hipStream_t s, int ref) {
  if (D & 63) return hipErrorInvalidValue;
  if (B <= 0 || N <= 0) return hipSuccess;
  // the fp32-MFMA kernel; ref (option vault_ref, diagnostic): the VALU kernel it is bit-identical to
  // (tests/test_gpu_vault_edge.py::test_vault_kernels_match_reference_kernels)
  if (ref)
    hipLaunchKernelGGL(vault_sims_kernel, dim3((N + 63) / 64, (B + 15) / 16), dim3(256), 0, s, q, v, S, B, N, D);
  else if ((D % (16 * MMF_VAULT_CH)) == 0)
    hipLaunchKernelGGL(vault_sims_mfma_kernel<MMF_VAULT_CH>, dim3((N + 63) / 64, (B + 15) / 16), dim3(256), 0, s, q, v, S, B, N, D);
  else
    hipLaunchKernelGGL(vault_sims_mfma_kernel<1>, dim3((N + 63) / 64, (B + 15) / 16), dim3(256), 0, s, q, v, S, B, N, D);
  return hipGetLastError();
}

hipError_t launch_vault_topk(const float* S, int B, int N, int k, float thresh, float* sims, int32_t* idx,
                             float* disc, int disc_stride, const float* text_emb, const float* title_emb, int D,
                             float* text_sim, hipStream_t s, int ref) {
  const dim3 grid(B), blk(256);  // one block (four waves) per query row
#define TOPK_CASE(KK)                                                                                          \
  case KK:                                                                                                     \
    hipLaunchKernelGGL(vault_topk_kernel<KK>, grid, blk, 0, s, S, B, N, thresh, sims, idx, disc, disc_stride, \
                       text_emb, title_emb, D, text_sim);                                                      \
    break;
  // k > N is the reference's argsort(...)[-k:] on a short vault: it keeps all N rows.  The
  // register kernels pad slots N..k-1 with (-inf, -1) (the host drops idx < 0), so a fixed k = 5
  // (mmf_analyze_batch) serves a vault of any size; the sort kernel pads the same way up to P.
  if (k < 1 || N < 1) return hipErrorInvalidValue;
  // ref (option vault_ref, diagnostic): every k through the full-sort kernel -- an independent
  // selection algorithm the register kernels must agree with bit for bit
  switch (ref && N <= 16384 ? 0 : k) {
    TOPK_CASE(1) TOPK_CASE(2) TOPK_CASE(3) TOPK_CASE(4) TOPK_CASE(5) TOPK_CASE(6) TOPK_CASE(7) TOPK_CASE(8)
    default: {
#define SORT_CASE(PP)                                                                                            \
  if (N <= PP && k <= PP) {                                                                                      \
    hipLaunchKernelGGL(vault_sort_topk_kernel<PP>, dim3(B), dim3(1024), 0, s, S, B, N, k, thresh, sims, idx, disc, \
                       disc_stride, text_emb, title_emb, D, text_sim);                                          \
    return hipGetLastError();                                                                                    \
  }
      SORT_CASE(2048) SORT_CASE(4096) SORT_CASE(8192) SORT_CASE(16384)
#undef SORT_CASE
      return hipErrorInvalidValue;
    }
  }
#undef TOPK_CASE
  return hipGetLastError();
}

namespace {
__global__ void fill_strided_kernel(float* p, int stride, int B, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) p[(size_t)i * stride] = v;
}
}  // namespace

hipError_t launch_fill_strided(float* p, int stride, int B, float v, hipStream_t s) {
  hipLaunchKernelGGL(fill_strided_kernel, dim3((B + 255) / 256), dim3(256), 0, s, p, stride, B, v);
  return hipGetLastError();
}
