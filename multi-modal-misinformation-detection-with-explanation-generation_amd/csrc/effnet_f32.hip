// EfficientNet-B0 tower in fp32 end to end (process/handle option "effnet_fp32"): activations NHWC
// fp32, 1x1 convolutions as fp32-FMA GEMMs, depthwise convs and pooling in fp32.  The default
// tower (effnet.hip + the fp16 MFMA GEMM) stores activations in fp16; that is within the north-star
// 1e-3 for a trained / BN-conditioned network, but a tower whose logits reach O(100) (random He
// fan_in convolutions with unit running statistics) amplifies fp16 storage rounding
// past it.  This path trades ~3x the tower time for fp32 rounding throughout (the torch fp32 eval
// forward of torchvision's EfficientNet-B0 that misinfo_forensics.py:95-104 runs).
//   pw32     C = act((A * scale[image]) W^T + bias) (+ residual): the expand / project / head convs
//   dw32     depthwise kxk + BN + SiLU, one thread per (output pixel, 4 channels); weights
//            tap-major [k*k][C] so a thread's 4 channels are one float4
//   sum32    per-(image, pixel chunk, channel) sums in a fixed order -> the SE pool partials (one wave per
//            block: 4-channel lanes x 4 pixel lanes x chunks, four float4 loads in flight per lane)
//   gap32    global average pool + Linear(1280, 2) + softmax[:, 1]
// The stem is effnet.hip's stem kernel with fp32 output; the SE is effnet.hip's se kernel.  Every
// SiLU / sigmoid here is the IEEE-division, full-precision-exp form torch's CPU kernels use
// (silu_precise): the towers this mode exists for amplify ~1e-7 relative perturbations to ~1e-4.
#include "common.h"
#include "kernels.h"

namespace {

// 64 x 64 output tile, K in steps of 16 staged through LDS ([k][m] / [k][n], so each thread's 4
// rows and 4 columns are one float4 read each); thread (ty, tx) owns rows ty*4.. and cols tx*4..
constexpr int PB = 64, PK = 16;

__global__ __launch_bounds__(256) void pw32_kernel(const float* __restrict__ A, const float* __restrict__ Wt,
                                                   const float* __restrict__ bias, const float* __restrict__ ascale,
                                                   int rows_per_image, const float* __restrict__ res,
                                                   float* __restrict__ C, int M, int N, int K, int act) {
  __shared__ __attribute__((aligned(16))) float As[PK][PB + 4];
  __shared__ __attribute__((aligned(16))) float Ws[PK][PB + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.x * PB, n0 = blockIdx.y * PB;
  // loader: thread -> (row lr, k quad lq) of the 64 x 16 slab
  const int lr = tid >> 2, lq = (tid & 3) * 4;
  const int am = m0 + lr, wn = n0 + lr;
  const float* sc = (ascale && am < M) ? ascale + (size_t)(am / rows_per_image) * K : nullptr;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += PK) {
    const int k = k0 + lq;  // K % 4 == 0 (checked by the launcher): a quad is in or out whole
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), w = a;
    if (am < M && k < K) {
      a = *reinterpret_cast<const float4*>(A + (size_t)am * K + k);
      if (sc) {
        const float4 s = *reinterpret_cast<const float4*>(sc + k);
        a.x *= s.x; a.y *= s.y; a.z *= s.z; a.w *= s.w;
      }
    }
    if (wn < N && k < K) w = *reinterpret_cast<const float4*>(Wt + (size_t)wn * K + k);
    __syncthreads();
    As[lq][lr] = a.x; As[lq + 1][lr] = a.y; As[lq + 2][lr] = a.z; As[lq + 3][lr] = a.w;
    Ws[lq][lr] = w.x; Ws[lq + 1][lr] = w.y; Ws[lq + 2][lr] = w.z; Ws[lq + 3][lr] = w.w;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < PK; ++kk) {
      const float4 av = *reinterpret_cast<const float4*>(&As[kk][ty * 4]);
      const float4 wv = *reinterpret_cast<const float4*>(&Ws[kk][tx * 4]);
      const float ar[4] = {av.x, av.y, av.z, av.w}, wr[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ar[i], wr[j], acc[i][j]);
    }
  }
  const int n = n0 + tx * 4;
  if (n >= N) return;  // N % 4 == 0
  const float4 bv = *reinterpret_cast<const float4*>(bias + n);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) break;
    float o[4] = {acc[i][0] + bv.x, acc[i][1] + bv.y, acc[i][2] + bv.z, acc[i][3] + bv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = act_precise(o[j], act);
    if (res) {
      const float4 r = *reinterpret_cast<const float4*>(res + (size_t)m * N + n);
      o[0] += r.x; o[1] += r.y; o[2] += r.z; o[3] += r.w;
    }
    *reinterpret_cast<float4*>(C + (size_t)m * N + n) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// The same contraction on the fp32-input MFMA (v_mfma_f32_16x16x4_f32: bit-for-bit a k-ordered fp32
// fmaf chain, cdna_hip_programming.md §3) -- BIT-IDENTICAL to pw32_kernel (products in ascending k
// from a zero accumulator, then bias / activation / residual in the same order) at the f32 MFMA rate
// instead of an LDS-read-bound VALU loop.  64 x 64 tile, 4 waves of 32 x 32 (2 x 2 MFMA blocks),
// K in chunks of 16 staged through LDS (double buffer, register-staged global loads).  The chunk is
// stored k-transposed ([row][g][s] = A[row][4 s + g]) so a lane of group g reads its four MFMA
// steps' operands (k = g, 4 + g, 8 + g, 12 + g) with ONE ds_read_b128, and step s covers
// k = 4 s .. 4 s + 3 in lane-group order: the chain runs in ascending k.  Operands are swapped
// (W rows are the MFMA's A operand) so each lane ends with 4 consecutive output columns.
constexpr int QB = 64, QK = 16;
// float offset of (row, lane group g) in a [QB][QK] chunk; chunk ^= 2 * bit3(row) makes the
// 16-lane ds_read_b128 groups conflict-free (the 64-B-row swizzle of gemm_ring.hip)
MMF_DEV int q_off(int row, int g) { return row * QK + ((g ^ (((row >> 3) & 1) << 1)) << 2); }

// D = global-load prefetch depth in K chunks: chunk c is requested D - 1 chunks before the one that
// stores it to LDS (D = 2: during the previous chunk's MFMAs only, the round-3 kernel).  The launches
// with few workgroups per CU (M = B * 7^2 or 14^2 rows, K = 480 ... 1152) cannot hide a global load
// behind one 16-deep chunk; D = 4 keeps three chunks of loads in flight (8 more VGPRs per chunk of
// depth).  The operation sequence, and so every result bit, is the same for every D.
template <int D>
__global__ __launch_bounds__(256) void pw32m_kernel(const float* __restrict__ A, const float* __restrict__ Wt,
                                                    const float* __restrict__ bias, const float* __restrict__ ascale,
                                                    int rows_per_image, const float* __restrict__ res,
                                                    float* __restrict__ C, int M, int N, int K, int act) {
  static_assert(D >= 2, "the stored chunk is at least one chunk ahead");
  __shared__ __attribute__((aligned(16))) float As[2][QB * QK];
  __shared__ __attribute__((aligned(16))) float Ws[2][QB * QK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fg = lane >> 4;
  const int m0 = blockIdx.x * QB, n0 = blockIdx.y * QB;
  // loader: thread -> (row lr, k quad lc) of the 64 x 16 chunk
  const int lr = tid >> 2, lc = tid & 3;
  const int am = m0 + lr, wr = n0 + lr;
  const float* sc = (ascale && am < M) ? ascale + (size_t)(am / rows_per_image) * K : nullptr;
  auto gload = [&](int k0, float4& a, float4& w) {
    const int k = k0 + lc * 4;  // K % 4 == 0: a quad is in or out whole
    a = make_float4(0.f, 0.f, 0.f, 0.f);
    w = a;
    if (am < M && k < K) {
      a = *reinterpret_cast<const float4*>(A + (size_t)am * K + k);
      if (sc) {
        const float4 s4 = *reinterpret_cast<const float4*>(sc + k);
        a.x *= s4.x; a.y *= s4.y; a.z *= s4.z; a.w *= s4.w;
      }
    }
    if (wr < N && k < K) w = *reinterpret_cast<const float4*>(Wt + (size_t)wr * K + k);
  };
  auto lstore = [&](int buf, const float4& a, const float4& w) {  // k = 4 lc + e -> [lr][g = e][s = lc]
    const float av[4] = {a.x, a.y, a.z, a.w}, wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      As[buf][q_off(lr, e) + lc] = av[e];
      Ws[buf][q_off(lr, e) + lc] = wv[e];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // register slots: chunk c lives in slot c % D from its request until it is stored to LDS
  float4 ra[D], rw[D];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) gload(d * QK, ra[d], rw[d]);
  lstore(0, ra[0], rw[0]);
  __syncthreads();
  const int nch = (K + QK - 1) / QK;
  // chunk c = c0 + d with d compile-time (slot indices static); c0 steps by D
  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      if (c >= nch) break;
      const int buf = c & 1;
      // request chunk c + D - 1 into the slot chunk c - 1 occupied (stored to LDS a chunk ago)
      if (c + D - 1 < nch) gload((c + D - 1) * QK, ra[(d + D - 1) % D], rw[(d + D - 1) % D]);
      float4 wf[2], xf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) wf[i] = *reinterpret_cast<const float4*>(&Ws[buf][q_off(wn * 32 + i * 16 + fr, fg)]);
#pragma unroll
      for (int j = 0; j < 2; ++j) xf[j] = *reinterpret_cast<const float4*>(&As[buf][q_off(wm * 32 + j * 16 + fr, fg)]);
      const float wfs[2][4] = {{wf[0].x, wf[0].y, wf[0].z, wf[0].w}, {wf[1].x, wf[1].y, wf[1].z, wf[1].w}};
      const float xfs[2][4] = {{xf[0].x, xf[0].y, xf[0].z, xf[0].w}, {xf[1].x, xf[1].y, xf[1].z, xf[1].w}};
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfs[i][st], xfs[j][st], acc[i][j], 0, 0, 0);
      if (c + 1 < nch) lstore(buf ^ 1, ra[(d + 1) % D], rw[(d + 1) % D]);
      __syncthreads();
    }
  }
  // lane: C[m][n .. n + 3] of each 16 x 16 block (operands swapped)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + wm * 32 + j * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = n0 + wn * 32 + i * 16 + fg * 4;
      if (n >= N) continue;  // N % 4 == 0
      const float4 bv = *reinterpret_cast<const float4*>(bias + n);
      float o[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_precise(o[e], act);
      if (res) {
        const float4 r = *reinterpret_cast<const float4*>(res + (size_t)m * N + n);
        o[0] += r.x; o[1] += r.y; o[2] += r.z; o[3] += r.w;
      }
      *reinterpret_cast<float4*>(C + (size_t)m * N + n) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// Small-K / narrow-N form of the same contraction (pw32_mfma = 3, K <= 64 and N <= 256: the expands of
// stages 2.1 - 4.1 and the stage-1 project, which write 6-10x the bytes they read): one block owns 64
// WHOLE output rows (every column), so its output is one contiguous run of 64 N floats.  Wave w computes
// rows 16 w .. 16 w + 15 over all NF = ceil(N / 16) column blocks on the fp32-input MFMA with the K
// chunks, LDS images and step order of pw32m_kernel -- every output element is the same ascending-k
// fmaf chain, then + bias, activation, + residual in the same order: BIT-IDENTICAL -- and the finished
// (bias + activation) tile goes to LDS in its global row-major layout, from where the block stores it
// (residual added on the way) as consecutive 16-B lanes: full-line writes instead of pw32m's 64-B row
// pieces per 16 rows (the write rate, not the arithmetic, bounds these launches).
template <int NF, int D>
__global__ __launch_bounds__(256) void pw32r_kernel(const float* __restrict__ A, const float* __restrict__ Wt,
                                                    const float* __restrict__ bias, const float* __restrict__ ascale,
                                                    int rows_per_image, const float* __restrict__ res,
                                                    float* __restrict__ C, int M, int N, int K, int act, int NC) {
  constexpr int NT = NF * 16, AS = QB * QK, WS = NT * QK;
  extern __shared__ __attribute__((aligned(16))) float r_smem[];
  // column tile: columns n0 .. n0 + nc of every row (NC = N, one tile, below 256 columns; wider
  // launches split N into equal multiples of 16)
  const int n0 = blockIdx.y * NC, nc = min(NC, N - n0);
  float* As = r_smem;           // [2][QB * QK]
  float* Ws = r_smem + 2 * AS;  // [2][NT * QK]
  float* Cs = r_smem;           // [QB][nc] (aliases As / Ws once the K loop is done)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int m0 = blockIdx.x * QB;
  // loaders: A chunk 64 x 16 = one float4 per thread (row lr, k quad lc); W chunk NT x 16 = NF / 4
  // float4 per thread (rows wr0 + 64 q)
  const int lr = tid >> 2, lc = tid & 3;
  const int am = m0 + lr;
  const float* sc = (ascale && am < M) ? ascale + (size_t)(am / rows_per_image) * K : nullptr;
  constexpr int WQ = (NT * 4 + 255) / 256;  // float4 of the W chunk per thread
  auto gload = [&](int k0, float4& a, float4 (&w)[WQ]) {
    const int k = k0 + lc * 4;  // K % 4 == 0: a quad is in or out whole
    a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (am < M && k < K) {
      a = *reinterpret_cast<const float4*>(A + (size_t)am * K + k);
      if (sc) {
        const float4 s4 = *reinterpret_cast<const float4*>(sc + k);
        a.x *= s4.x; a.y *= s4.y; a.z *= s4.z; a.w *= s4.w;
      }
    }
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int wr = lr + 64 * q;
      w[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (wr < nc && k < K) w[q] = *reinterpret_cast<const float4*>(Wt + (size_t)(n0 + wr) * K + k);
    }
  };
  auto lstore = [&](int buf, const float4& a, const float4 (&w)[WQ]) {  // k = 4 lc + e -> [row][g = e][s = lc]
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) As[buf * AS + q_off(lr, e) + lc] = av[e];
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int wr = lr + 64 * q;
      if (wr < NT) {
        const float wv[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) Ws[buf * WS + q_off(wr, e) + lc] = wv[e];
      }
    }
  };
  f32x4 acc[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = (K + QK - 1) / QK;
  // register slots: chunk c is requested D - 1 chunks before the one that stores it to LDS (pw32m's
  // scheme; D = 2 for the K <= 64 launches, deeper for the long-K projects)
  float4 ra[D], rw[D][WQ];
#pragma unroll
  for (int d = 0; d < D - 1; ++d)
    if (d < nch) gload(d * QK, ra[d], rw[d]);
  lstore(0, ra[0], rw[0]);
  __syncthreads();
  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      if (c >= nch) break;
      const int buf = c & 1;
      if (c + D - 1 < nch) gload((c + D - 1) * QK, ra[(d + D - 1) % D], rw[(d + D - 1) % D]);
      const float4 xf = *reinterpret_cast<const float4*>(&As[buf * AS + q_off(wave * 16 + fr, fg)]);
      const float xfs[4] = {xf.x, xf.y, xf.z, xf.w};
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const float4 wf = *reinterpret_cast<const float4*>(&Ws[buf * WS + q_off(i * 16 + fr, fg)]);
        const float wfs[4] = {wf.x, wf.y, wf.z, wf.w};
#pragma unroll
        for (int st = 0; st < 4; ++st) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfs[st], xfs[st], acc[i], 0, 0, 0);
      }
      if (c + 1 < nch) lstore(buf ^ 1, ra[(d + 1) % D], rw[(d + 1) % D]);
      __syncthreads();
    }
  }
  // lane: C[m][n .. n + 3] of each 16 x 16 block (operands swapped) -> + bias, activation -> LDS tile
  const int ml = wave * 16 + fr;
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int n = i * 16 + fg * 4;
    if (n < nc) {  // N % 4 == 0, NC % 16 == 0
      const float4 bv = *reinterpret_cast<const float4*>(bias + n0 + n);
      float o[4] = {acc[i][0] + bv.x, acc[i][1] + bv.y, acc[i][2] + bv.z, acc[i][3] + bv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_precise(o[e], act);
      *reinterpret_cast<float4*>(&Cs[ml * nc + n]) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  __syncthreads();
  // the block's rows: nc contiguous floats each (one contiguous run of C when nc = N), stored (and the
  // residual read) as consecutive 16-B lanes
  const int rows = min(QB, M - m0), q4 = nc / 4;
  const float4* cs4 = reinterpret_cast<const float4*>(Cs);
  for (int idx = tid; idx < rows * q4; idx += 256) {
    const int r = idx / q4, cq = idx - r * q4;
    const size_t g = (size_t)(m0 + r) * N + n0 + 4 * cq;
    float4 v = cs4[idx];
    if (res) {
      const float4 rv = *reinterpret_cast<const float4*>(res + g);
      v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
    }
    *reinterpret_cast<float4*>(C + g) = v;
  }
}

#ifndef MMF_DW32_R
#define MMF_DW32_R 7  // outputs per thread along x (every EfficientNet-B0 width is a multiple of 7)
#endif

// torchvision pads (k - 1) / 2 on every side; output edge (H - 1) / S + 1.  A thread computes R
// horizontally adjacent outputs of one 4-channel group: per kernel row it loads the (R - 1) S + K
// input columns and the K weights once and reuses them across the R outputs (R K loads -> R S + K).
// Each output's fmaf chain is bias, then (ky, kx) ascending with out-of-image taps skipped -- the
// same chain at every R (R = 1 is the one-output-per-thread kernel), so the bits do not depend on R.
template <int K, int S, int R>
__global__ __launch_bounds__(256) void dw32_kernel(const float* __restrict__ in, const float* __restrict__ w,
                                                   const float* __restrict__ bias, float* __restrict__ out, int H,
                                                   int W, int C, int Ho, int Wo, int Wg, size_t total4) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C / 4, c4 = (int)(i % C4);
  const size_t g = i / C4;
  const int ox0 = (int)(g % Wg) * R, oy = (int)((g / Wg) % Ho), bi = (int)(g / ((size_t)Wg * Ho));
  const int c = c4 * 4;
  constexpr int P = (K - 1) / 2, NC = (R - 1) * S + K;
  const float4 b4 = make_float4(bias[c], bias[c + 1], bias[c + 2], bias[c + 3]);
  float4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = b4;
  const int ix0 = ox0 * S - P;
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int iy = oy * S - P + ky;
    if (iy < 0 || iy >= H) continue;
    const float* row = in + ((size_t)bi * H + iy) * W * C + c;
    float4 v[NC], wt[K];
#pragma unroll
    for (int kx = 0; kx < K; ++kx) wt[kx] = *reinterpret_cast<const float4*>(w + (size_t)(ky * K + kx) * C + c);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int ix = ix0 + j;
      v[j] = (ix >= 0 && ix < W) ? *reinterpret_cast<const float4*>(row + (size_t)ix * C) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int j = r * S + kx, ix = ix0 + j;
        if (ix < 0 || ix >= W) continue;
        acc[r].x = fmaf(v[j].x, wt[kx].x, acc[r].x);
        acc[r].y = fmaf(v[j].y, wt[kx].y, acc[r].y);
        acc[r].z = fmaf(v[j].z, wt[kx].z, acc[r].z);
        acc[r].w = fmaf(v[j].w, wt[kx].w, acc[r].w);
      }
  }
  float* o = out + (((size_t)bi * Ho + oy) * Wo + ox0) * C + c;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (ox0 + r < Wo)
      *reinterpret_cast<float4*>(o + (size_t)r * C) = make_float4(silu_precise(acc[r].x), silu_precise(acc[r].y),
                                                                  silu_precise(acc[r].z), silu_precise(acc[r].w));
}

// Chunk j of image b covers pixels [j HW / nchunks, (j + 1) HW / nchunks).  Per channel, 4 pixel
// lanes each sum their pixels in order (lane r: p0 + r, p0 + r + 4, ...), then the 4 lane sums are
// added in a fixed order ((r0 + r1) + (r2 + r3)) -> part[b][j][c].  One wave: L lanes of 4 channels
// (float4 loads) x 4 pixel lanes x 16 / L chunks; grid (C / 4 / L, ceil(nchunks L / 16), B).
template <int L>
__global__ __launch_bounds__(64) void sum32_kernel(const float* __restrict__ x, int HW, int C, int nch,
                                                   float* __restrict__ part) {
  __shared__ float4 red[64];
  constexpr int G = 16 / L;
  const int lane = threadIdx.x, bi = blockIdx.z;
  const int c = (blockIdx.x * L + lane % L) * 4, r = (lane / L) & 3, j = blockIdx.y * G + lane / (4 * L);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < nch) {
    const int p0 = (int)((long)j * HW / nch), p1 = (int)((long)(j + 1) * HW / nch);
    const float* xp = x + (size_t)bi * HW * C + c;
    int p = p0 + r;
    for (; p + 12 < p1; p += 16) {  // four loads in flight, added in pixel order
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(xp + (size_t)(p + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u) { a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w; }
    }
    for (; p < p1; p += 4) {
      const float4 v = *reinterpret_cast<const float4*>(xp + (size_t)p * C);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[lane] = a;
  __syncthreads();
  if (r == 0 && j < nch) {
    const float4 s0 = red[lane], s1 = red[lane + L], s2 = red[lane + 2 * L], s3 = red[lane + 3 * L];
    *reinterpret_cast<float4*>(part + ((size_t)bi * nch + j) * C + c) =
        make_float4((s0.x + s1.x) + (s2.x + s3.x), (s0.y + s1.y) + (s2.y + s3.y), (s0.z + s1.z) + (s2.z + s3.z),
                    (s0.w + s1.w) + (s2.w + s3.w));
  }
}

__global__ __launch_bounds__(256) void gap32_kernel(const float* __restrict__ x, int HW, int C,
                                                    const float* __restrict__ w, const float* __restrict__ b,
                                                    float* logits, float* score, int score_stride) {
  __shared__ float red[2][4];
  const int bi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float inv = 1.0f / (float)HW;
  float l0 = 0.f, l1 = 0.f;
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += x[((size_t)bi * HW + p) * C + c];
    l0 = fmaf(w[c], s * inv, l0);
    l1 = fmaf(w[C + c], s * inv, l1);
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

hipError_t launch_pw32(const float* A, const float* W, const float* bias, const float* ascale, int rows_per_image,
                       const float* res, float* C, int M, int N, int K, int act, hipStream_t s, int mfma) {
  if (M <= 0 || N <= 0 || K <= 0 || (N % 4) || (K % 4) || (ascale && rows_per_image <= 0) ||
      (act != ACT_NONE && act != ACT_SILU))
    return hipErrorInvalidValue;
  // mode 5: mode 4 only where the whole-row grid has the parallelism for its long K (>= 1024 blocks,
  // or >= 512 at NF <= 5): the 14^2 / 7^2 projects with 112 / 192 columns keep pw32m's 64-column tiles
  const long rblocks = (M + QB - 1) / QB;
  const bool rows_ok = mfma != 5 || rblocks >= 1024 || (N <= 80 && rblocks >= 512);
  if (mfma >= 3 && N <= 256 && (K <= 64 || (mfma >= 4 && rows_ok))) {
    // mfma = 3: the whole-row tile kernel for the small-K, write-bound launches; 4 (default): also
    // for every long-K launch of N <= 256 (the projects: A read once instead of once per 64-column
    // tile).  The wider launches (N 320 ... 1280) stay on pw32m: split into <= 256-column tiles of
    // this kernel they measured slower (B = 512 tower 11.39 -> 11.86 ms)
    const int ntl = (N + 255) / 256;
    const int NC = ((N + ntl - 1) / ntl + 15) / 16 * 16;
    const int NF = NC / 16;
    const size_t lds = std::max((size_t)(2 * QB * QK + 2 * NF * 16 * QK), (size_t)QB * NC) * 4;
    const dim3 grid((M + QB - 1) / QB, (N + NC - 1) / NC);
    const bool deep = K >= 4 * QK;
    switch (NF) {
#define MMF_PW32R(F)                                                                                              \
  case F:                                                                                                         \
    if (deep) hipLaunchKernelGGL((pw32r_kernel<F, 4>), grid, dim3(256), lds, s, A, W, bias, ascale, rows_per_image, res, C, M, N, K, act, NC); \
    else hipLaunchKernelGGL((pw32r_kernel<F, 2>), grid, dim3(256), lds, s, A, W, bias, ascale, rows_per_image, res, C, M, N, K, act, NC); \
    break;
      MMF_PW32R(1) MMF_PW32R(2) MMF_PW32R(3) MMF_PW32R(4) MMF_PW32R(5) MMF_PW32R(6) MMF_PW32R(7) MMF_PW32R(8)
      MMF_PW32R(9) MMF_PW32R(10) MMF_PW32R(11) MMF_PW32R(12) MMF_PW32R(13) MMF_PW32R(14) MMF_PW32R(15) MMF_PW32R(16)
#undef MMF_PW32R
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (mfma) {
    // mfma = 1: loads one chunk ahead (round 3); 2: three chunks ahead where K has >= 4 chunks and
    // the grid leaves < 4 workgroups per CU (the 7^2-stage projects, K = 672 / 1152: 134 -> 107 and
    // 199 -> 160 us per launch); launches with more workgroups hide the latency by occupancy and
    // measured 1.3-1.7x SLOWER with the deeper prefetch (its 16 more VGPRs)
    const dim3 grid((M + QB - 1) / QB, (N + QB - 1) / QB);
    if (mfma >= 2 && K >= 4 * QK && (long)grid.x * grid.y < 4 * 256)
      hipLaunchKernelGGL(pw32m_kernel<4>, grid, dim3(256), 0, s, A, W, bias, ascale, rows_per_image, res, C, M, N, K, act);
    else
      hipLaunchKernelGGL(pw32m_kernel<2>, grid, dim3(256), 0, s, A, W, bias, ascale, rows_per_image, res, C, M, N, K, act);
    return hipGetLastError();
  }
  const dim3 grid((M + PB - 1) / PB, (N + PB - 1) / PB);
  hipLaunchKernelGGL(pw32_kernel, grid, dim3(256), 0, s, A, W, bias, ascale, rows_per_image, res, C, M, N, K, act);
  return hipGetLastError();
}

hipError_t launch_dw32(const float* in, const float* w, const float* bias, float* out, int B, int H, int W, int C,
                       int k, int stride, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  constexpr int R = MMF_DW32_R;
  const int Wg = (Wo + R - 1) / R;
  const size_t total4 = (size_t)B * Ho * Wg * (C / 4);
  const dim3 grid((unsigned)((total4 + 255) / 256)), blk(256);
#define MMF_DW32(KK, SS)                                                                                       \
  if (k == KK && stride == SS) {                                                                               \
    hipLaunchKernelGGL((dw32_kernel<KK, SS, R>), grid, blk, 0, s, in, w, bias, out, H, W, C, Ho, Wo, Wg, total4); \
    return hipGetLastError();                                                                                  \
  }
  MMF_DW32(3, 1)
  MMF_DW32(3, 2)
  MMF_DW32(5, 1)
  MMF_DW32(5, 2)
#undef MMF_DW32
  return hipErrorInvalidValue;
}

hipError_t launch_sum32(const float* x, int B, int HW, int C, int nchunks, float* part, hipStream_t s) {
  if (nchunks < 1 || nchunks > HW || (C % 16)) return hipErrorInvalidValue;
  const int C4 = C / 4;
  const int L = C4 % 16 == 0 ? 16 : C4 % 8 == 0 ? 8 : 4;
  const dim3 grid(C4 / L, (nchunks * L + 15) / 16, B);
  if (L == 16) hipLaunchKernelGGL(sum32_kernel<16>, grid, dim3(64), 0, s, x, HW, C, nchunks, part);
  else if (L == 8) hipLaunchKernelGGL(sum32_kernel<8>, grid, dim3(64), 0, s, x, HW, C, nchunks, part);
  else hipLaunchKernelGGL(sum32_kernel<4>, grid, dim3(64), 0, s, x, HW, C, nchunks, part);
  return hipGetLastError();
}

hipError_t launch_gap32(const float* x, int HW, int C, const float* w, const float* b, float* logits, float* score,
                        int score_stride, int B, hipStream_t s) {
  hipLaunchKernelGGL(gap32_kernel, dim3(B), dim3(256), 0, s, x, HW, C, w, b, logits, score, score_stride);
  return hipGetLastError();
}

