// HBM-bound 1x1 convolutions of EfficientNet-B0 (expand: K = cin <= 192, project: N = cout <= 320
// with K = cexp <= 256) as a streaming MFMA kernel:
//     C[M][N] = act((A[M][K] * s[b][K]) . W[N][K]^T + bias) (+ res16), fp16 in / fp16 out.
// M = B*H*W pixels is huge and N, K are small, so these launches are bounded by streaming A in
// and C out: a GEMM tiling (K loop, double-buffered LDS tiles, 128x128 tiles
// padded to K = 64) spends most of its time in per-tile latency instead.  Here instead:
//  * a workgroup stages its W column block (<= 128 x KP fp16) and bias in LDS once, then walks
//    row blocks persistently;
//  * each wave loads its A fragments straight from HBM into registers (16 rows x 16 B per lane,
//    the MFMA B-operand layout), with the next row block's loads issued before the current
//    block's MFMAs and epilogue (software pipelining across the persistent loop);
//  * the epilogue (bias, SiLU, SE scale on A, residual) goes through a per-wave fp32 LDS stage so
//    that every output byte leaves in a 16-B-per-lane, row-contiguous store (coalesced), with a
//    single fp16 rounding, matching the tiled GEMM's numerics exactly.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int PW_THREADS = 256;  // 4 waves
#ifndef PW_SCALE_PRE
#define PW_SCALE_PRE 1
#endif

// LDS image of W: [BN][KP] fp16, 16-B chunks XOR-swizzled per row so the 16-lane groups of the
// fragment ds_read_b128 are conflict-free (brute-forced against the gfx950 lane groups).
template <int KS>
MMF_DEV int pw_swz(int r) {
  return (KS & 3) == 0 ? (r & 15) : ((KS & 1) == 0 ? (r & 7) : ((r & 8) >> 2));
}

template <int KS>
constexpr int pw_rpw() {  // 16-row fragments per wave per row block
  return KS <= 2 ? 4 : (KS <= 4 ? 2 : 1);
}

// CF = 16-column fragments per block (BN = 16 CF); columns past N are computed on zero weights
// and never stored -- MFMA work is free here, HBM bytes are not.
template <int KS, int CF, int ACT>
__global__ __launch_bounds__(PW_THREADS, 4) void pw_kernel(GemmArgs g, int nrb) {
  constexpr int KP = KS * 32, RPW = pw_rpw<KS>(), BN = CF * 16;
  constexpr int ROWS = 4 * RPW * 16;  // rows per row block (4 waves)
  constexpr int SLD = BN + 4;         // stage row stride (floats): conflict-free float4 writes
  constexpr int CPR = BN / 8;         // 16-B output chunks per stage row
  __shared__ __attribute__((aligned(16))) f16_t sW[BN * KP];
  __shared__ __attribute__((aligned(16))) float sBias[BN];
  __shared__ __attribute__((aligned(16))) float sStage[4][16 * SLD];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* stage = sStage[wave];
  const int fr = lane & 15, fg = lane >> 4;
  const int M = g.M, N = g.N, K = g.K;
  const int n0 = blockIdx.y * BN;

  // ---- W column block + bias -> LDS (zero outside N x K) ----
  for (int idx = tid; idx < BN * (KP / 8); idx += PW_THREADS) {
    const int r = idx / (KP / 8), c = idx - r * (KP / 8);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n0 + r < N && c * 8 < K) v = *reinterpret_cast<const uint4*>(g.W + (size_t)(n0 + r) * g.ldw + c * 8);
    *reinterpret_cast<uint4*>(sW + r * KP + ((c ^ pw_swz<KS>(r)) << 3)) = v;
  }
  for (int i = tid; i < BN; i += PW_THREADS) sBias[i] = (g.bias && n0 + i < N) ? g.bias[n0 + i] : 0.f;
  __syncthreads();

  const rsrc_t ra = make_rsrc(g.A, ((uint32_t)(M - 1) * g.lda + K) * 2u);
  const rsrc_t rs = make_rsrc(g.ascale, g.ascale ? (uint32_t)((M - 1) / g.rows_per_batch + 1) * K * 4u : 0u);
  const rsrc_t rr = make_rsrc(g.res16, g.res16 ? ((uint32_t)(M - 1) * g.ldr + N) * 2u : 0u);
  const rsrc_t rc = make_rsrc(g.c16, ((uint32_t)(M - 1) * g.ldc + N) * 2u);
  const bool has_scale = g.ascale != nullptr, has_res = g.res16 != nullptr;

  u32x4 acur[RPW * KS], anext[RPW * KS];
  int rb = blockIdx.x;
  if (rb >= nrb) return;
#define PW_LOAD_A(dst, rbx)                                                                   \
  _Pragma("unroll") for (int f = 0; f < RPW; ++f) {                                          \
    const uint32_t m = (uint32_t)(rbx) * ROWS + (wave * RPW + f) * 16 + fr;                  \
    _Pragma("unroll") for (int s = 0; s < KS; ++s) {                                         \
      const int k = s * 32 + fg * 8;                                                          \
      dst[f * KS + s] = __builtin_amdgcn_raw_buffer_load_b128(                               \
          ra, k < K ? (m * (uint32_t)g.lda + k) * 2u : kOOB, 0, 0);                          \
    }                                                                                         \
  }
  PW_LOAD_A(acur, rb)
  for (; rb < nrb; rb += gridDim.x) {
    // SE excitation factors of this row block, loaded BEFORE the next block's A prefetch: the
    // in-order vmcnt then lets them be consumed while the prefetch is still in flight (issued after
    // it, every wait for them also waited for the prefetch)
    // (only where the 8 RPW KS factor registers fit without spills or a lost wave: the narrow
    // projects; the expands -- ACT_SILU -- never carry a scale)
    constexpr bool PRE = PW_SCALE_PRE && ACT == ACT_NONE && CF <= 2 && RPW * KS <= 6;
    float4 sc[PRE ? RPW * KS : 1][2];
    if (PRE && has_scale) {
#pragma unroll
      for (int f = 0; f < RPW; ++f) {
        const uint32_t bimg = min((uint32_t)rb * ROWS + (wave * RPW + f) * 16 + fr, (uint32_t)(M - 1)) / (uint32_t)g.rows_per_batch;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int k = s * 32 + fg * 8;
          const uint32_t off = k < K ? (bimg * (uint32_t)K + k) * 4u : kOOB;
          sc[PRE ? f * KS + s : 0][0] = buf_load_f4(rs, off);
          sc[PRE ? f * KS + s : 0][1] = buf_load_f4(rs, off + 16u);
        }
      }
    }
    if (rb + (int)gridDim.x < nrb) { PW_LOAD_A(anext, rb + (int)gridDim.x) }
#pragma unroll
    for (int f = 0; f < RPW; ++f) {
      const uint32_t mrow0 = (uint32_t)rb * ROWS + (wave * RPW + f) * 16;
      if (has_scale) {  // SE excitation: A *= s[image][k] (rounded to fp16 like the tiled GEMM)
        const uint32_t bimg = min(mrow0 + fr, (uint32_t)(M - 1)) / (uint32_t)g.rows_per_batch;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int k = s * 32 + fg * 8;
          const uint32_t off = k < K ? (bimg * (uint32_t)K + k) * 4u : kOOB;
          const float4 s0 = PRE ? sc[PRE ? f * KS + s : 0][0] : buf_load_f4(rs, off);
          const float4 s1 = PRE ? sc[PRE ? f * KS + s : 0][1] : buf_load_f4(rs, off + 16u);
          u32x4& v = acur[f * KS + s];
          v.x = pack2h(lo_h(v.x) * s0.x, hi_h(v.x) * s0.y);
          v.y = pack2h(lo_h(v.y) * s0.z, hi_h(v.y) * s0.w);
          v.z = pack2h(lo_h(v.z) * s1.x, hi_h(v.z) * s1.y);
          v.w = pack2h(lo_h(v.w) * s1.z, hi_h(v.w) * s1.w);
        }
      }
      f32x4 acc[CF];
#pragma unroll
      for (int c = 0; c < CF; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f16x8 xb = __builtin_bit_cast(f16x8, acur[f * KS + s]);
#pragma unroll
        for (int c = 0; c < CF; ++c) {
          const int r = c * 16 + fr;
          const f16x8 wb =
              as_f16x8(*reinterpret_cast<const uint4*>(sW + r * KP + (((s * 4 + fg) ^ pw_swz<KS>(r)) << 3)));
          acc[c] = mfma16x16x32(wb, xb, acc[c]);
        }
      }
      // lane holds C[mrow0 + fr][n0 + 16c + 4fg .. +3]: bias + activation -> fp32 stage
#pragma unroll
      for (int c = 0; c < CF; ++c) {
        const int nl = c * 16 + fg * 4;
        const float4 b = *reinterpret_cast<const float4*>(sBias + nl);
        float v[4] = {acc[c][0] + b.x, acc[c][1] + b.y, acc[c][2] + b.z, acc[c][3] + b.w};
        if (ACT != ACT_NONE) {
          act4<ACT>(v);
        }
        *reinterpret_cast<float4*>(stage + fr * SLD + nl) = make_float4(v[0], v[1], v[2], v[3]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // row-contiguous 16-B stores: chunk q = (row, 8-column group)
#pragma unroll
      for (int q0 = 0; q0 < 16 * CPR; q0 += 64) {
        const int q = q0 + lane;
        if (16 * CPR % 64 == 0 || q < 16 * CPR) {
          const int row = q / CPR, c8 = q - row * CPR;
          const uint32_t m = mrow0 + row;
          const int n = n0 + c8 * 8;
          const float4 v0 = *reinterpret_cast<const float4*>(stage + row * SLD + c8 * 8);
          const float4 v1 = *reinterpret_cast<const float4*>(stage + row * SLD + c8 * 8 + 4);
          float o[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          if (has_res) {
            const u32x4 r4 =
                __builtin_amdgcn_raw_buffer_load_b128(rr, n < N ? (m * (uint32_t)g.ldr + n) * 2u : kOOB, 0, 0);
            o[0] += lo_h(r4.x); o[1] += hi_h(r4.x); o[2] += lo_h(r4.y); o[3] += hi_h(r4.y);
            o[4] += lo_h(r4.z); o[5] += hi_h(r4.z); o[6] += lo_h(r4.w); o[7] += hi_h(r4.w);
          }
          const uint4 pk =
              make_uint4(pack2h(o[0], o[1]), pack2h(o[2], o[3]), pack2h(o[4], o[5]), pack2h(o[6], o[7]));
          buf_store_u4(rc, n < N ? (m * (uint32_t)g.ldc + n) * 2u : kOOB, pk);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int i = 0; i < RPW * KS; ++i) acur[i] = anext[i];
  }
#undef PW_LOAD_A
}

template <int KS, int CF>
hipError_t run_pw(const GemmArgs& a, int nbn, hipStream_t s) {
  constexpr int ROWS = 4 * pw_rpw<KS>() * 16;
  const int nrb = (a.M + ROWS - 1) / ROWS;
  // persistent in x: about four workgroups per CU across the column blocks.  gx is a multiple of 8
  // so that the nbn workgroups (x, 0..nbn-1), which walk the same row blocks, share an XCD (linear
  // id x + y * gx lands on XCD (x + y * gx) % 8 = x % 8): each A row block is fetched from HBM into
  // that XCD's L2 once instead of once per column block (N = 672: nbn = 6, gx was 171)
  int gx = (1024 + nbn - 1) / nbn;
  if (nbn > 1) gx = gx / 8 * 8;
  if (gx > nrb) gx = nrb;
  const dim3 grid(gx, nbn);
  if (a.act == ACT_SILU)
    hipLaunchKernelGGL((pw_kernel<KS, CF, ACT_SILU>), grid, dim3(PW_THREADS), 0, s, a, nrb);
  else if (a.act == ACT_NONE)
    hipLaunchKernelGGL((pw_kernel<KS, CF, ACT_NONE>), grid, dim3(PW_THREADS), 0, s, a, nrb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int KS>
hipError_t run_pw_ks(const GemmArgs& a, hipStream_t s) {
  // column block: 32, 64 or 128 wide (padding beyond N costs MFMA time only)
  if (a.N <= 32) return run_pw<KS, 2>(a, 1, s);
  if (a.N <= 64) return run_pw<KS, 4>(a, 1, s);
  return run_pw<KS, 8>(a, (a.N + 127) / 128, s);
}

}  // namespace

bool pw_applicable(const GemmArgs& a) {
  if (a.act != ACT_NONE && a.act != ACT_SILU) return false;
  if (a.c32 || a.res32 || !a.c16) return false;
  if ((a.N & 7) || (a.K & 7) || a.K > 256 || a.M < 2048) return false;
  if (!(a.K <= 128 || a.N <= 256)) return false;
  const size_t lim = (size_t)1 << 31;
  const size_t rows = (size_t)a.M + 256;
  return rows * a.lda * 2 < lim && rows * a.ldc * 2 < lim && rows * (a.res16 ? a.ldr : 0) * 2 < lim;
}

hipError_t launch_pw(const GemmArgs& a, hipStream_t s) {
  switch ((a.K + 31) / 32) {
    case 1: return run_pw_ks<1>(a, s);
    case 2: return run_pw_ks<2>(a, s);
    case 3: return run_pw_ks<3>(a, s);
    case 4: return run_pw_ks<4>(a, s);
    case 5: return run_pw_ks<5>(a, s);
    case 6: return run_pw_ks<6>(a, s);
    case 7:
    case 8: return run_pw_ks<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}
