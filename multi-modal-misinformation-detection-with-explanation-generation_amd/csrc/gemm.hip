// fp16 MFMA GEMM for gfx950: C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ residual), fp32 accumulate.
//
// Used for every dense contraction of the hot path: RoBERTa / CLIP QKV, out-proj, FFN (SURVEY.md
// §2.1), the CLIP patch embedding (im2col GEMM), the CLIP projections and the EfficientNet 1x1
// convolutions (BatchNorm folded into W/bias; SE excitation folded into the A load).
//
// Design (CDNA4, 64-wide waves):
//  * 256 threads = 4 waves in a WGM x WGN grid; each wave owns a (BM/WGM) x (BN/WGN) output block
//    of 16x16 tiles computed with v_mfma_f32_16x16x32_f16.
//  * Operands are "swapped" (MFMA A-operand = W rows, B-operand = A rows) so that each lane ends
//    with 4 CONSECUTIVE output columns of one row -> 16-B fp32 / 8-B fp16 epilogue stores and
//    vector bias/residual loads.
//  * BK = 64: LDS tiles [rows][64] fp16 (128-B rows) with an XOR swizzle (16-B chunk ^= row & 7)
//    that makes the 16-lane ds_read_b128 fragment reads conflict-free; double-buffered, register
//    staged (next tile's global loads issued before the MFMAs, written to LDS after them).
//  * XCD-aware bijective block remap so consecutive tiles of one row panel share an XCD's L2.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;

template <int BM, int BN, int WGM, int WGN>
struct Cfg {
  static constexpr int TM = BM / WGM, TN = BN / WGN;
  static constexpr int MI = TM / 16, NI = TN / 16;
  static constexpr int XC = BM * 8 / 256;  // 16-B chunks per thread, A tile
  static constexpr int WC = BN * 8 / 256;  // 16-B chunks per thread, W tile
  static_assert(WGM * WGN == 4, "4 waves");
  static_assert(MI >= 1 && NI >= 1, "tile");
  static_assert(XC >= 1 && WC >= 1, "chunking");
};

MMF_DEV int swz(int row, int kc) { return row * BK + ((kc ^ (row & 7)) << 3); }

// PF = 2: the global loads of K-step kt + 2 are issued at step kt into a second register set, so
// two K-steps of compute cover each load's latency instead of one (long-K, few-workgroup launches:
// the EfficientNet SE-scaled projects, M = B * 49 or B * 196 rows, K = 480 ... 1152)
// ASC: the A operand carries an SE scale (g.ascale); instantiated apart so that plain launches keep
// their register budget
template <int BM, int BN, int WGM, int WGN, int PF = 1, bool ASC = false>
__global__ __launch_bounds__(256) void gemm_f16_kernel(GemmArgs g, int tilesN) {
  using C = Cfg<BM, BN, WGM, WGN>;
  __shared__ __attribute__((aligned(16))) f16_t lds[2 * (BM + BN) * BK];
  auto Xs = [&](int buf) { return lds + buf * (BM + BN) * BK; };
  auto Ws = [&](int buf) { return lds + buf * (BM + BN) * BK + BM * BK; };

  // XCD-aware bijective remap of the 1-D grid
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tilesN, tn = wgid - tm * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  if (gridDim.y > 1) {  // split-K slice z: K-range [z*K, (z+1)*K) (g.K = slice depth), fp32 partials
    const int z = blockIdx.y;
    g.A += (size_t)z * g.K;
    g.W += (size_t)z * g.K;
    g.c32 += (size_t)z * g.M * g.ldc;
  }
  const int M = g.M, N = g.N, K = g.K;
  const int nk = (K + BK - 1) / BK;

  // A chunks are loaded raw with their SE scales (ascale: 8 fp32 per 16-B chunk) and scaled when
  // they are stored to LDS: the loads stay in flight under the compute phase (scaling at load
  // time made every K-step wait for its own loads)
  uint4 xr[C::XC], wr[C::WC];
  float4 sr[ASC ? C::XC : 1][2];
  uint4 xr2[PF == 2 ? C::XC : 1], wr2[PF == 2 ? C::WC : 1];
  float4 sr2[PF == 2 && ASC ? C::XC : 1][2];

  auto load_to = [&](int kt, uint4* xd, float4 (*sd)[2], uint4* wd) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < C::XC; ++i) {
      const int c = tid + 256 * i, row = c >> 3, kc = c & 7;
      const int m = m0 + row, k = k0 + kc * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      float4 s0 = make_float4(1.f, 1.f, 1.f, 1.f), s1 = s0;
      if (m < M && k < K) {
        v = *reinterpret_cast<const uint4*>(g.A + (size_t)m * g.lda + k);
        if constexpr (ASC) {
          const float* sp = g.ascale + (size_t)(m / g.rows_per_batch) * K + k;
          s0 = *reinterpret_cast<const float4*>(sp);
          s1 = *reinterpret_cast<const float4*>(sp + 4);
        }
      }
      xd[i] = v;
      if constexpr (ASC) {
        sd[i][0] = s0;
        sd[i][1] = s1;
      }
    }
#pragma unroll
    for (int i = 0; i < C::WC; ++i) {
      const int c = tid + 256 * i, row = c >> 3, kc = c & 7;
      const int n = n0 + row, k = k0 + kc * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < N && k < K) v = *reinterpret_cast<const uint4*>(g.W + (size_t)n * g.ldw + k);
      wd[i] = v;
    }
  };
  auto store_from = [&](int buf, const uint4* xs, const float4 (*ss)[2], const uint4* ws) {
#pragma unroll
    for (int i = 0; i < C::XC; ++i) {
      const int c = tid + 256 * i;
      uint4 v = xs[i];
      if constexpr (ASC) {  // SE excitation, rounded to fp16 like the unscaled operand
        const float4 s0 = ss[i][0], s1 = ss[i][1];
        v.x = pack2h(lo_h(v.x) * s0.x, hi_h(v.x) * s0.y);
        v.y = pack2h(lo_h(v.y) * s0.z, hi_h(v.y) * s0.w);
        v.z = pack2h(lo_h(v.z) * s1.x, hi_h(v.z) * s1.y);
        v.w = pack2h(lo_h(v.w) * s1.z, hi_h(v.w) * s1.w);
      }
      *reinterpret_cast<uint4*>(Xs(buf) + swz(c >> 3, c & 7)) = v;
    }
#pragma unroll
    for (int i = 0; i < C::WC; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<uint4*>(Ws(buf) + swz(c >> 3, c & 7)) = ws[i];
    }
  };

  f32x4 acc[C::NI][C::MI];
#pragma unroll
  for (int i = 0; i < C::NI; ++i)
#pragma unroll
    for (int j = 0; j < C::MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_to(0, xr, sr, wr);
  store_from(0, xr, sr, wr);
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  auto compute = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 wf[C::NI], xf[C::MI];
#pragma unroll
      for (int i = 0; i < C::NI; ++i) {
        const int row = wn * C::TN + i * 16 + fr;
        wf[i] = as_f16x8(*reinterpret_cast<const uint4*>(Ws(buf) + swz(row, ks * 4 + fg)));
      }
#pragma unroll
      for (int j = 0; j < C::MI; ++j) {
        const int row = wm * C::TM + j * 16 + fr;
        xf[j] = as_f16x8(*reinterpret_cast<const uint4*>(Xs(buf) + swz(row, ks * 4 + fg)));
      }
#pragma unroll
      for (int i = 0; i < C::NI; ++i)
#pragma unroll
        for (int j = 0; j < C::MI; ++j) acc[i][j] = mfma16x16x32(wf[i], xf[j], acc[i][j]);
    }
  };
  if constexpr (PF == 2) {
    // register set A carries the odd K-steps, set B the even ones (>= 2); each set's loads are
    // issued two compute phases before its LDS store
    if (nk > 1) load_to(1, xr, sr, wr);
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) load_to(kt + 2, xr2, sr2, wr2);
      compute(0);
      if (kt + 1 < nk) store_from(1, xr, sr, wr);
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) load_to(kt + 3, xr, sr, wr);
      compute(1);
      if (kt + 2 < nk) store_from(0, xr2, sr2, wr2);
      __syncthreads();
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load_to(kt + 1, xr, sr, wr);
      compute(buf);
      if (kt + 1 < nk) store_from(buf ^ 1, xr, sr, wr);
      __syncthreads();
    }
  }

  // epilogue: lane holds C[m][n..n+3].  All loads (bias, fp16 residual) are issued before the
  // first store and from clamped addresses (no divergent region around them): with one in-order
  // vmcnt a load issued after a store waits for that store, and a store's data VGPRs cannot be
  // rewritten until it completes, so interleaving them serialises the tail on store latency
  // (measured: the SE-scaled EfficientNet projects with a residual 16-18 % faster).
  const int mb = m0 + wm * C::TM + fr, nb = n0 + wn * C::TN + fg * 4;
  float4 bv[C::NI];
#pragma unroll
  for (int i = 0; i < C::NI; ++i) {
    const int n = min(nb + i * 16, N - 4);
    bv[i] = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  uint2 r16[C::NI][C::MI];
  if (g.res16) {
#pragma unroll
    for (int j = 0; j < C::MI; ++j)
#pragma unroll
      for (int i = 0; i < C::NI; ++i)
        r16[i][j] = *reinterpret_cast<const uint2*>(g.res16 + (size_t)min(mb + j * 16, M - 1) * g.ldr +
                                                    min(nb + i * 16, N - 4));
  }
#pragma unroll
  for (int j = 0; j < C::MI; ++j) {
#pragma unroll
    for (int i = 0; i < C::NI; ++i) {
      float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z, acc[i][j][3] + bv[i].w};
      if (g.act) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = act_apply(v[t], g.act);
      }
      if (g.res32) {
        const int m = min(mb + j * 16, M - 1), n = min(nb + i * 16, N - 4);
        const float4 rr = *reinterpret_cast<const float4*>(g.res32 + (size_t)m * g.ldr + n);
        v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
      } else if (g.res16) {
        v[0] += lo_h(r16[i][j].x); v[1] += hi_h(r16[i][j].x); v[2] += lo_h(r16[i][j].y); v[3] += hi_h(r16[i][j].y);
      }
      acc[i][j] = f32x4{v[0], v[1], v[2], v[3]};
    }
  }
  if (g.c32) {
#pragma unroll
    for (int j = 0; j < C::MI; ++j)
#pragma unroll
      for (int i = 0; i < C::NI; ++i) {
        const int m = mb + j * 16, n = nb + i * 16;
        if (m < M && n < N)
          *reinterpret_cast<float4*>(g.c32 + (size_t)m * g.ldc + n) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
  }
  if (g.c16) {
    uint2 o[C::NI][C::MI];
#pragma unroll
    for (int j = 0; j < C::MI; ++j)
#pragma unroll
      for (int i = 0; i < C::NI; ++i) {
        o[i][j] = make_uint2(pack2h(acc[i][j][0], acc[i][j][1]), pack2h(acc[i][j][2], acc[i][j][3]));
        asm volatile("" : "+v"(o[i][j].x), "+v"(o[i][j].y)::"memory");
      }
#pragma unroll
    for (int j = 0; j < C::MI; ++j)
#pragma unroll
      for (int i = 0; i < C::NI; ++i) {
        const int m = mb + j * 16, n = nb + i * 16;
        if (m < M && n < N) *reinterpret_cast<uint2*>(g.c16 + (size_t)m * g.ldc + n) = o[i][j];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Large-tile kernel for the encoder GEMMs (K % 64 == 0): 512 threads = 8 waves, 256-row tiles,
// operands staged HBM/L2 -> LDS directly with global_load_lds_dwordx4 (no VGPR round trip, no
// ds_write).  The LDS image keeps the same XOR swizzle as above; because an LDS-DMA writes
// lane-linearly (base + 16*lane), the swizzle is applied to each lane's SOURCE address instead.
// Two LDS stages: the next K-tile's DMA is in flight while the current one feeds the MFMAs.
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

template <int ROWS, int NW>
MMF_DEV void glds_tile(const f16_t* __restrict__ G, int ld, int row0, int rowmax, int k0, f16_t* tile, int wave,
                       int lane) {
  constexpr int PER_WAVE = ROWS / (8 * NW);  // 1-KB segments (8 rows x 128 B) per wave
  static_assert(PER_WAVE * 8 * NW == ROWS, "rows must split evenly over the waves");
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int seg = wave * PER_WAVE + j;
    const int r = seg * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (lane >> 3);  // logical chunk stored at physical slot (lane & 7) of row r
    int grow = row0 + r;
    grow = grow < rowmax ? grow : rowmax - 1;  // clamped rows are loaded but never stored
    const f16_t* src = G + (size_t)grow * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (lds_void_t*)((__attribute__((address_space(3))) f16_t*)tile + seg * 512),
                                     16, 0, 0);
  }
}

// The same fill through a buffer descriptor (buffer_load_dwordx4 ... lds): the per-lane part of
// the source address is ONE loop-invariant VGPR (lane_off: row within the 8-row piece, swizzled
// chunk), the piece's row base and k0 ride in the scalar soffset.  glds_tile keeps a 64-bit
// pointer per piece live across the K loop (20 VGPRs for 640 rows), which the 256x384 tiles'
// accumulators leave no room for.  Full tiles only (soffset is outside the descriptor's range
// check; the caller takes glds_tile for a ragged last row panel).
template <int ROWS, int NW>
MMF_DEV void glds_tile_buf(rsrc_t r, uint32_t row_bytes, int row0, int k0, uint32_t lane_off, f16_t* tile, int wave) {
  constexpr int PER_WAVE = ROWS / (8 * NW);
  static_assert(PER_WAVE * 8 * NW == ROWS, "rows must split evenly over the waves");
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int seg = wave * PER_WAVE + j;
    const uint32_t soff = (uint32_t)(row0 + seg * 8) * row_bytes + (uint32_t)k0 * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)((__attribute__((address_space(3))) f16_t*)tile + seg * 512),
                                             16, lane_off, soff, 0, 0);
  }
}

// Tile t -> (row panel, column panel).  gm > 0: grouped order -- gm row panels are walked
// column by column, so the tiles one XCD runs together share A panels and W panels in its L2.
MMF_DEV void tile_coords(int t, int tilesM, int tilesN, int gm, int& tm, int& tn) {
  if (gm <= 0) {
    tm = t / tilesN;
    tn = t - tm * tilesN;
    return;
  }
  const int per_group = gm * tilesN, group = t / per_group, first_m = group * gm;
  const int gsz = min(tilesM - first_m, gm), r = t - group * per_group;
  tm = first_m + r % gsz;
  tn = r / gsz;
}

// Lazy LayerNorm (GemmArgs::epi, option lazy_ln) for the pre-LN CLIP encoders: no LayerNorm is
// materialised.
//  * a "producer" (out-projection / FFN-2, N = hidden width, 256x192 tiles, epi 2) adds the raw
//    fp16 residual stream in its epilogue, stores the new stream in place and, per row and per
//    wave, the partial statistics (mean, M2) of the STORED values over the wave's 96 columns;
//  * a "consumer" (QKV / FFN-1, epi 1) reads the stream s itself as its A operand against
//    W' = W diag(gamma) and finishes LN(s) W^T + b = r (s W'^T - mean u) + c with u = W' 1 and
//    c = b + W beta (folded on the host), mean / r = rstd from the partials (Chan's combination).
// The partials of a consumer tile's 256 rows and its column vectors (u, c) are LDS-DMA'd during
// the second K-step and combined into (mean, rstd) per row at the top of the third.
constexpr int kLnPMax = 8;  // partials per row a reader accepts

// Attention epilogue (EPI 3; RoBERTa layers with L = 128, option qkv_attn).  The tile is 256 rows =
// two whole sequences x 192 columns = q | k | v of head tn (the QKV weight's rows interleaved per
// head on the host).  Its values, rounded to fp16 exactly as the plain epilogue stores them, go to
// LDS rows [key][64] in attention.hip's swizzle; then each of the 8 waves runs attention_kernel's
// arithmetic (S^T = K Q^T, exp2-domain masked softmax, O^T = V^T P^T with V^T by transposed LDS
// reads) for two 16-query tiles of one sequence and stores its ctx rows -- so ctx is bit-identical to
// the QKV GEMM + attention_kernel<128> pair, without qkv's HBM round trip or the second launch.
// win: 96 KB of LDS -- q of sequence s at win + 8192 s, k at win + 16384 + 16384 s, v 8192 after it.
template <int MI, int NI>
MMF_DEV void attention_epilogue(const GemmArgs& g, const f32x4 (&acc)[NI][MI], const float4 (&bias_r)[NI], f16_t* win,
                                float* kbias, int m0, int head, int M, int wm, int wn, int wave, int tid, int fr,
                                int fg) {
  constexpr int TM = MI * 16, TN = NI * 16;
  f16_t* qs = win;
  f16_t* kvs = win + 16384;
#pragma unroll
  for (int j = 0; j < MI; ++j) {
    const int row = wm * TM + j * 16 + fr, sq = row >> 7, key = row & 127;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = wn * TN + i * 16 + fg * 4, part = c >> 6, d = c & 63;
      const float4 bi = bias_r[i];
      const uint2 pk = make_uint2(pack2h(acc[i][j][0] + bi.x, acc[i][j][1] + bi.y),
                                  pack2h(acc[i][j][2] + bi.z, acc[i][j][3] + bi.w));
      f16_t* dst = part == 0 ? qs + sq * 8192 : kvs + sq * 16384 + (part - 1) * 8192;
      *reinterpret_cast<uint2*>(dst + swz(key, d >> 3) + (d & 7)) = pk;
    }
  }
  if (tid < 256) {  // key bias of the two sequences (rows past M: masked, their queries not stored)
    const bool keep = m0 + tid < M && (!g.amask || g.amask[(size_t)m0 + tid] != 0);
    kbias[tid] = keep ? 0.f : -INFINITY;
  }
  __syncthreads();
  const int sq = wave >> 2, wq = wave & 3;
  if (m0 + sq * 128 < M) {
    const f16_t* Ks = kvs + sq * 16384;
    const f16_t* Vs = Ks + 8192;
    const f16_t* Qs = qs + sq * 8192;
    const float* kb = kbias + sq * 128;
    constexpr int NKT = 8, NQ = 2;  // the wave's two 16-query tiles share every K / V fragment read
    f16x8 qf[NQ][2];
#pragma unroll
    for (int it = 0; it < NQ; ++it)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        qf[it][ks] = as_f16x8(*reinterpret_cast<const uint4*>(Qs + swz((wq + 4 * it) * 16 + fr, ks * 4 + fg)));
    f32x4 sc[NQ][NKT];
#pragma unroll
    for (int j = 0; j < NKT; ++j) {
#pragma unroll
      for (int it = 0; it < NQ; ++it) sc[it][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 kf = as_f16x8(*reinterpret_cast<const uint4*>(Ks + swz(j * 16 + fr, ks * 4 + fg)));
#pragma unroll
        for (int it = 0; it < NQ; ++it) sc[it][j] = mfma16x16x32(kf, qf[it][ks], sc[it][j]);
      }
    }
    constexpr float kScaleLog2e = 0.125f * 1.44269504088896341f;
    float inv[NQ];
#pragma unroll
    for (int it = 0; it < NQ; ++it) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < NKT; ++j) {
        const float4 kbv = *reinterpret_cast<const float4*>(kb + j * 16 + fg * 4);
        const float kbr[4] = {kbv.x, kbv.y, kbv.z, kbv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = fmaf(sc[it][j][r], kScaleLog2e, kbr[r]);
          sc[it][j][r] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (mx == -INFINITY) mx = 0.f;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < NKT; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[it][j][r] - mx);
          sc[it][j][r] = e;
          sum += e;
        }
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      inv[it] = sum == 0.f ? 0.f : 1.0f / sum;  // (a non-finite sum propagates: norm.hip overflow sentinel)
    }
    f32x4 o[NQ][4];
#pragma unroll
    for (int it = 0; it < NQ; ++it)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[it][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kq = 0; kq < NKT / 2; ++kq) {
      f16x8 pf[NQ];
#pragma unroll
      for (int it = 0; it < NQ; ++it)
        pf[it] = as_f16x8(make_uint4(pack2h(sc[it][2 * kq][0], sc[it][2 * kq][1]),
                                     pack2h(sc[it][2 * kq][2], sc[it][2 * kq][3]),
                                     pack2h(sc[it][2 * kq + 1][0], sc[it][2 * kq + 1][1]),
                                     pack2h(sc[it][2 * kq + 1][2], sc[it][2 * kq + 1][3])));
      const int key0 = kq * 32 + fg * 4 + (fr >> 2), p = fr & 3;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int c = dt * 2 + (p >> 1), e = (p & 1) * 4;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + swz(key0, c) + e));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(Vs + swz(key0 + 16, c) + e));
        const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
        const f16x8 vf = as_f16x8(make_uint4(l2.x, l2.y, h2.x, h2.y));
#pragma unroll
        for (int it = 0; it < NQ; ++it) o[it][dt] = mfma16x16x32(vf, pf[it], o[it][dt]);
      }
    }
#pragma unroll
    for (int it = 0; it < NQ; ++it) {
      f16_t* dst = g.c16 + (size_t)(m0 + sq * 128 + (wq + 4 * it) * 16 + fr) * g.ldc + head * 64 + fg * 4;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<uint2*>(dst + dt * 16) = make_uint2(pack2h(o[it][dt][0] * inv[it], o[it][dt][1] * inv[it]),
                                                              pack2h(o[it][dt][2] * inv[it], o[it][dt][3] * inv[it]));
    }
  }
  __syncthreads();  // the window is the next tile's second-slab stage
}

// Diagnostic build only (-DMMF_GEMM_STAMP, tools/gemm_stamps.py): per-workgroup
// phase stamps of the persistent kernel into a buffer of its own ([workgroup][kGStampSlots]: 0 / 1 =
// s_memrealtime at start / end, 2 = number of stamps, 3.. = s_memtime at each tile's start, after its
// first K-step and after its K loop, then once after the last tile).  No output is computed from
// them.  In the production build every GST macro is empty.
#ifdef MMF_GEMM_STAMP
constexpr int kGStampSlots = 96;
__device__ unsigned long long* g_gemm_stamp;
MMF_DEV unsigned long long gst_time() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define GST_INIT()                                                                                           \
  unsigned long long* gst_ = (g_gemm_stamp && blockIdx.x < 256u) ? g_gemm_stamp + (size_t)blockIdx.x * kGStampSlots \
                                                                 : nullptr;                                  \
  int gst_n_ = 3;                                                                                            \
  bool gst_first_ = true;                                                                                    \
  {                                                                                                          \
    const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                                          \
    const unsigned long long m_ = gst_time();                                                                \
    if (gst_ && threadIdx.x == 0) { gst_[0] = r_; gst_[kGStampSlots - 2] = m_; }                             \
  }
#if MMF_GEMM_STAMP == 2
// phase mode (-DMMF_GEMM_STAMP=2, tools/gemm_stamps.py --phases): wave 0 of each
// workgroup stamps 4 points of K-steps 1 .. 20 of its FIRST tile -- step start, after the LDS-DMA
// issue, after the last MFMA issue, after the step barrier -- into slots 3 + 4 (kt - 1) + p
#define GST() {}
#define GSTP(p)                                                                                              \
  if (gst_first_ && kt >= 1 && kt <= 20) {                                                                   \
    const unsigned long long t_ = gst_time();                                                                \
    if (gst_ && threadIdx.x == 0) gst_[3 + 4 * (kt - 1) + (p)] = t_;                                          \
  }
#else
#define GSTP(p)
#define GST()                                                                                                \
  {                                                                                                          \
    const unsigned long long t_ = gst_time();                                                                \
    if (gst_ && threadIdx.x == 0 && gst_n_ < kGStampSlots - 2) gst_[gst_n_] = t_;                                \
    ++gst_n_;                                                                                                \
  }
#endif
#define GST_TILE_DONE() gst_first_ = false;
#define GST_END()                                                                                            \
  {                                                                                                          \
    GST()                                                                                                    \
    const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                                          \
    const unsigned long long m_ = gst_time();                                                                \
    if (gst_ && threadIdx.x == 0) { gst_[1] = r_; gst_[2] = (unsigned long long)gst_n_; gst_[kGStampSlots - 1] = m_; } \
  }
#else
#define GST_INIT()
#define GST()
#define GSTP(p)
#define GST_TILE_DONE()
#define GST_END()
#endif

#ifndef MMF_DMA_ILV
#define MMF_DMA_ILV 1  // LDS-DMA pieces interleaved with the MFMAs of the PIPE2 K loop (gemm_glds_body.inc; 0: A/B builds)
#endif
#ifndef MMF_ILV_G192
#define MMF_ILV_G192 0  // 256x192 plain / producer tiles: 0 = up-front issue, g = interleaved over g groups (A/B builds)
#endif

#ifndef MMF_GLDS_BUF
#define MMF_GLDS_BUF 1  // descriptor LDS-DMA fills for full panels (0: 64-bit-address fills everywhere; A/B builds)
#endif

// DBG (measurement builds, forced configs 15 / 16 only; outputs garbage): 1 = LDS-DMA + barriers only,
// 2 = fragment reads + MFMAs + barriers only
template <int BM, int BN, int WGM, int WGN, int ACT, bool PIPE2 = false, int EPI = 0, int DBG = 0>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_glds_kernel(GemmArgs g, int tilesN, int tiles, int tilesM,
                                                                       int gm) {
#define MMF_GLDS_FIRST_TILE wgid
#include "gemm_glds_body.inc"
#undef MMF_GLDS_FIRST_TILE
}

// persistent grid: one workgroup per CU (256 CUs), fewer when the launch has fewer tiles
template <int BM, int BN, int WGM, int WGN, bool PIPE2 = false, int DBG = 0>
hipError_t run_glds(const GemmArgs& a, hipStream_t s) {
  const int tilesM = (a.M + BM - 1) / BM, tilesN = (a.N + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  const int grid = tiles < 256 ? tiles : 256;
  const dim3 blk(64 * WGM * WGN);
  const int gm = a.group_m;  // tile-order option (handle option "gemm_group_m"; 0 = row-major)
#define MMF_GLDS_CASE(ACT)                                                                                  \
  case ACT:                                                                                                 \
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WGM, WGN, ACT, PIPE2, 0, DBG>), dim3(grid), blk, 0, s, a, tilesN, tiles, \
                       tilesM, gm);                                                                          \
    break;
  if constexpr (DBG != 0) {
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WGM, WGN, ACT_NONE, PIPE2, 0, DBG>), dim3(grid), blk, 0, s, a, tilesN,
                       tiles, tilesM, gm);
    return hipGetLastError();
  }
  switch (a.act) {
    MMF_GLDS_CASE(ACT_NONE)
    MMF_GLDS_CASE(ACT_GELU)
    MMF_GLDS_CASE(ACT_QUICK_GELU)
    MMF_GLDS_CASE(ACT_SILU)
    MMF_GLDS_CASE(ACT_RELU)
    default:
      return hipErrorInvalidValue;
  }
#undef MMF_GLDS_CASE
  return hipGetLastError();
}

// lazy-LN / attention epilogues (pipelined 256-row tiles only)
template <int BM, int BN, int WGM, int WGN>
hipError_t run_glds_epi(const GemmArgs& a, hipStream_t s) {
  const int tilesM = (a.M + BM - 1) / BM, tilesN = (a.N + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  const int grid = tiles < 256 ? tiles : 256;
  const dim3 blk(64 * WGM * WGN);
  const int gm = a.group_m;
#define MMF_EPI_CASE(EPI, ACT)                                                                                 \
  hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WGM, WGN, ACT, true, EPI>), dim3(grid), blk, 0, s, a, tilesN, tiles, \
                     tilesM, gm)
  if (a.epi == 1) {
    switch (a.act) {
      case ACT_NONE: MMF_EPI_CASE(1, ACT_NONE); break;
      case ACT_GELU: MMF_EPI_CASE(1, ACT_GELU); break;
      case ACT_QUICK_GELU: MMF_EPI_CASE(1, ACT_QUICK_GELU); break;
      default: return hipErrorInvalidValue;
    }
  } else if (a.epi == 4) {
    if (a.act != ACT_GELU) return hipErrorInvalidValue;
    MMF_EPI_CASE(4, ACT_GELU);
  } else if (a.act != ACT_NONE || BN != 192) {
    return hipErrorInvalidValue;
  } else if (a.epi == 2) {
    if constexpr (BN == 192) MMF_EPI_CASE(2, ACT_NONE);
  } else if (a.epi == 3) {
    if constexpr (BN == 192) MMF_EPI_CASE(3, ACT_NONE);
  } else {
    return hipErrorInvalidValue;
  }
#undef MMF_EPI_CASE
  return hipGetLastError();
}

#ifndef MMF_GEMM_PF2_K
#define MMF_GEMM_PF2_K 0  // K from which the 2-deep register prefetch is used (0 = never; A/B builds)
#endif
template <int BM, int BN, int WGM, int WGN>
hipError_t run(const GemmArgs& a, hipStream_t s) {
  const int tilesM = (a.M + BM - 1) / BM, tilesN = (a.N + BN - 1) / BN;
  const dim3 grid(tilesM * tilesN);
  const bool pf2 = MMF_GEMM_PF2_K > 0 && a.K >= MMF_GEMM_PF2_K;
  if (a.ascale) {
    if (pf2) hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WGM, WGN, 2, true>), grid, dim3(256), 0, s, a, tilesN);
    else hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WGM, WGN, 1, true>), grid, dim3(256), 0, s, a, tilesN);
  } else {
    if (pf2) hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WGM, WGN, 2>), grid, dim3(256), 0, s, a, tilesN);
    else hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WGM, WGN>), grid, dim3(256), 0, s, a, tilesN);
  }
  return hipGetLastError();
}

// Split-K reduction: C = act(sum_z P[z] + bias) (+ residual), the epilogue of gemm_f16_kernel
// in the same order; one thread per 4 consecutive columns.  res32 may alias c32 (in place).
template <int ACT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P, int S, GemmArgs g) {
  const int nq = g.N >> 2;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= g.M * nq) return;
  const int m = idx / nq, n = (idx - m * nq) * 4;
  const size_t plane = (size_t)g.M * g.N;
  const float* p = P + (size_t)m * g.N + n;
  float4 acc = *reinterpret_cast<const float4*>(p);
  int z = 1;
  for (; z + 4 <= S; z += 4) {  // four slices' loads in flight, added in slice order
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(p + (z + u) * plane);
#pragma unroll
    for (int u = 0; u < 4; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  for (; z < S; ++z) {
    const float4 v = *reinterpret_cast<const float4*>(p + z * plane);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  float v[4] = {acc.x, acc.y, acc.z, acc.w};
  if (g.bias) {
    const float4 b = *reinterpret_cast<const float4*>(g.bias + n);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
  if (ACT != ACT_NONE) act4<ACT>(v);
  if (g.res32) {
    const float4 r = *reinterpret_cast<const float4*>(g.res32 + (size_t)m * g.ldr + n);
    v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
  } else if (g.res16) {
    const uint2 r = *reinterpret_cast<const uint2*>(g.res16 + (size_t)m * g.ldr + n);
    v[0] += lo_h(r.x); v[1] += hi_h(r.x); v[2] += lo_h(r.y); v[3] += hi_h(r.y);
  }
  if (g.c32) *reinterpret_cast<float4*>(g.c32 + (size_t)m * g.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
  if (g.c16)
    *reinterpret_cast<uint2*>(g.c16 + (size_t)m * g.ldc + n) = make_uint2(pack2h(v[0], v[1]), pack2h(v[2], v[3]));
}

// Skinny-M GEMMs with a deep K (the compact last encoder layers and projections, M = batch): the
// 64x128 tiles alone give 16-96 workgroups, each walking K = 768..3072 serially (latency-bound).
// Split K into S slices of 256 (grid.y = S, fp32 partials in a caller workspace) and reduce.
template <int BM, int BN, int WGM, int WGN>
hipError_t run_splitk(const GemmArgs& a, int S, hipStream_t s) {
  const int tilesM = (a.M + BM - 1) / BM, tilesN = (a.N + BN - 1) / BN;
  GemmArgs p{};
  p.A = a.A; p.lda = a.lda; p.W = a.W; p.ldw = a.ldw;
  p.c32 = a.ws; p.ldc = a.N;
  p.M = a.M; p.N = a.N; p.K = a.K / S;
  hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WGM, WGN>), dim3(tilesM * tilesN, S), dim3(256), 0, s, p, tilesN);
  const int threads = a.M * (a.N >> 2);
  const dim3 grid((threads + 255) / 256);
  switch (a.act) {
    case ACT_NONE: hipLaunchKernelGGL(splitk_reduce_kernel<ACT_NONE>, grid, dim3(256), 0, s, a.ws, S, a); break;
    case ACT_GELU: hipLaunchKernelGGL(splitk_reduce_kernel<ACT_GELU>, grid, dim3(256), 0, s, a.ws, S, a); break;
    case ACT_QUICK_GELU:
      hipLaunchKernelGGL(splitk_reduce_kernel<ACT_QUICK_GELU>, grid, dim3(256), 0, s, a.ws, S, a);
      break;
    case ACT_SILU: hipLaunchKernelGGL(splitk_reduce_kernel<ACT_SILU>, grid, dim3(256), 0, s, a.ws, S, a); break;
    case ACT_RELU: hipLaunchKernelGGL(splitk_reduce_kernel<ACT_RELU>, grid, dim3(256), 0, s, a.ws, S, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

// The LDS-DMA kernel addresses its epilogue operands with 32-bit raw-buffer byte offsets.
static bool glds_ok(const GemmArgs& a) {
  const size_t lim = (size_t)1 << 31;
  const size_t rows = (size_t)a.M + 256;
  // (the interleaved LDS-DMA, MMF_DMA_ILV, forms every operand offset -- rows up to M + 255 / N + 255 --
  // as one 32-bit voffset)
  const size_t lim32 = (size_t)1 << 32;
  return (a.K % BK) == 0 && !a.ascale && rows * a.ldc * 4 < lim && rows * (a.ldr > 0 ? a.ldr : 0) * 4 < lim &&
         rows * (size_t)a.lda * 2 < lim32 && ((size_t)a.N + 256) * a.ldw * 2 < lim32;
}

#ifndef MMF_GEMM_DIAG
#define MMF_GEMM_DIAG 0  // 1: the measurement builds of the 256x192 kernel (forced configs 15 / 16; tools/)
#endif

// Instantiations launch_gemm can run (the rest of the numbering belonged to variants measured slower
// and removed in round 5 -- 128-row and 256x384 tiles, the ring / loader-consumer kernels, the 4-wave
// 256x192 tile: DESIGN.md §3 records each measurement and its last commit).
static bool config_exists(int c) {
  return c == 0 || c == 1 || c == 2 || c == 3 || c == 5 || c == 9 || c == 10 || c == 11 ||
         (MMF_GEMM_DIAG && (c == 15 || c == 16));
}

static int forced_config(const GemmArgs& a) {
  // handle option "gemm_config" (benchmarking override, tools/gemm_bench.py); ignored if inapplicable
  if (a.force_cfg <= 0) return -1;
  const int c = a.force_cfg - 1;
  if (!config_exists(c)) return -1;
  if ((c == 5 || c >= 10) && !glds_ok(a)) return -1;
  if (c == 9 && !pw_applicable(a)) return -1;
  return c;
}

// persistent 256-row LDS-DMA tiles: the column tile that minimises whole "rounds" of 256 CUs x
// per-tile time (wider tiles are more efficient per flop); with_128 = also consider 256x128
static int glds_pick(const GemmArgs& a, bool with_128) {
  // (the 256- and 192-column tiles run the half-step-pipelined K loop, configs 11 / 10)
  const long tm = (a.M + 255) / 256;
  const int bns[3] = {256, 192, 128}, cfg[3] = {11, 10, 5};
  const double eff[3] = {1.0, 0.88, 0.80};  // measured per-flop efficiency (tools/gemm_bench.py)
  int best = 11;
  double bc = 1e30;
  for (int i = 0; i < (with_128 ? 3 : 2); ++i) {
    const long tiles = tm * ((a.N + bns[i] - 1) / bns[i]);
    const double c = (double)((tiles + 255) / 256) * bns[i] / eff[i];
    if (c < bc) { bc = c; best = cfg[i]; }
  }
  return best;
}

int gemm_config(const GemmArgs& a) {
  // producers: 256x192 tiles, 96-column partials (P = ceil(N / 96) <= kLnPMax), decided from N
  // only, so a row's statistics (and so its result) do not depend on the batch it runs in
  if (a.epi == 2 || a.epi == 3) return 10;
  const int f = forced_config(a);
  if (a.epi == 1 || a.epi == 4) return (f == 10 || f == 11) ? f : glds_pick(a, false);
  if (f >= 0) return f;
  if (pw_applicable(a)) return 9;  // HBM-bound 1x1 convolutions (pointwise.hip)
  if (a.N <= 32) return 0;
  if (a.N <= 64) return 1;
  if (a.M <= 512) return 2;  // skinny-M (projections, M = batch)
  if (glds_ok(a) && a.N >= 128) return glds_pick(a, true);
  // register-staged tiles (e.g. the SE-scaled EfficientNet projects): 64x128 tiles when 128x128
  // ones would leave the chip short of workgroups (late stages, M = B * 7^2, K = 1152)
  const long t128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128);
  return t128 < 384 ? 2 : 3;
}

int gemm_splitk_factor(const GemmArgs& a) {
  // slices of 256 (4 K-steps) when that gives >= 2 of them; the partial planes need N % 4 == 0
  // and 16-B aligned rows for the reduction's float4 accesses
  if (a.ascale || (a.K % 256) || a.K < 512 || (a.N & 3) || (a.ldc & 3) || (a.ldr & 3)) return 1;
  if (a.no_splitk) return 1;  // handle option "gemm_splitk" = 0 (A/B tests)
  return a.K / 256;
}

int gemm_ln_tn(const GemmArgs&) { return 96; }

// what the lazy-LN epilogues need (the host mirrors it before choosing that path)
static bool epi_ok(const GemmArgs& a) {
  if (!glds_ok(a) || a.K < 3 * BK || a.M <= 0) return false;  // partials DMA'd at kt = 1, combined at kt = 2
  if (a.epi == 1)
    return a.ln_in && a.ln_u && a.bias && a.c16 && !a.c32 && !a.res16 && !a.res32 && a.ln_in_P >= 1 && a.ln_in_P <= kLnPMax &&
           a.ln_in_tn > 0 && (long)a.ln_in_P * a.ln_in_tn >= a.K;
  if (a.epi == 2) return a.c16 && !a.c32 && a.res16 && !a.res32 && a.ln_out && (a.N + 95) / 96 <= kLnPMax;
  if (a.epi == 3)  // whole 128-row sequences, whole heads (192 = q | k | v columns of one head)
    return a.c16 && !a.c32 && !a.res16 && !a.res32 && a.bias && a.act == ACT_NONE && a.N % 192 == 0 &&
           a.M % 128 == 0 && a.ldc >= a.N / 3;
  if (a.epi == 4)
    return a.c16 && !a.c32 && !a.res16 && !a.res32 && a.bias && a.act == ACT_GELU && a.N % 8 == 0 &&
           a.ldc >= (a.split_lo ? 3 * a.N : a.N) && (size_t)(a.M + 256) * a.ldc * 2 < ((size_t)1 << 31);
  return false;
}

bool gemm_epi_ok(const GemmArgs& a) { return epi_ok(a); }

const char* gemm_config_name(int c) {
  static const char* names[kGemmConfigs] = {
      "gemm_f16<256,32,4,1>", "gemm_f16<256,64,4,1>", "gemm_f16<64,128,1,4>", "gemm_f16<128,128,2,2>", "(removed)",
      "gemm_glds<256,128,4,2>", "(removed)", "(removed)", "(removed)", "pw_conv", "gemm_glds_pipe2<256,192,4,2>",
      "gemm_glds_pipe2<256,256,2,4>", "(removed)", "(removed)", "(removed)", "gemm_glds_dma_only",
      "gemm_glds_compute_only"};
  return (c >= 0 && c < kGemmConfigs) ? names[c] : "gemm_f16<?>";
}

#ifdef MMF_GEMM_STAMP
// diagnostic build: where the persistent GEMM writes its stamps (nullptr = off)
extern "C" int mmf_debug_gemm_stamp(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamp), &buf, sizeof(buf));
}
#endif

hipError_t launch_gemm(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return hipSuccess;
  if ((a.K & 7) || (a.N & 3) || (a.lda & 7) || (a.ldw & 7) || (a.ldc & 3)) return hipErrorInvalidValue;
  if (a.epi != 0) {
    if (!epi_ok(a)) return hipErrorInvalidValue;
    return gemm_config(a) == 11 ? run_glds_epi<256, 256, 2, 4>(a, s) : run_glds_epi<256, 192, 4, 2>(a, s);
  }
  const int cfg = gemm_config(a);
#if MMF_GEMM_DIAG
  if (cfg == 15) return run_glds<256, 192, 4, 2, true, 1>(a, s);
  if (cfg == 16) return run_glds<256, 192, 4, 2, true, 2>(a, s);
#endif
  switch (cfg) {
    case 0: return run<256, 32, 4, 1>(a, s);
    case 1: return run<256, 64, 4, 1>(a, s);
    case 2: {
      const int S = gemm_splitk_factor(a);
      if (S > 1 && a.ws && (size_t)S * a.M * a.N <= a.ws_elems) return run_splitk<64, 128, 1, 4>(a, S, s);
      return run<64, 128, 1, 4>(a, s);
    }
    case 5: return run_glds<256, 128, 4, 2>(a, s);
    case 9: return launch_pw(a, s);
    case 10: return run_glds<256, 192, 4, 2, true>(a, s);
    case 11: return run_glds<256, 256, 2, 4, true>(a, s);
    default: return run<128, 128, 2, 2>(a, s);
  }
}
