// Ring-pipelined fp16 MFMA GEMM for the encoder shapes (gfx950): C[M,N] = act(A . W^T + bias), fp16 out.
//
// Why (profiles/r03_gemm_pmc.txt): the two-stage LDS-DMA kernel of gemm.hip
// (gemm_glds_kernel) waits vmcnt(0) + barrier at the end of every 64-deep K-step, so each step costs
// one full DMA round trip: its waves spend 0.31-0.38 of their cycles parked at that wait
// (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the MFMA pipe is busy 0.38-0.44 of the time.  This kernel
// keeps the DMA of the next NS-2 stages in flight across the barriers:
//  * persistent 512-thread workgroups (8 waves, 4 x 2), 256 x 192 output tiles, wave tile 64 x 96;
//  * K in 32-deep stages (A 256 x 32 + W 192 x 32 fp16 = 28 KB) in an NS-slot LDS ring; stage g+NS-1
//    is issued at the top of step g, so NS-2 stages (56-84 KB) are in flight under the MFMAs;
//  * the LDS-DMA (global_load_lds_dwordx4) is issued from inline asm: hipcc neither counts it nor
//    orders its own LDS reads behind it, so there is no compiler vmcnt(0) anywhere in the loop --
//    each step waits with a COUNTED vmcnt for exactly the stage it is about to read, then one
//    s_barrier (in the same asm statement, so no LDS read can be scheduled above it);
//  * fragments of stage g+1 are read (ds_read_b128, conflict-free 64-B-row swizzle) while the
//    MFMAs of stage g run (sched_group_barrier interleave), from two register sets;
//  * the epilogue's bias comes through LDS (DMA'd with the tile's first stage), so no
//    compiler-visible global load -- which hipcc would wait for with vmcnt(0), draining the ring
//    -- exists in the kernel; the epilogue's 12 stores per lane are counted into the waits of the
//    next NS-2 steps (a store is a vector-memory op on the same in-order counter).
// Per output element the MFMA accumulation order (32-deep chunks in ascending K) is the one of
// gemm_glds_kernel, so both kernels return bit-identical results.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int RBM = 256, RBN = 192, RBK = 32;
constexpr int RTM = 64, RTN = 96, RMI = RTM / 16, RNI = RTN / 16;  // wave tile 64 x 96 (waves 4 x 2)
constexpr int kSlotBytes = (RBM + RBN) * RBK * 2;                    // 28 KB: A 16 KB | W 12 KB
constexpr int kWOff = RBM * RBK * 2;                                  // W part of a slot (bytes)
constexpr int kBiasBytes = 1024;                                      // one tile's bias (192 floats used)
constexpr int kStores = RMI * RNI / 2;                                // 16-B epilogue stores per lane

typedef __attribute__((address_space(3))) char lds_char;

// element offset (halfs) of logical 16-B chunk c (0..3) of row r in a slab of 64-B rows.  A
// ds_read_b128 fragment read (lane: row fr = lane & 15, chunk fg = lane >> 4) is served in four
// lane groups of 16 ({0-3,12-15,20-27}, ...); with chunk ^= 2 * bit3(row) every group touches 16
// distinct 16-B bank slots (checked against the gfx950 lane grouping, MI355X_MICROARCH.md §LDS).
MMF_DEV int rswz(int r, int c) { return r * RBK + ((c ^ (((r >> 3) & 1) << 1)) << 3); }

// one 1-KB LDS-DMA wave-instruction: lane l's 16 source bytes land at lds_byte + 16 l
MMF_DEV void dma16(const void* src, uint32_t lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_byte)
      : "memory");
}

// all but this wave's N youngest vector-memory ops complete, then the workgroup barrier
template <int N>
MMF_DEV void wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}

// DBG (measurement builds, forced configs 13 / 14 only): 1 = LDS-DMA, waits and barriers only (no
// fragment reads, no MFMA: the fill rate of the ring), 2 = no LDS-DMA (fragment reads, MFMAs and
// barriers on whatever the LDS holds: the compute side alone).  Outputs are garbage in both.
template <int ACT, int NS, int DBG = 0>
__global__ __launch_bounds__(512, 2) void gemm_ring_kernel(GemmArgs g, int tilesN, int tiles) {
  static_assert(NS >= 4, "the ring needs a slot being read, one being filled and >= 1 in flight");
  __shared__ __attribute__((aligned(16))) char lds[NS * kSlotBytes + 2 * kBiasBytes];

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  if (wgid >= tiles) return;
  const int my_tiles = (tiles - wgid + nwg - 1) / nwg;
  const int nk = g.K / RBK;  // even (K % 64 == 0): the two-step unroll below keeps fragment sets static
  const int G = my_tiles * nk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = g.M, N = g.N;
  const bool w4 = wave < 4;  // waves 0-3 DMA 4 segments per stage, waves 4-7 3 (28 = 16 A + 12 W)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
  const uint32_t out_elems = (uint32_t)(M - 1) * g.ldc + N;
  const rsrc_t rc16 = make_rsrc(g.c16, out_elems * 2u);

  // per-lane parts of the DMA addresses: segment s covers rows 16 s .. 16 s + 15 of its operand;
  // lane l fills physical row (l >> 2), 16-B slot (l & 3), which holds logical chunk slot ^ swz
  const int lrow = lane >> 2;
  auto chunk_of = [&](int row) { return (lane & 3) ^ (((row >> 3) & 1) << 1); };

  // the LDS-DMA pieces of stage gs for this wave: A segments 2w, 2w+1; W segments 2w, 2w+1
  // (waves 0-3) or 8 + (w - 4) (waves 4-7, whose 4th piece is the tile's bias at kt = 0, wave 7)
  struct Pieces { const void* src[4]; uint32_t dst[4]; bool has3; };
  auto plan = [&](int gs, Pieces& d) {
    int i = gs / nk, kt = gs - i * nk;
    if (i >= my_tiles) {  // past the last stage: re-load it (a free slot), so every step issues
      i = my_tiles - 1;   // the same number of DMAs and the counted waits stay exact
      kt = nk - 1;
    }
    const int t = wgid + i * nwg, tm = t / tilesN, tn = t - tm * tilesN;
    const int m0 = tm * RBM, n0 = tn * RBN, k0 = kt * RBK;
    const uint32_t sb = lds0 + (uint32_t)(gs % NS) * kSlotBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int sg = 2 * wave + j, row = 16 * sg + lrow;
      const int gm = min(m0 + row, M - 1);
      d.src[j] = g.A + (size_t)gm * g.lda + k0 + chunk_of(row) * 8;
      d.dst[j] = __builtin_amdgcn_readfirstlane(sb + sg * 1024);
    }
    if (w4) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sg = 2 * wave + j, row = 16 * sg + lrow;
        const int gn = min(n0 + row, N - 1);
        d.src[2 + j] = g.W + (size_t)gn * g.ldw + k0 + chunk_of(row) * 8;
        d.dst[2 + j] = __builtin_amdgcn_readfirstlane(sb + kWOff + sg * 1024);
      }
      d.has3 = true;
    } else {
      const int sg = 8 + (wave - 4), row = 16 * sg + lrow;
      const int gn = min(n0 + row, N - 1);
      d.src[2] = g.W + (size_t)gn * g.ldw + k0 + chunk_of(row) * 8;
      d.dst[2] = __builtin_amdgcn_readfirstlane(sb + kWOff + sg * 1024);
      d.has3 = kt == 0 && wave == 7;  // the tile's bias, into the buffer of its parity
      d.src[3] = g.bias + min(n0 + lane * 4, N - 4);
      d.dst[3] = __builtin_amdgcn_readfirstlane(lds0 + NS * kSlotBytes + (uint32_t)(i & 1) * kBiasBytes);
    }
  };
  auto issue = [&](int gs) {
    if constexpr (DBG == 2) return;
    Pieces d;
    plan(gs, d);
#pragma unroll
    for (int c = 0; c < 3; ++c) dma16(d.src[c], d.dst[c]);
    if (d.has3) dma16(d.src[3], d.dst[3]);
  };

  auto read_frags = [&](int gs, f16x8* wf, f16x8* xf) {
    const f16_t* xs = reinterpret_cast<const f16_t*>(lds + (gs % NS) * kSlotBytes);
    const f16_t* ws = reinterpret_cast<const f16_t*>(lds + (gs % NS) * kSlotBytes + kWOff);
#pragma unroll
    for (int i = 0; i < RNI; ++i) wf[i] = as_f16x8(*reinterpret_cast<const uint4*>(ws + rswz(wn * RTN + i * 16 + fr, fg)));
#pragma unroll
    for (int j = 0; j < RMI; ++j) xf[j] = as_f16x8(*reinterpret_cast<const uint4*>(xs + rswz(wm * RTM + j * 16 + fr, fg)));
  };

  f32x4 acc[RNI][RMI];
#pragma unroll
  for (int i = 0; i < RNI; ++i)
#pragma unroll
    for (int j = 0; j < RMI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 wa[RNI], xa[RMI], wb[RNI], xb[RMI];

  // wait for stage gs + 1 (issued at step gs - NS + 2), then the barrier.  Younger than it: the
  // NS - 3 stages issued since and, in the NS - 2 steps after an epilogue, that epilogue's stores.
  auto top_wait = [&](bool after_epi) {
    if (after_epi) {
      if (w4) wait_barrier<4 * (NS - 3) + kStores>();
      else wait_barrier<3 * (NS - 3) + kStores>();
    } else {
      if (w4) wait_barrier<4 * (NS - 3)>();
      else wait_barrier<3 * (NS - 3)>();
    }
  };
  // one 32-deep step: the wait + barrier for stage gs + 1, then the 24 MFMAs of stage gs in four
  // groups of 6 with one LDS-DMA piece of stage gs + NS - 1 issued ahead of each group and the 10
  // fragment reads of stage gs + 1 between the MFMAs (3, 3, 2, 2 per group).  A piece issued as a
  // block at the top of the step stalls both waves of a SIMD at once (measured: fill and MFMA
  // time added up, tools/gemm_bench.py configs 13 / 14); spread out, the other wave keeps the MFMA
  // pipe busy while one waits on its DMA issue.
  auto step = [&](const f16x8* wc, const f16x8* xc, int gs, f16x8* wnx, f16x8* xnx, bool after_epi) {
    top_wait(after_epi);
    Pieces d;
    if constexpr (DBG != 2) plan(gs + NS - 1, d);
    const f16_t* xs = reinterpret_cast<const f16_t*>(lds + ((gs + 1) % NS) * kSlotBytes);
    const f16_t* ws = reinterpret_cast<const f16_t*>(lds + ((gs + 1) % NS) * kSlotBytes + kWOff);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DBG != 2) {
        if (c < 3 || d.has3) dma16(d.src[c], d.dst[c]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DBG != 1) {
        constexpr int r0[5] = {0, 3, 6, 8, 10};
#pragma unroll
        for (int r = r0[c]; r < r0[c + 1]; ++r) {
          if (r < RNI) wnx[r] = as_f16x8(*reinterpret_cast<const uint4*>(ws + rswz(wn * RTN + r * 16 + fr, fg)));
          else xnx[r - RNI] = as_f16x8(*reinterpret_cast<const uint4*>(xs + rswz(wm * RTM + (r - RNI) * 16 + fr, fg)));
        }
#pragma unroll
        for (int q6 = 0; q6 < 6; ++q6) {
          const int ii = (6 * c + q6) / RMI, jj = (6 * c + q6) % RMI;
          acc[ii][jj] = mfma16x16x32(wc[ii], xc[jj], acc[ii][jj]);
        }
        // DS read, 2 MFMAs, ... (literal arguments: one call site per pattern)
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (c < 2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: NS - 1 stages in flight, stage 0 landed and read
#pragma unroll 1
  for (int p = 0; p < NS - 1; ++p) issue(p);
  if (w4) wait_barrier<4 * (NS - 2)>();
  else wait_barrier<3 * (NS - 2)>();
  read_frags(0, wa, xa);

  int gs = 0;
#pragma unroll 1
  for (int i = 0; i < my_tiles; ++i) {
    const int t = wgid + i * nwg, tm = t / tilesN, tn = t - tm * tilesN;
    const int m0 = tm * RBM, n0 = tn * RBN;
#pragma unroll 1
    for (int kt = 0; kt < nk; kt += 2) {
      step(wa, xa, gs, wb, xb, i > 0 && kt < NS - 2);
      ++gs;
      step(wb, xb, gs, wa, xa, i > 0 && kt + 1 < NS - 2);
      ++gs;
    }
    (void)G;

    // epilogue: bias (LDS) + activation, fp16 pairs of adjacent column groups swapped across lanes
    // l and l ^ 16 (v_permlane16_swap) so each lane stores 16 contiguous bytes: exactly kStores
    // stores per lane (out-of-range rows / columns are dropped by the buffer descriptor)
    const float* bias_l = reinterpret_cast<const float*>(lds + NS * kSlotBytes + (i & 1) * kBiasBytes);
#pragma unroll
    for (int j = 0; j < RMI; ++j) {
      const uint32_t m = m0 + wm * RTM + j * 16 + fr;
#pragma unroll
      for (int ii = 0; ii < RNI; ii += 2) {
        uint2 pk[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float4 bi = *reinterpret_cast<const float4*>(bias_l + wn * RTN + (ii + h2) * 16 + fg * 4);
          float v[4] = {acc[ii + h2][j][0] + bi.x, acc[ii + h2][j][1] + bi.y, acc[ii + h2][j][2] + bi.z,
                        acc[ii + h2][j][3] + bi.w};
          if (ACT != ACT_NONE) act4<ACT>(v);
          pk[h2] = make_uint2(pack2h(v[0], v[1]), pack2h(v[2], v[3]));
        }
        const bool odd = fg & 1;
        const int n8 = n0 + wn * RTN + (odd ? (ii + 1) * 16 + (fg - 1) * 4 : ii * 16 + fg * 4);
        const uint4 o = pair_rows16(pk[0], pk[1]);
        buf_store_u4(rc16, n8 < N ? (m * (uint32_t)g.ldc + n8) * 2u : kOOB, o);
      }
    }
#pragma unroll
    for (int ii = 0; ii < RNI; ++ii)
#pragma unroll
      for (int j = 0; j < RMI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // no LDS-DMA may still be writing when the workgroup's LDS is handed to the next one
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Loader / consumer split (gemm_lc_kernel).  Measured on the two kernels above (tools/gemm_bench.py,
// measurement configs 13-16): the LDS-DMA fill of a 256 x 192 tile runs at ~52 GB/s per CU
// (DMA-only: 1.07 us per 64-deep K-step of 56 KB, full 128-B lines; 64-B half lines cost 12 %
// more), the fragment reads + MFMAs alone at 0.86 us -- and the full kernels take 1.42 us (two
// stages) / 1.70 us (ring): fill and compute ADD UP, because a wave that issues LDS-DMA pieces
// stalls on their issue and every wave of the workgroup issues them.  Here 4 dedicated loader
// waves issue every piece and the 8 MFMA waves never touch the vector-memory queue in the K loop:
//  * 768 threads: waves 0-7 compute (4 x 2, wave tile 64 x 96), waves 8-11 load (14 pieces of
//    8 rows x 128 B each per stage, full lines, XOR-swizzled on the source address as gemm.hip);
//  * two 56-KB stages (BK = 64); per step the loaders issue stage k+1, wait for their own DMA
//    (vmcnt(0)) and meet the compute waves at ONE barrier, after which stage k+1 has landed and
//    stage k's slot is free -- fill of k+1 runs entirely under the MFMAs of k;
//  * the tile's bias is one more piece (loader wave 11, with the tile's first stage), so the
//    compute waves' only vector-memory ops are their epilogue stores, issued after the barrier.
// Accumulation order per element (32-deep chunks, ascending K) is the one of gemm_glds_kernel:
// bit-identical results.
// ---------------------------------------------------------------------------------------------
constexpr int LBK = 64, kLcStage = (RBM + RBN) * LBK;  // halfs per stage (56 KB)
constexpr int kLcLoaders = 4, kLcPieces = (RBM + RBN) / 8, kLcPerLoader = kLcPieces / kLcLoaders;
static_assert(kLcPieces % kLcLoaders == 0, "pieces split evenly over the loader waves");
typedef __attribute__((address_space(3))) void lds_void;

MMF_DEV int lswz(int row, int kc) { return row * LBK + ((kc ^ (row & 7)) << 3); }

template <int ACT, int DBG = 0>
__global__ __launch_bounds__(768, 3) void gemm_lc_kernel(GemmArgs g, int tilesN, int tiles) {
  __shared__ __attribute__((aligned(16))) f16_t lds[2 * kLcStage + 2 * 256];  // + bias[2][256] fp32 (as halfs)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  if (wgid >= tiles) return;
  const int my_tiles = (tiles - wgid + nwg - 1) / nwg;
  const int nk = g.K / LBK;
  const int G = my_tiles * nk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = g.M, N = g.N;
  float* bias_lds = reinterpret_cast<float*>(lds + 2 * kLcStage);

  if (wave >= 8) {  // ---------------- loaders
    const int li = wave - 8;
    const int prow = lane >> 3, pc = (lane & 7) ^ prow;  // row within a piece, source 16-B chunk
    auto stage = [&](int gs) {
      if constexpr (DBG == 2) return;
      const int i = gs / nk, kt = gs - i * nk;
      const int t = wgid + i * nwg, tm = t / tilesN, tn = t - tm * tilesN;
      const int m0 = tm * RBM, n0 = tn * RBN, k0 = kt * LBK;
      f16_t* base = lds + (gs & 1) * kLcStage;
#pragma unroll
      for (int j = 0; j < kLcPerLoader; ++j) {
        const int p = li + kLcLoaders * j;
        const f16_t* src;
        if (p < RBM / 8) {
          const int gm = min(m0 + 8 * p + prow, M - 1);
          src = g.A + (size_t)gm * g.lda + k0 + pc * 8;
        } else {
          const int gn = min(n0 + 8 * (p - RBM / 8) + prow, N - 1);
          src = g.W + (size_t)gn * g.ldw + k0 + pc * 8;
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + p * 512), 16, 0, 0);
      }
      if (kt == 0 && li == kLcLoaders - 1)  // 256 bias floats (192 used; clamped source, N % 4 == 0)
        __builtin_amdgcn_global_load_lds((const void*)(g.bias + min(n0 + lane * 4, N - 4)),
                                         (lds_void*)(bias_lds + (i & 1) * 256), 16, 0, 0);
    };
    stage(0);
    __syncthreads();
#pragma unroll 1
    for (int gs = 0; gs < G; ++gs) {
      if (gs + 1 < G) stage(gs + 1);
      __syncthreads();  // vmcnt(0) (own DMAs landed) + barrier
    }
    return;
  }

  // ---------------- MFMA waves
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const uint32_t out_elems = (uint32_t)(M - 1) * g.ldc + N;
  const rsrc_t rc16 = make_rsrc(g.c16, out_elems * 2u);
  f32x4 acc[RNI][RMI];
#pragma unroll
  for (int i = 0; i < RNI; ++i)
#pragma unroll
    for (int j = 0; j < RMI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // stage 0 landed
  int gs = 0;
#pragma unroll 1
  for (int i = 0; i < my_tiles; ++i) {
    const int t = wgid + i * nwg, tm = t / tilesN, tn = t - tm * tilesN;
    const int m0 = tm * RBM, n0 = tn * RBN;
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt, ++gs) {
      const f16_t* xs = lds + (gs & 1) * kLcStage;
      const f16_t* ws = xs + RBM * LBK;
#pragma unroll
      for (int ks = 0; ks < (DBG == 1 ? 0 : 2); ++ks) {
        f16x8 wf[RNI], xf[RMI];
#pragma unroll
        for (int ii = 0; ii < RNI; ++ii)
          wf[ii] = as_f16x8(*reinterpret_cast<const uint4*>(ws + lswz(wn * RTN + ii * 16 + fr, ks * 4 + fg)));
#pragma unroll
        for (int j = 0; j < RMI; ++j)
          xf[j] = as_f16x8(*reinterpret_cast<const uint4*>(xs + lswz(wm * RTM + j * 16 + fr, ks * 4 + fg)));
#pragma unroll
        for (int ii = 0; ii < RNI; ++ii)
#pragma unroll
          for (int j = 0; j < RMI; ++j) acc[ii][j] = mfma16x16x32(wf[ii], xf[j], acc[ii][j]);
      }
      __syncthreads();  // stage gs + 1 landed; stage gs's slot may be refilled
    }
    // epilogue (after the barrier: the loaders already fill the next tile's stages)
    const float* bias_l = bias_lds + (i & 1) * 256;
#pragma unroll
    for (int j = 0; j < RMI; ++j) {
      const uint32_t m = m0 + wm * RTM + j * 16 + fr;
#pragma unroll
      for (int ii = 0; ii < RNI; ii += 2) {
        uint2 pk[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float4 bi = *reinterpret_cast<const float4*>(bias_l + wn * RTN + (ii + h2) * 16 + fg * 4);
          float v[4] = {acc[ii + h2][j][0] + bi.x, acc[ii + h2][j][1] + bi.y, acc[ii + h2][j][2] + bi.z,
                        acc[ii + h2][j][3] + bi.w};
          if (ACT != ACT_NONE) act4<ACT>(v);
          pk[h2] = make_uint2(pack2h(v[0], v[1]), pack2h(v[2], v[3]));
        }
        const bool odd = fg & 1;
        const int n8 = n0 + wn * RTN + (odd ? (ii + 1) * 16 + (fg - 1) * 4 : ii * 16 + fg * 4);
        buf_store_u4(rc16, n8 < N ? (m * (uint32_t)g.ldc + n8) * 2u : kOOB, pair_rows16(pk[0], pk[1]));
      }
    }
#pragma unroll
    for (int ii = 0; ii < RNI; ++ii)
#pragma unroll
      for (int j = 0; j < RMI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

}  // namespace

bool gemm_ring_ok(const GemmArgs& a) {
  const size_t lim = (size_t)1 << 31;
  return a.epi == 0 && !a.ascale && !a.res32 && !a.res16 && !a.c32 && a.c16 && a.bias && (a.K % 64) == 0 &&
         a.K >= 128 && (a.N % 8) == 0 && a.N >= 8 && a.M > 0 && (size_t)(a.M + RBM) * a.ldc * 2 < lim;
}

hipError_t launch_gemm_lc(const GemmArgs& a, hipStream_t s, int dbg) {
  if (!gemm_ring_ok(a)) return hipErrorInvalidValue;
  const int tilesM = (a.M + RBM - 1) / RBM, tilesN = (a.N + RBN - 1) / RBN;
  const int tiles = tilesM * tilesN;
  const int grid = tiles < 256 ? tiles : 256;
  if (dbg == 1 || dbg == 2) {
    if (dbg == 1) hipLaunchKernelGGL((gemm_lc_kernel<ACT_NONE, 1>), dim3(grid), dim3(768), 0, s, a, tilesN, tiles);
    else hipLaunchKernelGGL((gemm_lc_kernel<ACT_NONE, 2>), dim3(grid), dim3(768), 0, s, a, tilesN, tiles);
    return hipGetLastError();
  }
#define MMF_LC_CASE(ACT)                                                                                   \
  case ACT:                                                                                                \
    hipLaunchKernelGGL((gemm_lc_kernel<ACT>), dim3(grid), dim3(768), 0, s, a, tilesN, tiles);                \
    break;
  switch (a.act) {
    MMF_LC_CASE(ACT_NONE)
    MMF_LC_CASE(ACT_GELU)
    MMF_LC_CASE(ACT_QUICK_GELU)
    MMF_LC_CASE(ACT_SILU)
    MMF_LC_CASE(ACT_RELU)
    default:
      return hipErrorInvalidValue;
  }
#undef MMF_LC_CASE
  return hipGetLastError();
}

hipError_t launch_gemm_ring(const GemmArgs& a, hipStream_t s, int dbg) {
  if (!gemm_ring_ok(a)) return hipErrorInvalidValue;
  const int tilesM = (a.M + RBM - 1) / RBM, tilesN = (a.N + RBN - 1) / RBN;
  const int tiles = tilesM * tilesN;
  const int grid = tiles < 256 ? tiles : 256;
  constexpr int NS = 5;
  if (dbg == 1) {
    hipLaunchKernelGGL((gemm_ring_kernel<ACT_NONE, NS, 1>), dim3(grid), dim3(512), 0, s, a, tilesN, tiles);
    return hipGetLastError();
  }
  if (dbg == 2) {
    hipLaunchKernelGGL((gemm_ring_kernel<ACT_NONE, NS, 2>), dim3(grid), dim3(512), 0, s, a, tilesN, tiles);
    return hipGetLastError();
  }
#define MMF_RING_CASE(ACT)                                                                                      \
  case ACT:                                                                                                     \
    hipLaunchKernelGGL((gemm_ring_kernel<ACT, NS>), dim3(grid), dim3(512), 0, s, a, tilesN, tiles);             \
    break;
  switch (a.act) {
    MMF_RING_CASE(ACT_NONE)
    MMF_RING_CASE(ACT_GELU)
    MMF_RING_CASE(ACT_QUICK_GELU)
    MMF_RING_CASE(ACT_SILU)
    MMF_RING_CASE(ACT_RELU)
    default:
      return hipErrorInvalidValue;
  }
#undef MMF_RING_CASE
  return hipGetLastError();
}
