// Device-side helpers shared by the gfx950 kernels of libmmf_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t f16_t;  // raw IEEE binary16 (fp16) storage: every 16-bit GEMM / MFMA operand
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MMF_DEV __device__ __forceinline__
#define MMF_DEV_HOST_INLINE __host__ __device__ inline

// Operand precision: fp16 (11 significant bits) rather than bf16 (8).  The MFMA rate is the same
// (v_mfma_f32_16x16x32_f16 / _bf16 take the same cycles on gfx950) and every conversion is one
// instruction either way, but the operand rounding moves the five scores ~9x less (DESIGN.md §4:
// max |d score| 0.93e-3 -> 0.10e-3 in the CPU emulation), which is what holds the 1e-3 parity bar
// at full batch size.  Range: |x| < 65504, far above the activations of these encoders.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
MMF_DEV float h2f(f16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
MMF_DEV f16_t f2h(float f) { return __builtin_bit_cast(f16_t, (_Float16)f); }
// one v_cvt_pk_f16_f32 (RNE) for both halves
MMF_DEV uint32_t pack2h(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
}
// halves of a packed pair (v_cvt_f32_f16, the high one with an SDWA word select)
MMF_DEV float lo_h(uint32_t w) { return (float)__builtin_bit_cast(f16x2_t, w).x; }
MMF_DEV float hi_h(uint32_t w) { return (float)__builtin_bit_cast(f16x2_t, w).y; }

MMF_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MMF_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// activations (fp32).  Epilogue cost matters: a GEMM epilogue runs serially after the MFMA loop,
// so IEEE erff / division (30-40 VALU ops) are replaced by short forms built on v_rcp_f32 /
// v_exp_f32 (~1 ulp each).
MMF_DEV float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// GELU-erf as relu(x) - |h|, h = 0.5 x erfc(|x| / sqrt 2), erfc by Abramowitz & Stegun 7.1.26
// (|err| <= 1.5e-7): 11 FMA-class ops + v_rcp + v_exp per element, about 2/3 of a 7/5 rational
// erf, and max |GELU error| 3.3e-7 over [-12, 12] (float32 emulation vs float64 erf).
MMF_DEV float gelu_erf(float x) {
  const float az = fabsf(x) * 0.70710678118654752f;
  const float t = fast_rcp(fmaf(0.3275911f, az, 1.0f));
  float p = fmaf(0.5307027145f, t, -0.7265760135f);  // a5/2, a4/2
  p = fmaf(p, t, 0.7107068705f);                      // a3/2
  p = fmaf(p, t, -0.142248368f);                      // a2/2
  p = fmaf(p, t, 0.127414796f);                       // a1/2
  p *= t;
  const float e = __builtin_amdgcn_exp2f(az * (az * -1.4426950408889634f));
  return fmaf(-fabsf(x), p * e, fmaxf(x, 0.0f));
}
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_QUICK_GELU = 2, ACT_SILU = 3, ACT_RELU = 4 };
// SiLU as torch's CPU kernel evaluates it (x / (1 + exp(-x)), IEEE division, ~1-ulp exp): the fp32
// EfficientNet tower (effnet_f32.hip), where approximate transcendentals would be amplified
MMF_DEV float silu_precise(float x) { return x / (1.0f + expf(-x)); }
MMF_DEV float act_precise(float x, int act) { return act == ACT_SILU ? silu_precise(x) : x; }

MMF_DEV float act_apply(float x, int act) {
  switch (act) {
    case ACT_GELU: return gelu_erf(x);
    case ACT_QUICK_GELU: return x * fast_rcp(1.0f + __expf(-1.702f * x));          // x*sigmoid(1.702x)
    case ACT_SILU: return x * fast_rcp(1.0f + __expf(-x));
    case ACT_RELU: return fmaxf(x, 0.0f);
    default: return x;
  }
}

// Two elements at once: the FMA-class steps become packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32, 2 results per lane per issue), only the transcendentals stay per element.  Same
// operations in the same order as the scalar forms above, so results are bit-identical.
MMF_DEV f32x2_t gelu_erf2(f32x2_t x) {
  const f32x2_t ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2_t az = ax * 0.70710678118654752f;
  const f32x2_t d = __builtin_elementwise_fma(az, (f32x2_t)0.3275911f, (f32x2_t)1.0f);
  const f32x2_t t = {fast_rcp(d.x), fast_rcp(d.y)};
  f32x2_t p = __builtin_elementwise_fma((f32x2_t)0.5307027145f, t, (f32x2_t)-0.7265760135f);
  p = __builtin_elementwise_fma(p, t, (f32x2_t)0.7107068705f);
  p = __builtin_elementwise_fma(p, t, (f32x2_t)-0.142248368f);
  p = __builtin_elementwise_fma(p, t, (f32x2_t)0.127414796f);
  p = p * t;
  const f32x2_t a = az * (az * -1.4426950408889634f);
  const f32x2_t pe = p * (f32x2_t){__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  return (f32x2_t){fmaf(-ax.x, pe.x, fmaxf(x.x, 0.0f)), fmaf(-ax.y, pe.y, fmaxf(x.y, 0.0f))};
}
// x * sigmoid(k x) for a pair (SiLU k = 1, quick-GELU k = 1.702)
// PKX: exp(a) evaluated exactly as hipcc lowers __expf -- v_exp_f32(a * 0x3fb8aa3b) -- with the
// log2(e) scale as one packed multiply for the pair instead of two scalar ones (bit-identical; the
// EfficientNet fronts / depthwise convs are VALU-bound on their SiLU: tower -1 %.  The GEMM epilogues
// keep the scalar form: the packed one measured +0.6 % on the step)
template <bool PKX = false>
MMF_DEV f32x2_t xsigmoid2(f32x2_t x, float k) {
  const f32x2_t a = x * -k;
  f32x2_t e;
  if constexpr (PKX) {
    const f32x2_t t = a * 1.44269502f;
    e = (f32x2_t){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  } else {
    e = (f32x2_t){__expf(a.x), __expf(a.y)};
  }
  const f32x2_t d = e + 1.0f;
  return x * (f32x2_t){fast_rcp(d.x), fast_rcp(d.y)};
}
// activation of 4 consecutive accumulator values (compile-time ACT), packed where it pays
template <int ACT, bool PKX = false>
MMF_DEV void act4(float* v) {
#pragma unroll
  for (int h = 0; h < 4; h += 2) {
    f32x2_t x = {v[h], v[h + 1]};
    if constexpr (ACT == ACT_GELU) x = gelu_erf2(x);
    else if constexpr (ACT == ACT_QUICK_GELU) x = xsigmoid2(x, 1.702f);
    else if constexpr (ACT == ACT_SILU) x = xsigmoid2<PKX>(x, 1.0f);
    else if constexpr (ACT == ACT_RELU) x = (f32x2_t){fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)};
    v[h] = x.x;
    v[h + 1] = x.y;
  }
}

MMF_DEV f32x4 mfma16x16x32(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Rows of 16 lanes pair up (lanes l, l ^ 16): a = this lane's 4-column group i, b = group i + 1
// (packed fp16x4 each).  Even rows end with [own a | partner's a], odd rows with
// [partner's b | own b]: 16 contiguous bytes per lane.  v_permlane16_swap (VALU, no LDS trip).
MMF_DEV uint4 pair_rows16(uint2 a, uint2 b) {
  const auto x = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return make_uint4(x[0], y[0], x[1], y[1]);
}

MMF_DEV f16x8 as_f16x8(const uint4& v) { return __builtin_bit_cast(f16x8, v); }

// Raw buffer access (CDNA SRSRC): 32-bit byte offsets with hardware bounds checking -- loads at
// offsets >= `bytes` return 0 and such stores are dropped, so null operands (bytes = 0) and
// ragged tile edges need no branches.  Descriptors must be built from wave-uniform values.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0x80000000u;  // an offset past every buffer the launchers allow
// Cache policy of the raw-buffer epilogue stores: plain (0: the written lines stay in the XCD's L2
// and the Infinity Cache for the next kernel, which reads them).  Write-through sc1 (16) made the
// isolated encoder GEMMs 2-13 % faster (tools/ab_lib.py: nothing re-reads their outputs) but the
// whole analyze step 2.7 % slower (tools/lib_step_ab.sh: 14.46 -> 14.08 ms with plain stores, three
// interleaved rounds; sc0 ties with plain).
#ifndef MMF_STORE_AUX
#define MMF_STORE_AUX 0
#endif
MMF_DEV rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? (int)bytes : 0, 0x00020000);
}
MMF_DEV float4 buf_load_f4(rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
MMF_DEV uint2 buf_load_u2(rsrc_t r, uint32_t off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v.x, v.y);
}
MMF_DEV void buf_store_f4(rsrc_t r, uint32_t off, float4 v) {
  const u32x4 w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, MMF_STORE_AUX);
}
MMF_DEV void buf_store_u4(rsrc_t r, uint32_t off, uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, MMF_STORE_AUX);
}
MMF_DEV void buf_store_u2(rsrc_t r, uint32_t off, uint2 v) {
  const u32x2 w = {v.x, v.y};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, off, 0, MMF_STORE_AUX);
}
