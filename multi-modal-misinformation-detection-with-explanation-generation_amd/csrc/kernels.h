// Host-side launchers of the gfx950 kernels (implemented in *.hip).  All enqueue on `stream`
// and return hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t f16_t;

struct GemmArgs {
  const f16_t* A;  int lda;     // activations [M][K] fp16
  const f16_t* W;  int ldw;     // weights [N][K] fp16 (PyTorch Linear layout)
  const float* bias;             // [N] or null
  const float* res32;            // fp32 residual [M][N] (ldr) or null
  const f16_t* res16;           // fp16 residual [M][N] (ldr) or null
  int ldr;
  float* c32;                    // fp32 out [M][N] (ldc) or null
  f16_t* c16;                   // fp16 out [M][N] (ldc) or null
  int ldc;
  const float* ascale;           // per-(batch, k) fp32 scale of A (SE excitation) or null
  int rows_per_batch;            // rows of A per batch item when ascale != null
  int M, N, K, act;
  int force_cfg;                 // 0 = automatic tile choice, c + 1 = instantiation c (A/B option)
  int no_splitk;                 // 1 = never split K on the skinny-M path (A/B option)
  int group_m;                   // persistent-tile order: 0 row-major, g > 0 grouped by g row panels
  float* ws;                     // split-K partials workspace (skinny-M GEMMs) or null
  size_t ws_elems;               // its capacity in floats
  // Lazy LayerNorm (option lazy_ln; gemm.hip).  A row's LN statistics travel as P partials
  // (mean_p, M2_p) over consecutive column blocks of tn columns ([rows][P] float2, buffers padded
  // to whole 256-row blocks), combined with Chan's formula by the reader.
  int epi;                       // 0 plain; 1 A = raw rows s: out = r (acc - mean u) + bias (LN folded
                                 // into W, bias padded by 256); 2 out = acc + bias + res16 (in
                                 // place allowed), partials of out written
  const float2* ln_in;           // epi 1: partials of A's rows
  int ln_in_P, ln_in_tn;         //   their count per row and column-block width
  const float* ln_u;             // epi 1: [N] sum_k W[n][k] (padded to N + 256)
  float2* ln_out;                // epi 2: partials of the output rows, [rows][ceil(N / tn_out)]
  float ln_eps;
  // epi 3 (RoBERTa, L = 128, option qkv_attn): W / bias are the fused QKV with rows interleaved per
  // head ([q_h; k_h; v_h] = 192 rows for head h), so a 256 x 192 tile holds q, k and v of one head
  // for two whole sequences; the epilogue runs their attention and writes ctx [M][ldc] (c16, head h
  // at columns 64 h) instead of qkv.  amask: key-padding mask int32 [M / 128][128] (1 keep) or null
  const int32_t* amask;
  // epi 4 (RoBERTa precise mode, FFN-1): out = act(acc + bias) written as the next GEMM's split
  // operand row: c16[m * ldc + n] = hi, and with split_lo also [+ N] = lo = fp16(out - hi), [+ 2N] = hi
  // (ldc >= 3N), so the fp32 hidden and its split3 pass are never formed
  int split_lo;
};
// whether launch_gemm accepts a (epi != 0) epilogue for these arguments (the host falls back to
// the plain path otherwise)
bool gemm_epi_ok(const GemmArgs& a);
// epi 2: the column-block width (= P partials per row of ceil(N / tn)) launch_gemm will use
int gemm_ln_tn(const GemmArgs& a);
// split-K factor the skinny-M (M <= 512) GEMM path uses for this (K) -- independent of M, so
// results stay batch-invariant; 1 = no split.  Workspace need: splitk_factor * M * N floats.
int gemm_splitk_factor(const GemmArgs& a);
hipError_t launch_gemm(const GemmArgs& a, hipStream_t s);
int gemm_config(const GemmArgs& a);          // which instantiation launch_gemm picks
constexpr int kGemmConfigs = 17;  // numbering of the tile instantiations (0 .. 16; gemm.hip config_exists)
const char* gemm_config_name(int c);
// streaming 1x1-convolution kernel (pointwise.hip), picked by launch_gemm when applicable
bool pw_applicable(const GemmArgs& a);
hipError_t launch_pw(const GemmArgs& a, hipStream_t s);

// LayerNorm over rows of width C (multiple of 256): y = LN(x [+ add]) * g + b.
// x/add fp32 with row strides; writes fp32 y32 and/or fp16 y16.
hipError_t launch_layernorm(const float* x, int ldx, const float* add, int ldadd, const float* g, const float* b,
                            float eps, float* y32, int ldy32, f16_t* y16, int ldy16, int rows, int C,
                            hipStream_t s);

// Residual add + LayerNorm: s = x (fp32, row stride ldx) + y (fp16 GEMM output, ldy); optionally
// s32 = s, o32 = LN(s) (both with stride ldx; may alias x); o16 = LN(s) fp16 (ldo).  C in {512, 768}.
hipError_t launch_add_ln(const float* x, int ldx, const f16_t* y, int ldy, const float* g, const float* b, float eps,
                         float* s32, float* o32, f16_t* o16, int ldo, int rows, int C, hipStream_t s);
// the same with an fp16 residual stream (pre-LN CLIP, option clip_res16): s16 = s (may alias x)
hipError_t launch_add_ln(const f16_t* x, int ldx, const f16_t* y, int ldy, const float* g, const float* b, float eps,
                         f16_t* s16, f16_t* o16, int ldo, int rows, int C, hipStream_t s);

// Fused multi-head attention, head_dim 64, L <= 128: qkv fp16 [B*L][ldqkv] with q at col h*64,
// k at D + h*64, v at 2D + h*64 (D = H*64); mask int32 [B][L] (1 keep) or null; out fp16 [B*L][ldo].
// one query per sequence over the sequence's keys (the compact last encoder layer): q [B][ldq] fp32, out
// row b at out + b * ldo; qpos (nullable) = the query's position per sequence for a causal mask
hipError_t launch_attention_q1(const float* q, int ldq, const f16_t* qkv, int ld, int koff, int voff,
                               const int32_t* mask, const int32_t* qpos, f16_t* out, int ldo, int B, int L, int H,
                               hipStream_t s);
hipError_t launch_attention(const f16_t* qkv, int ldqkv, const int32_t* mask, f16_t* out, int ldo, int B,
                            int L, int H, int causal, hipStream_t s);

// RoBERTa embeddings + LayerNorm -> the split stream xb (hi) + xlo (lo, nullable) [B*L][H] fp16, or,
// with x32 non-null, the fp32 stream only (precise mode)
hipError_t launch_roberta_embed(const int32_t* ids, const float* word, const float* pos, const float* type0,
                                const float* g, const float* b, float eps, uint16_t* xlo, f16_t* xb, int B, int L,
                                int H, int pad_id, hipStream_t s, float* x32 = nullptr, int* ovf = nullptr);
// ovf (nullable, [B] int32): the overflow sentinel of the fp16 / split stream -- a row whose
// LayerNorm statistics are non-finite sets ovf[sequence] = 1 (embeddings and add+LN); the text heads
// then return NaN for that sequence (capi.cpp run_text)
// RoBERTa precise mode (precise.hip, option text_hilo = 2): fp32 rows -> [hi | lo | hi] fp16 rows of 3C
// (the K-concatenated GEMM operand), and fp32 attention over an fp32 qkv (q at h*64, k at koff + h*64,
// v at voff + h*64; key-padding mask int32 [B][L] or null) -> fp32 out [B*L][ldo]
// with_lo = 0: only the hi third is written (a consumer on fp16 operands)
hipError_t launch_split3(const float* x, int ldx, f16_t* out, int rows, int C, hipStream_t s, int with_lo = 1);
// out3 (nullable): ctx written as the next GEMM's operand rows [hi | lo | hi] (ld 3 * H * 64; with_lo = 0: hi
// alone) instead of fp32 rows to out
hipError_t launch_attention32(const float* qkv, int ld, int koff, int voff, const int32_t* mask, float* out, int ldo,
                              int B, int L, int H, hipStream_t s, f16_t* out3 = nullptr, int with_lo = 1);
// precise mode: x = LN(x + add) in place [rows][768] fp32, and s3 = [hi | lo | hi] rows of it (with_lo = 0: hi only)
hipError_t launch_layernorm_split3(float* x, const float* add, const float* g, const float* b, float eps, f16_t* s3,
                                   int with_lo, int rows, int C, hipStream_t s);
// RoBERTa post-LN residual stream split as hi = fp16(x) (also the GEMM operand), lo = fp16(x - hi)
hipError_t launch_add_ln_hilo(f16_t* hi, uint16_t* lo, int ld, const f16_t* y, int ldy, const float* g,
                              const float* b, float eps, int rows, int C, hipStream_t s, int* ovf = nullptr, int L = 0);
hipError_t launch_hilo_rows(const f16_t* hi, const uint16_t* lo, int row_stride, float* out, int B, int C,
                            hipStream_t s);
// CLIP text embeddings (tok + pos) -> x fp32 (or x16 fp16: exactly one non-null), then LN1 of layer 0
// -> xb fp16
hipError_t launch_clip_text_embed(const int32_t* ids, const float* tok, const float* pos, const float* g,
                                  const float* b, float eps, float* x, f16_t* x16, f16_t* xb, float2* st, int B, int L,
                                  int H, hipStream_t s);
// (lazy LN, st != null: st[row] = (mean, M2) of the stored stream instead of xb)
// CLIP patch im2col with normalisation: img uint8 [B,224,224,3] -> A fp16 [B*49][3072]
hipError_t launch_clip_im2col(const uint8_t* img, f16_t* A, int B, hipStream_t s);
// CLIP vision: x = preLN(cat(cls, patches) + pos) -> x fp32 [B*50][768] (or x16 fp16: exactly one
// non-null), xb = LN1(x) fp16
hipError_t launch_clip_vision_assemble(const float* patches, const float* cls, const float* pos,
                                       const float* pre_g, const float* pre_b, const float* ln1_g,
                                       const float* ln1_b, float eps, float* x, f16_t* x16, f16_t* xb, float2* st,
                                       int B, hipStream_t s);

// EOS index per row (first == eos_id, or argmax when eos_id == 2)
hipError_t launch_eos_index(const int32_t* ids, int32_t* out, int B, int L, int eos_id, hipStream_t s);
// gather rows: out fp16 [B][C] = LN(x[row_index(b)]) where row_index = b*L + (idx ? idx[b] : 0)
hipError_t launch_gather_ln(const float* x, const int32_t* idx, int L, const float* g, const float* b, float eps,
                            f16_t* out, float* out32, int B, int C, hipStream_t s);
// compact copies of rows b*L + (idx ? idx[b] : 0) of a fp16 (a16, nullable: then o16 is not written) and
// an fp32 (a32, or fp16 a32h: exactly one non-null) [.,C] buffer; o32 is fp32 either way
hipError_t launch_gather_rows2(const f16_t* a16, const float* a32, const f16_t* a32h, const int32_t* idx, int L,
                               int C, f16_t* o16, float* o32, int B, hipStream_t s);
// L2-normalise rows of fp32 [B][C] in place (C multiple of 64)
hipError_t launch_l2norm(float* x, int B, int C, hipStream_t s);
// two 768->256->2 heads (fp32) from CLS rows x[b*L*768]; writes logits and softmax[:,1] scores
hipError_t launch_text_heads(const float* x, int row_stride, const float* w1a, const float* b1a,
                             const float* w2a, const float* b2a, const float* w1m, const float* b1m,
                             const float* w2m, const float* b2m, float* ai_logits, float* mi_logits,
                             float* scores, int score_stride, int B, hipStream_t s, const int* ovf = nullptr);
// fusion MLP 5->64->32->2 (+ verdict, confidence, explanation rule)
hipError_t launch_fusion(const float* x5, const float* w0, const float* b0, const float* w3, const float* b3,
                         const float* w5, const float* b5, float* probs, int32_t* verdict, float* conf,
                         int32_t* rule, int B, hipStream_t s);
// cosine of unit rows: out[b*ostride] = dot(a[b], c[b])
hipError_t launch_rowdot(const float* a, const float* c, float* out, int ostride, int B, int C, hipStream_t s);
// vault: S[B][N] = Q[B][D] . V[N][D]^T (fp32)
hipError_t launch_vault_sims(const float* q, const float* v, float* S, int B, int N, int D, hipStream_t s, int ref = 0);
hipError_t launch_vault_topk(const float* S, int B, int N, int k, float thresh, float* sims, int32_t* idx,
                             float* disc, int disc_stride, const float* text_emb, const float* title_emb, int D,
                             float* text_sim, hipStream_t s, int ref = 0);

// EfficientNet-B0 pieces (NHWC fp16 activations)
hipError_t launch_effnet_stem(const uint8_t* img, const float* w, const float* bias, f16_t* out, int B,
                              hipStream_t s);
hipError_t launch_effnet_stem_f32(const float* x_nchw, const float* w, const float* bias, f16_t* out, int B,
                                  hipStream_t s);
// stem fused into the stage-1 depthwise conv (3x3 s1, 32 channels at 112^2) + its SE pool partials;
// exactly one of img (uint8 HWC) / xf32 (normalised fp32 NCHW) is non-null
hipError_t launch_effnet_stem_dw(const uint8_t* img, const float* xf32, const float* ws, const float* bs,
                                 const float* wd, const float* bd, f16_t* out, float* pool_part, int B,
                                 int* nchunks_out, hipStream_t s);
// flags: bit 0 = compile-time tile geometries where one exists (runtime-geometry kernels otherwise),
// bit 3 = 32-channel groups for C in {480, 672, 1152} (option dw_cw32)
hipError_t launch_dwconv(const f16_t* in, const float* w, const float* bias, f16_t* out, float* pool_part,
                         int B, int H, int W, int C, int k, int stride, int* nchunks_out, hipStream_t s, int ct = 1);
hipError_t launch_se(const float* pool_part, int nchunks, float inv_hw, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* scale, int B, int C, int Csq, hipStream_t s,
                     bool precise = false);  // precise: the fc1 SiLU in silu_precise form (fp32 tower)
hipError_t launch_gap_classifier(const f16_t* x, int HW, int C, const float* w, const float* b, float* logits,
                                 float* score, int score_stride, int B, hipStream_t s);
hipError_t launch_fill_strided(float* p, int stride, int B, float v, hipStream_t s);
// fused MBConv front: expand 1x1 (we fp16 [C][cin], be fp32, BN folded) + SiLU computed per input
// tile into LDS, then the depthwise conv of launch_dwconv (same outputs, same pool partials)
bool expand_dw_applicable(int cin, int cexp, int k);
hipError_t launch_expand_dw(const f16_t* x, int cin, const f16_t* we, const float* be, const float* w,
                            const float* bias, f16_t* out, float* pool_part, int B, int H, int W, int C, int k,
                            int stride, int* nchunks_out, hipStream_t s, int ct = 1);
// number of pool-partial chunks launch_dwconv uses for an output of Ho x Wo with C channels
int dwconv_nchunks(int H, int W, int C, int stride);
// JPEG reconstruction (jpeg.hip): islow IDCT per block, then fancy upsampling + YCbCr -> RGBX per pixel
hipError_t launch_jpeg_reconstruct(const uint8_t* packed, const uint32_t* block_off, const int64_t* pk_off,
                                   const uint16_t* qt, const int64_t* coef_blocks, const int32_t* infos,
                                   const int64_t* out_offsets, int B, int max_blocks, int max_pixels, uint8_t* samples,
                                   uint8_t* out, hipStream_t s);

// Pillow-exact resampling of decoded images to the towers' 224 x 224 windows (resize.hip)
constexpr int kResizeKMax = 96;  // taps per output coordinate (bicubic support 2 x scale <= 47)
struct ResizeJob {
  long long src_off;  // byte offset of the source image (uint8 HWC RGB) in the source buffer
  int w, h;           // source size
  int ow, oh;         // Pillow resize output size (before the crop)
  int cx, cy;         // window offset in the resize output (centre crop; 0 for the squash)
  int filt;           // 0 bilinear, 1 bicubic
  int need_h, need_v; // Pillow runs the pass (size changes on that axis)
  int y0, y1;         // source rows the window's vertical taps read
  int ksh, ksv;       // taps per coordinate, horizontal / vertical
  long long tmp_off;  // byte offset of this job's [y1 - y0][224][3] horizontal-pass rows
  int coef_off;       // int32 offset of [224][ksh] then [224][ksv] coefficients
  int ps;             // source bytes per pixel: 3 (RGB) or 4 (RGBX, Pillow's in-memory layout)
};
hipError_t launch_resize_pil(const uint8_t* src, const ResizeJob* jobs, int njobs, int max_rows, int32_t* coef,
                             int32_t* bounds, uint8_t* tmp, uint8_t* const* outs, hipStream_t s);

// fp32 EfficientNet tower (option effnet_fp32, effnet_f32.hip): NHWC fp32 activations
hipError_t launch_effnet_stem32(const uint8_t* img, const float* x_nchw, const float* w, const float* bias,
                                float* out, int B, hipStream_t s);
// C[M][N] = act((A .* ascale[m / rows_per_image]) W^T + bias) (+ res); W fp32 [N][K]; N, K % 4 == 0
hipError_t launch_pw32(const float* A, const float* W, const float* bias, const float* ascale, int rows_per_image,
                       const float* res, float* C, int M, int N, int K, int act, hipStream_t s, int mfma = 1);
// w tap-major [k*k][C]
hipError_t launch_dw32(const float* in, const float* w, const float* bias, float* out, int B, int H, int W, int C,
                       int k, int stride, hipStream_t s);
// part[b][j][c] = sum over pixel chunk j of nchunks (the SE's pool partials)
hipError_t launch_sum32(const float* x, int B, int HW, int C, int nchunks, float* part, hipStream_t s);
hipError_t launch_gap32(const float* x, int HW, int C, const float* w, const float* b, float* logits, float* score,
                        int score_stride, int B, hipStream_t s);
