/*
 * mmf_hip.h — C-ABI of libmmf_hip.so, the MI355X-native (gfx950) hot path of the reference's
 * MisinfoForensics.analyze() 5-signal forward.
 *
 * The reference has no FFI: its boundary is the Python API of misinfo_forensics.py.  Each entry
 * point below replaces one reference call site; the Python host side (mmf_amd/hip.py, ctypes)
 * keeps the reference's method names and return dicts on top of these.
 *
 * Conventions
 *   - Plain C types only; every function returns 0 on success or a negative errno-style code
 *     (MMF_EINVAL bad argument/shape/missing weight, MMF_ENOMEM allocation, MMF_EIO HIP error).
 *     Nothing throws across the ABI.  mmf_last_error() gives a thread-local message.
 *   - All tensor I/O of the forward calls are caller-owned DEVICE pointers (e.g. torch tensors'
 *     data_ptr()), enqueued asynchronously on the caller's hipStream_t `stream` (NULL = default
 *     stream).  No implicit device synchronisation.
 *   - Weights, workspaces and the Truth-Vault are owned by the handle.  A handle is bound to one
 *     device and is not thread-safe: one handle per (process, device).
 *   - Layouts: token ids / masks int32 row-major [B, L]; images uint8 [B, 224, 224, 3] (HWC, RGB);
 *     embeddings / logits / scores fp32 row-major.
 */
#ifndef MMF_HIP_H
#define MMF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMF_OK 0
#define MMF_EINVAL (-22)
#define MMF_ENOMEM (-12)
#define MMF_EIO (-5)
#define MMF_ERANGE (-34) /* an input outside a kernel's supported range (mmf_resize_pil: too many taps) */
#define MMF_EUNSUPPORTED (-95) /* a valid input of a kind this path does not handle (mmf_jpeg_*: CMYK, lossless, ...) */

#define MMF_DTYPE_F32 0
#define MMF_DTYPE_I64 1

typedef struct mmf_handle mmf_handle;

/* Create a handle on HIP device `device` (ordinal within HIP_VISIBLE_DEVICES). */
int mmf_create(int device, mmf_handle** out);
void mmf_destroy(mmf_handle* h);
/* Thread-local description of the last error (empty string if none). */
const char* mmf_last_error(void);
/* Library/ABI version string. */
const char* mmf_version(void);

/* Stage one host tensor under its state-dict name.  Names are the reference's state-dict keys:
 * detector keys as in MultiModalMisinfoDetector (misinfo_forensics.py:43-108 — "roberta.*",
 * "ai_head.*", "misinfo_head.*", "efficientnet.*", "fusion_layer.*") and CLIP keys as in HF
 * CLIPModel prefixed with "clip." (misinfo_forensics.py:210-212).  Replaces the reference's
 * load_state_dict (misinfo_forensics.py:175-186, 260-317); the data are copied. */
int mmf_load_tensor(mmf_handle* h, const char* name, int dtype, int ndim, const int64_t* shape,
                    const void* host_data);
/* Pack staged tensors into device layouts (fused QKV, BatchNorm folded into convs, fp16 GEMM
 * operands).  Components whose tensors are all present become available; `clip_eos_token_id`
 * selects the HF EOS-pooling rule (2 = argmax(ids), else first index of that id;
 * TF clip:561-582). */
int mmf_finalize(mmf_handle* h, int clip_eos_token_id);
/* Bit mask of ready components: 1 text(RoBERTa+heads) 2 effnet 4 clip-vision 8 clip-text
 * 16 fusion 32 vault. */
int mmf_ready(mmf_handle* h);

/* Allocate activation workspaces for up to `max_batch` rows with RoBERTa length `max_text_len`
 * (<= 512) and CLIP text length `max_clip_len` (<= 77).  Forward calls with larger shapes fail
 * with MMF_EINVAL; call before graph capture. */
int mmf_reserve(mmf_handle* h, int max_batch, int max_text_len, int max_clip_len);

/* Signals 1-2 — analyze_text (misinfo_forensics.py:319-352): RoBERTa + dual heads.
 * ids/mask int32 [B, L <= 512] device (the reference tokenizer truncates at 512, :327-333; L > 128
 * takes the long-sequence attention kernel).  Outputs fp32 [B, 2] logits each (may be NULL) and
 * scores fp32 [B, 2] = softmax(.)[:,1] of (ai, misinfo) (may be NULL). */
int mmf_text_forward(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L,
                     float* ai_logits, float* misinfo_logits, float* scores2, void* stream);

/* Signal 3 — analyze_image (misinfo_forensics.py:354-373, 249-253): ImageNet normalisation +
 * EfficientNet-B0.  img uint8 [B, 224, 224, 3] device.  logits fp32 [B, 2] (may be NULL),
 * deepfake_score fp32 [B] (may be NULL). */
int mmf_effnet_forward(mmf_handle* h, const uint8_t* img, int B, float* logits, float* deepfake_score,
                       void* stream);

/* Same as mmf_effnet_forward for an already-normalised fp32 NCHW tensor x [B, 3, 224, 224] (the
 * reference's detector.forward_image(image_tensor) signature, misinfo_forensics.py:102-104). */
int mmf_effnet_forward_f32(mmf_handle* h, const float* x, int B, float* logits, float* deepfake_score,
                           void* stream);

/* CLIP image embedding — get_image_features + L2 normalisation (misinfo_forensics.py:395-401,
 * 432-439).  img uint8 [B, 224, 224, 3] (CLIP-preprocessed geometry); emb fp32 [B, 512] unit. */
int mmf_clip_image(mmf_handle* h, const uint8_t* img, int B, float* emb_unit, void* stream);

/* CLIP text embedding — get_text_features + L2 normalisation (misinfo_forensics.py:395-401,
 * 473-481).  ids/mask int32 [B, L<=77]; emb fp32 [B, 512] unit. */
int mmf_clip_text(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* emb_unit,
                  void* stream);

/* analyze_consistency (misinfo_forensics.py:375-408) / CLIPSimilarityEngine.calculate_similarity
 * (clip_similarity_engine.py:63-119): both CLIP towers (text tower on a concurrent stream) and the
 * cosine of the unit embeddings.  img uint8 [B,224,224,3], ids/mask int32 [B, L<=77]; sim fp32 [B];
 * img_emb / txt_emb fp32 [B, 512] unit (may be NULL: handle workspaces are used). */
int mmf_clip_consistency(mmf_handle* h, const uint8_t* img, const int32_t* ids, const int32_t* mask, int B, int L,
                         float* img_emb, float* txt_emb, float* sim, void* stream);

/* Host-input geometry on the device (misinfo_forensics.py:249-253 and the
 * CLIPImageProcessor the reference calls at :386-401): B decoded uint8 images (HWC, pixel_bytes =
 * 3 for RGB or 4 for RGBX -- Pillow's in-memory layout --, any size up to a 47x downscale)
 * concatenated in device memory at byte offsets[i] with sizes wh[2i] = width, wh[2i+1] = height
 * (host arrays) -> out_effnet uint8 [B,224,224,3] =
 * Image.resize((224,224), BILINEAR) and out_clip uint8 [B,224,224,3] = shortest edge -> 224 BICUBIC
 * + centre crop, both bit-exact with Pillow's resampler (either output may be NULL).  Returns after
 * the work on `stream` has completed; MMF_ERANGE (nothing launched) when an image needs more taps
 * per output pixel than the kernels hold (mmf_resize_supported). */
int mmf_resize_pil(mmf_handle* h, const uint8_t* src, const int64_t* offsets, const int32_t* wh, int B,
                   int pixel_bytes, uint8_t* out_effnet, uint8_t* out_clip, void* stream);

/* Device JPEG decode (the reference's Image.open(path).convert("RGB"),
 * misinfo_forensics.py:255-258, decodes through Pillow's libjpeg-turbo).  Host: marker parsing and
 * Huffman entropy decoding (the serial part); device: dequantisation, islow IDCT, fancy chroma
 * upsampling and YCbCr -> RGB, pixels bit-exact with Pillow's decoder.  Supported: 8-bit baseline /
 * extended sequential Huffman JPEGs with one scan, and progressive Huffman JPEGs (any scan script;
 * quantisation tables fixed before the first scan), grayscale or YCbCr 4:4:4 / 4:2:2 / 4:2:0;
 * anything else returns MMF_EUNSUPPORTED (decode that file on the host).
 *
 * mmf_jpeg_header: host-only, no handle.  info[MMF_JPEG_INFO_LEN] = {width, height, ncomp, hmax, vmax,
 * bw0, bh0, bw1, bh1, bw2, bh2, blocks, 0...} (bw_c x bh_c = component c's MCU-padded block grid;
 * blocks = their sum = the int16[64] blocks mmf_jpeg_entropy writes).  Returns 0 if supported. */
#define MMF_JPEG_INFO_LEN 16
int mmf_jpeg_header(const uint8_t* data, int64_t nbytes, int32_t* info);
/* Host-only, thread-safe: quantised coefficients of every component as [bh_c][bw_c][64] int16
 * (natural order, components back to back) and the components' quantisation tables qt[c][64]
 * (natural order, uint16).  Replaces libjpeg's decode_mcu (jdhuff.c; progressive files: every scan
 * accumulated as jdphuff.c does). */
int mmf_jpeg_entropy(const uint8_t* data, int64_t nbytes, int16_t* coefs, uint16_t* qt);
/* Host-only, thread-safe: the same coefficients packed for the H2D copy (~2.8x fewer bytes than the
 * dense planes on photos): one record per block -- uint64 mask of its nonzero ZIGZAG positions, then
 * their int16 values in zigzag order, padded to 8 bytes -- in decode order after an all-zero record
 * at offset 0; block_off[b] = byte offset of block b's record (b in the dense layout's order, padding
 * blocks -> 0).  `out` must hold mmf_jpeg_packed_bound(blocks) bytes (MMF_ERANGE otherwise); *used =
 * bytes written.  This is the format mmf_jpeg_reconstruct reads. */
int64_t mmf_jpeg_packed_bound(int32_t blocks);
int mmf_jpeg_entropy_packed(const uint8_t* data, int64_t nbytes, uint8_t* out, int64_t cap, uint32_t* block_off,
                            uint16_t* qt, int64_t* used);
/* Host-only, thread-safe: mmf_jpeg_entropy_packed for a batch staged by several threads.  Decodes
 * into a per-thread scratch, reserves 8-aligned room by an atomic add on *cursor, sets *rec_off to it
 * and copies the records to dst + *rec_off -- or returns MMF_ERANGE (room still reserved) when they
 * do not fit in dst_cap bytes: grow dst and place that image again (mmf_jpeg_entropy_packed). */
int mmf_jpeg_stage_packed(const uint8_t* data, int64_t nbytes, uint8_t* dst, int64_t dst_cap, int64_t* cursor,
                          uint32_t* block_off, uint16_t* qt, int64_t* rec_off);
/* Host-only: mmf_jpeg_header over n files (null datas[k] -> MMF_EINVAL) on up to `nthreads` threads;
 * infos [n][MMF_JPEG_INFO_LEN], rcs[k] = file k's return code. */
int mmf_jpeg_header_batch(const uint8_t* const* datas, const int64_t* nbytes, int n, int32_t* infos, int32_t* rcs,
                          int nthreads);
/* Host-only: mmf_jpeg_stage_packed over n files on `nthreads` threads of its own (one C call per
 * chunk: no per-file interpreter work); file k's block offsets go to block_off + block_base[k], its
 * tables to qt + 192 k, its record offset to rec_off[k] and its status to rcs[k]. */
int mmf_jpeg_stage_packed_batch(const uint8_t* const* datas, const int64_t* nbytes, int n, uint8_t* dst,
                                int64_t dst_cap, int64_t* cursor, uint32_t* block_off, const int64_t* block_base,
                                uint16_t* qt, int64_t* rec_off, int nthreads, int32_t* rcs);
/* Device: B images' packed coefficients and tables -> uint8 RGBX pixels, bit-exact with Pillow's
 * decoder.  Every pointer is DEVICE memory: packed = the images' mmf_jpeg_entropy_packed records
 * (image i's at byte offset pk_off[i]), block_off uint32 = their block-offset tables concatenated
 * (image i's from index coef_blocks[i]), qt uint16 [B][3][64], infos int32 [B][MMF_JPEG_INFO_LEN]
 * (mmf_jpeg_header's), out_offsets int64 [B] (byte offset of image i's [h][w][4] RGBX pixels in
 * out_rgbx; X = 255), samples = scratch of 64 * sum(blocks) bytes (component sample planes, image i's
 * from 64 * coef_blocks[i]).  max_blocks / max_pixels = the largest blocks / width * height over the B
 * images (grid sizes).  Feeds mmf_resize_pil (pixel_bytes 4).  Asynchronous on `stream`. */
int mmf_jpeg_reconstruct(mmf_handle* h, const uint8_t* packed, const uint32_t* block_off, const int64_t* pk_off,
                         const uint16_t* qt, const int64_t* coef_blocks, const int32_t* infos, const int64_t* out_offsets,
                         int B, int max_blocks, int max_pixels, uint8_t* samples, uint8_t* out_rgbx, void* stream);

/* 1 if a width x height image fits mmf_resize_pil's tap budget in both geometries (bicubic CLIP:
 * shortest side <= ~5264 px; bilinear EfficientNet: either side <= ~10528 px), else 0.  Host-only,
 * no handle: callers route the few larger images to a host resampler. */
int mmf_resize_supported(int width, int height);

/* Truth-Vault (misinfo_forensics.py:214-246, 443-445): host fp32 [N, D=512] raw embeddings; rows
 * are L2-normalised once here instead of on every search call. */
int mmf_set_vault(mmf_handle* h, const float* host_vault, int N, int D);
/* The same with rows already L2-normalised by the caller: the Python host side normalises exactly
 * as the reference line does, in the vault's own dtype (numpy, misinfo_forensics.py:443-445 --
 * float16 vaults renormalise in float16; a zero row becomes NaN), and uploads the float32 result.
 * Replaces the previous vault and its title embeddings (their device memory is freed). */
int mmf_set_vault_normalized(mmf_handle* h, const float* host_vault_unit, int N, int D);
/* Pre-compute the CLIP text embeddings of the vault titles (used for text_similarity,
 * misinfo_forensics.py:467-484) from device ids/mask int32 [N, L<=77].  Synchronous. */
int mmf_set_vault_titles(mmf_handle* h, const int32_t* ids, const int32_t* mask, int N, int L, void* stream);

/* search_vault core (misinfo_forensics.py:443-464, 467-484): q fp32 [B, 512] unit image
 * embeddings; top-k (1 <= k <= N; k > 8 needs N <= 16384) similarities fp32 [B, k] and indices
 * int32 [B, k] in np.argsort(sims)[-k:][::-1] order (descending; NaN rows first, exact ties by
 * descending index);
 * discrepancy fp32 [B] = top1 > thresh ? top1 : 0; optional text_emb fp32 [B, 512] unit caption
 * embeddings -> text_sim fp32 [B] = cos(caption, title[top1]) where top1 > thresh, else 0. */
int mmf_vault_topk(mmf_handle* h, const float* q_unit, int B, int k, float thresh, float* sims, int32_t* idx,
                   float* discrepancy, const float* text_emb, float* text_sim, void* stream);

/* fusion_verdict (misinfo_forensics.py:575-615): scores5 fp32 [B, 5] -> probs fp32 [B, 2]
 * (real, fake); verdict int32 [B] (fake > 0.5); confidence fp32 [B]; explanation rule index
 * int32 [B] of _generate_fallback_explanation (misinfo_forensics.py:742-765; 0 vault, 1 deepfake,
 * 2 ai, 3 misinfo, 4 clip, 5 default).  Any output except probs may be NULL. */
int mmf_fusion(mmf_handle* h, const float* scores5, int B, float* probs2, int32_t* verdict, float* confidence,
               int32_t* rule, void* stream);

/* The whole text+image analyze() path for B pairs (misinfo_forensics.py:767-927) with the ViT
 * computed once per pair.  Inputs device: RoBERTa ids/mask [B, Lr], CLIP ids/mask [B, Lc],
 * img_effnet uint8 [B,224,224,3], img_clip uint8 [B,224,224,3] (may equal img_effnet).
 * Outputs device (all fp32 unless noted): scores5 [B,5] (ai, misinfo, deepfake, clip_similarity,
 * vault_discrepancy), text_sim [B], probs2 [B,2], verdict int32 [B], confidence [B], rule int32 [B],
 * top_sims [B,5], top_idx int32 [B,5].  Vault outputs are zero when no vault is set. */
int mmf_analyze_batch(mmf_handle* h, const int32_t* rob_ids, const int32_t* rob_mask, int Lr,
                      const int32_t* clip_ids, const int32_t* clip_mask, int Lc, const uint8_t* img_effnet,
                      const uint8_t* img_clip, int B, float* scores5, float* text_sim, float* probs2,
                      int32_t* verdict, float* confidence, int32_t* rule, float* top_sims, int32_t* top_idx,
                      void* stream);

/* Per-kernel timing for roofline accounting: while profiling is on, every kernel launch of the
 * forward calls is bracketed by two hipEvents on its stream.  mmf_profile_end synchronises and
 * aggregates per kernel kind (arrays of >= 16 entries): launch counts, summed device ms, summed
 * ALGORITHMIC flops and HBM bytes; returns the number of kinds.  Names via mmf_profile_kind_name. */
int mmf_profile_begin(mmf_handle* h);
int mmf_profile_end(mmf_handle* h, int max_kinds, int* counts, double* ms, double* flops, double* bytes);
const char* mmf_profile_kind_name(int kind);

/* Run-time options.  Defaults are read once per process from MMF_<NAME> environment variables
 * (e.g. MMF_GEMM_KLOOP), copied into every handle at mmf_create and changed with mmf_set_option
 * (h = NULL: the process defaults, used by the handle-less ops below and by handles created
 * afterwards).  The library's list is exactly the following (mmf_option_name enumerates it; the CPU
 * test tests/test_capi_cpu.py::test_header_options_match_library ties the two):
 *   "concurrent"     1: towers of mmf_analyze_batch on concurrent streams (0: one stream)
 *   "fuse_stem"      1: EfficientNet stem fused into the stage-1 depthwise conv
 *   "fuse_expand"    1: 1x1 expand fused into the depthwise conv (stages 2 - 4.3)
 *   "gemm_splitk"    1: split-K on the skinny-M (M <= 512) GEMM path
 *   "gemm_config"   -1: automatic GEMM tile choice; c >= 0 forces instantiation c (A/B tools)
 *   "gemm_group_m"   0: persistent GEMM tile order (g > 0: grouped by g row panels)
 *   "text_hilo"     -1: RoBERTa stream layout: -1 chosen at weight-load time from the LayerNorm
 *                       bound (fp16 hi + lo if max_c |beta_c| + sqrt(767) |gamma_c| > 64, fp16 alone
 *                       otherwise), 0 fp16, 1 fp16 hi + lo, 2 precise mode (fp32 stream, LayerNorm,
 *                       attention and branch outputs; GEMM operands per "text_prec_mask").  2 needs
 *                       the precise weights (packed unless the layout was pinned to 0 / 1 at load)
 *   "text_prec_mask" 255: precise mode operands per GEMM kind k (0 QKV, 1 out-proj, 2 FFN-1, 3 FFN-2):
 *                       bit k = hi / lo activations ([A_hi | A_lo] x [W_hi | W_hi], K = 2 in), bit
 *                       k + 4 = also W_lo (+ A_hi x W_lo, K = 3 in: ~22-bit operands); neither = fp16
 *   "effnet_fp32"    0: 1 = EfficientNet tower with fp32 activations, fp32-MFMA 1x1 convs and
 *                       precise SiLU (checkpoints whose logits amplify fp16 storage rounding)
 *   "clip_res16"     1: CLIP pre-LN residual streams in fp16 (0: fp32)
 *   "lazy_ln"        1: CLIP encoder LayerNorms folded into the GEMM epilogues
 *   "pw32_mfma"      5: fp32 tower's 1x1 convs (0 fp32-FMA VALU, 1 / 2 fp32 MFMA with 1 / 3 K-chunks
 *                       prefetched, 3 / 4 / 5 whole-row tiles; bit-identical)
 *   "effnet_chunks"  2: mmf_effnet_forward batch chunks on concurrent streams
 *   "dw_cw32"        1: 32-channel groups for the standalone depthwise convs
 *   "diag_skip"      0: diagnostic bitmask of towers mmf_analyze_batch leaves out (2 EfficientNet,
 *                       4 CLIP text, 8 ViT, ...; measurement only)
 *   "qkv_attn"       1: RoBERTa L = 128: attention in the QKV GEMM's epilogue
 *   "vault_ref"      0: diagnostic: vault similarities on the VALU kernel, top-k by full sort (the
 *                       reference kernels the production MFMA / register top-k kernels equal bit for bit)
 *   "mt_enqueue"    64: batches of <= this many pairs: towers enqueued by host threads side by side
 *   "last_q1"        1: compact last encoder layers (bit 1 RoBERTa, bit 2 CLIP towers)
 *   "after_text"    12: towers of the concurrent step that start once RoBERTa is done (bitmask as
 *                       diag_skip)
 * The defaults are the measured best; with them a row's results do not depend on the
 * batch it runs in (tests/test_gpu_parity.py).  Read-only names for mmf_get_option with a handle:
 * "text_hilo_effective" (the RoBERTa layout in use) and "text_precise_packed" (bitmask of the GEMM
 * kinds whose precise-mode weights are packed, bits 0-3 as "text_prec_mask"; setting it to a subset
 * releases the others' weights). */
const char* mmf_option_name(int i); /* i-th option name, NULL past the end */
int mmf_set_option(mmf_handle* h, const char* name, int value);
int mmf_get_option(mmf_handle* h, const char* name, int* value);
/* Device bytes currently owned by the handle (weights, workspaces, vault). */
int64_t mmf_device_bytes(mmf_handle* h);

/* Low-level op exported for unit tests of the GEMM kernel: C = act(A @ W^T + bias) + residual.
 * A fp16 [M,K] (lda), W fp16 [N,K] (ldw), bias fp32 [N] or NULL, residual fp32 [M,N] (ldc) or NULL,
 * act 0 none 1 gelu-erf 2 quick_gelu 3 silu 4 relu; outputs fp32 (c32) and/or fp16 (c16) [M,N] ldc. */
int mmf_gemm_f16(const void* A, int lda, const void* W, int ldw, const float* bias, const float* residual,
                  float* c32, void* c16, int ldc, int M, int N, int K, int act, void* stream);

/* The same with the EfficientNet operands of the 1x1 convolutions: fp16 residual res16 [M,N] (ldc)
 * and a per-(image, k) fp32 scale ascale [M / rows_per_batch, K] applied to A (SE excitation). */
int mmf_gemm_f16_ex(const void* A, int lda, const void* W, int ldw, const float* bias, const void* res16,
                     const float* ascale, int rows_per_batch, void* c16, int ldc, int M, int N, int K, int act,
                     void* stream);

/* The RoBERTa precise mode's FFN-1 epilogue (gemm.hip epi 4), exported for its bit-identity test:
 * out = act(A @ W^T + bias) written as the next GEMM's split operand row -- c16[m*ldc + n] = fp16(out)
 * and, with split_lo, c16[m*ldc + N + n] = fp16(out - fp16(out)), c16[m*ldc + 2N + n] = fp16(out)
 * (ldc >= 3N).  bias fp32 [N] (required), act 1 (gelu-erf) only; persistent-tile shapes only
 * (K % 64 == 0, N % 8 == 0), else MMF_EINVAL. */
int mmf_gemm_f16_split(const void* A, int lda, const void* W, int ldw, const float* bias, void* c16, int ldc, int M,
                       int N, int K, int act, int split_lo, void* stream);

/* Low-level attention op for tests: qkv fp16 [B*L, 3*H*64] (q|k|v), mask int32 [B,L] or NULL,
 * causal 0/1 -> out fp16 [B*L, H*64].  L <= 512. */
int mmf_attention_f16(const void* qkv, const int32_t* mask, void* out, int B, int L, int H, int causal,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMF_HIP_H */
