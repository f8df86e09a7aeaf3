// C-ABI of libmmf_hip.so (include/mmf_hip.h): handle, weight packing, workspaces and the launch
// sequences of the five signals.  Host C++ over the HIP runtime; no torch types cross this ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mmf_hip.h"
#include "kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(MMF_EIO, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)
#define CHK(expr)            \
  do {                       \
    int r_ = (expr);         \
    if (r_ != 0) return r_;  \
  } while (0)

// float -> IEEE fp16 bits, round-to-nearest-even (the compiler's _Float16 conversion)
uint16_t f2h_host(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}

float h2f_host(uint16_t b) {
  _Float16 h;
  std::memcpy(&h, &b, 2);
  return (float)h;
}

struct HostT {
  std::vector<int64_t> shape;
  std::vector<float> f;
  size_t numel() const { return f.size(); }
};

struct Lin16 {
  f16_t* w = nullptr;
  float* b = nullptr;
  int out = 0, in = 0;
  float* w32 = nullptr;  // fp32 copy of w (EfficientNet 1x1 convs: the effnet_fp32 tower)
};
struct LNp { float* g = nullptr; float* b = nullptr; };
// qkv_f / fc1_f (CLIP): the QKV and FFN-1 projections with their input LayerNorm folded in (lazy
// LN, gemm.hip): w' = fp16(w diag(gamma)), bias c = b + w beta, u = rows of w' summed (fp16 values)
struct EncLayer {
  Lin16 qkv, o, fc1, fc2;
  LNp ln1, ln2;
  Lin16 qkv_f, fc1_f;
  float *qkv_u = nullptr, *fc1_u = nullptr;
  Lin16 qkv_h;  // RoBERTa: the fused QKV with rows interleaved per head, [q_h; k_h; v_h] (gemm.hip epi 3)
  // RoBERTa precise mode (text_hilo = 2, precise.hip): [W_hi | W_hi | W_lo] along K (in = 3 K), the
  // bias shared with the fp16 copy
  Lin16 qkv3, o3, fc13, fc23;
};

struct EffBlock {
  int expand, k, stride, cin, cout, cexp, csq, residual;
  Lin16 e, p;            // expand / project 1x1 convs (BN folded)
  float* wd = nullptr;   // depthwise [cexp][k*k] (BN folded)
  float* wd_t = nullptr; // the same, tap-major [k*k][cexp] (fp32 tower)
  float* bd = nullptr;
  float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr, *b2 = nullptr;  // SE
};

const int kStages[7][6] = {{1, 3, 1, 32, 16, 1},  {6, 3, 2, 16, 24, 2},   {6, 5, 2, 24, 40, 2},  {6, 3, 2, 40, 80, 3},
                           {6, 5, 1, 80, 112, 3}, {6, 5, 2, 112, 192, 4}, {6, 3, 1, 192, 320, 1}};

struct Workspace {
  // RoBERTa
  float *r_x = nullptr, *r_y = nullptr;
  uint16_t* r_lo = nullptr;  // fp16 low part of the split post-LN residual stream (hi = r_xb)
  int* r_ovf = nullptr;      // [cap_b] overflow sentinel of the fp16 / split stream (norm.hip; run_text)
  f16_t *r_xb = nullptr, *r_qkv = nullptr, *r_ctx = nullptr, *r_h = nullptr;
  // CLIP vision
  f16_t *v_col = nullptr, *v_xb = nullptr, *v_qkv = nullptr, *v_ctx = nullptr, *v_h = nullptr, *v_cls = nullptr;
  float *v_patch = nullptr, *v_x = nullptr, *v_emb = nullptr, *v_xc = nullptr;
  f16_t* v_ctxc = nullptr;
  // CLIP text
  f16_t *t_xb = nullptr, *t_qkv = nullptr, *t_ctx = nullptr, *t_h = nullptr, *t_pool = nullptr, *t_ctxc = nullptr;
  float *t_x = nullptr, *t_emb = nullptr, *t_xc = nullptr;
  int32_t* t_eos = nullptr;
  // lazy-LN row partials of the CLIP streams (gemm.hip), two per tower (a producer writes the one
  // its stream's previous partials are not in): [rows padded to 256][kLnP] float2
  float2 *v_st[2] = {nullptr, nullptr}, *t_st[2] = {nullptr, nullptr};
  // EfficientNet
  f16_t *e_a = nullptr, *e_b = nullptr, *e_exp = nullptr, *e_dw = nullptr;
  float *e_pool = nullptr, *e_scale = nullptr;
  // fp32 EfficientNet activations (option effnet_fp32), allocated on first use for cap_b images
  float *e32_a = nullptr, *e32_b = nullptr, *e32_exp = nullptr, *e32_dw = nullptr;
  int e32_cap_b = 0;
  // RoBERTa precise mode (text_hilo = 2, group AG_TEXT32, allocated while the mode is selected): the
  // fp32 qkv / FFN hidden [rows][3072], the K-concatenated operands of the stream / ctx [rows][2304]
  // and of the FFN hidden [rows][9216]
  float* p32 = nullptr;
  f16_t *s3 = nullptr, *h3 = nullptr;
  size_t t32_rows = 0;
  // split-K partials of the skinny-M GEMMs, one per tower (the towers run on concurrent streams)
  float *sk_text = nullptr, *sk_vit = nullptr, *sk_ctext = nullptr;
  size_t sk_elems = 0;
  // vault
  float* s_sims = nullptr;
  int s_cap_n = 0;
};

// Run-time options.  Defaults come from the environment ONCE per process (MMF_* variables, for the
// A/B tools), are copied into every handle at mmf_create and changed with mmf_set_option; no kernel
// launch reads the environment.
struct Options {
  int concurrent = 1;   // towers of mmf_analyze_batch on concurrent streams
  int fuse_stem = 1;    // stem fused into the stage-1 depthwise conv
  int fuse_expand = 1;  // 1x1 expand fused into the depthwise conv (stages 2 - 4.3: effnet.hip expand_dw_applicable)
  int gemm_splitk = 1;  // split-K on the skinny-M GEMM path
  int gemm_config = -1; // forced GEMM instantiation (-1 = automatic)
  int gemm_group_m = 0; // persistent GEMM tile order
  int text_hilo = -1;   // RoBERTa residual stream as fp16 hi + fp16 lo (1), fp16 alone (0), or chosen at
                        // weight-load time from the LayerNorm parameters (-1, default: DESIGN §4); 2 = precise mode
  int text_prec_mask = 255;  // precise mode: bits 0-3 = GEMM kinds on hi / lo activations (1 QKV, 2 out-proj,
                             // 4 FFN-1, 8 FFN-2), bits 4-7 = the same kinds also on W_lo (3 products)
  int effnet_fp32 = 0;  // EfficientNet tower with fp32 activations (effnet_f32.hip) instead of fp16
  int clip_res16 = 1;   // CLIP pre-LN residual streams in fp16 (1, default) or fp32 (0)
  int lazy_ln = 1;      // CLIP encoder LayerNorms folded into the GEMM epilogues (gemm.hip)
  int pw32_mfma = 5;    // fp32 tower's 1x1 convs on the fp32-input MFMA (2: loads 3 K-chunks ahead, 1: one ahead;
                        // 3 / 4: whole-row tiles for the N <= 256 launches with K <= 64 / any K; 5: 4 where the
                        // row grid has the blocks for it) or the fp32-FMA VALU kernel (0) -- every mode bit-identical
  int dw_cw32 = 1;      // 32-channel groups for the standalone depthwise convs (effnet.hip dw_geometry; B=512 3.648 -> 3.595 ms)
  int effnet_chunks = 2;  // mmf_effnet_forward: batch chunks on concurrent streams (B=512: 3.82 -> 3.57 ms in bench.py)
  int qkv_attn = 1;     // RoBERTa L = 128: attention in the QKV GEMM's epilogue (gemm.hip epi 3)
  int mt_enqueue = 64;  // batches of <= this many pairs: the towers enqueued by host threads side by side
  int last_q1 = 1;      // compact last encoder layers: K / V of every row, Q + attention of the pooled rows only
                        // (bit 1: RoBERTa -- QKV 4.5 -> K/V 3 persistent rounds; bit 2: CLIP towers, whose K/V
                        // GEMMs round to as many rounds as QKV: measured slower, off)
  int diag_skip = 0;    // diagnostic: towers mmf_analyze_batch leaves out (bitmask; measurement only)
  int vault_ref = 0;    // diagnostic: vault similarities on the VALU kernel and top-k by full sort (the
                        // reference kernels the production ones are bit-identical to)
  int after_text = 12;  // towers of the concurrent B > mt_enqueue step that start only once RoBERTa is done
                        // (bitmask as diag_skip: 2 EfficientNet, 4 CLIP text, 8 ViT)
};
// (Round 6 measured and removed gemm_kloop -- ping-pong and A-ring K loops; round 5 removed
// the options whose variants were measured slower and stayed off: gemm_ring, gemm_wide,
// gemm_w4, dw_v2, dw_persist, ln_prod256, cu_split, fuse_expand32, qkv_attn_gm, splitk_fix, gemm_tq,
// se_group, splitk_min_k, and pinned gemm_prio = 2 / dw_ct = 1; DESIGN.md §3 keeps each measurement.)
struct OptName { const char* name; int Options::*field; const char* env; };
const OptName kOptNames[] = {
    {"concurrent", &Options::concurrent, "MMF_CONCURRENT"},   {"fuse_stem", &Options::fuse_stem, "MMF_FUSE_STEM"},
    {"fuse_expand", &Options::fuse_expand, "MMF_FUSE_EXPAND"},
    {"gemm_splitk", &Options::gemm_splitk, "MMF_GEMM_SPLITK"}, {"gemm_config", &Options::gemm_config, "MMF_GEMM_CONFIG"},
    {"gemm_group_m", &Options::gemm_group_m, "MMF_GEMM_GROUPM"},
    {"text_hilo", &Options::text_hilo, "MMF_TEXT_HILO"}, {"text_prec_mask", &Options::text_prec_mask, "MMF_TEXT_PREC_MASK"},
    {"effnet_fp32", &Options::effnet_fp32, "MMF_EFFNET_FP32"},
    {"clip_res16", &Options::clip_res16, "MMF_CLIP_RES16"}, {"lazy_ln", &Options::lazy_ln, "MMF_LAZY_LN"},
    {"pw32_mfma", &Options::pw32_mfma, "MMF_PW32_MFMA"},
    {"effnet_chunks", &Options::effnet_chunks, "MMF_EFFNET_CHUNKS"}, {"dw_cw32", &Options::dw_cw32, "MMF_DW_CW32"},
    {"diag_skip", &Options::diag_skip, "MMF_DIAG_SKIP"}, {"qkv_attn", &Options::qkv_attn, "MMF_QKV_ATTN"},
    {"vault_ref", &Options::vault_ref, "MMF_VAULT_REF"},
    {"mt_enqueue", &Options::mt_enqueue, "MMF_MT_ENQUEUE"}, {"last_q1", &Options::last_q1, "MMF_LAST_Q1"},
    {"after_text", &Options::after_text, "MMF_AFTER_TEXT"},
};
Options& process_options() {
  static Options o = [] {
    Options d;
    for (const OptName& n : kOptNames) {
      const char* e = getenv(n.env);
      if (e && *e) d.*(n.field) = atoi(e);
    }
    return d;
  }();
  return o;
}

void apply_options(const Options& o, GemmArgs* g) {
  g->force_cfg = o.gemm_config >= 0 ? o.gemm_config + 1 : 0;
  g->no_splitk = o.gemm_splitk ? 0 : 1;
  g->group_m = o.gemm_group_m;
}

// Device allocations are owned per group so that re-loading one component (or the vault, or the
// workspaces) frees exactly what it replaces.
enum AllocGroup {
  AG_WS = 0, AG_TEXT, AG_EFF, AG_VIS, AG_CTEXT, AG_FUSION, AG_VAULT, AG_TITLES, AG_SIMS, AG_EFF32, AG_RESIZE, AG_TEXT32,
  // the RoBERTa precise mode's K-concatenated weights, one group per GEMM kind (bit k of option
  // text_prec_mask <-> group AG_TP0 + k: QKV, out-proj, FFN-1, FFN-2), releasable one kind at a time
  AG_TP0, AG_TP1, AG_TP2, AG_TP3,
  AG_COUNT
};

}  // namespace

// Host threads that enqueue mmf_analyze_batch's towers side by side (option mt_enqueue).  A small
// batch is host-enqueue bound: each tower is a chain of ~140 launches at ~2.3 us of host time each,
// and enqueued one tower after another the last tower starts ~0.8 ms into the call.  Each worker
// owns one tower stream; HIP's current device is per thread, so every worker sets it once.
struct EnqueuePool {
  struct Slot {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<int()> job;
    bool busy = false, quit = false;
    int rc = 0;
    std::string err;
  };
  Slot slots[3];
  int device = 0;
  bool started = false;
  void start(int dev) {
    device = dev;
    for (Slot& sl : slots) sl.th = std::thread([this, &sl] { loop(sl); });
    started = true;
  }
  void loop(Slot& sl) {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(sl.mu);
    for (;;) {
      sl.cv.wait(lk, [&] { return sl.busy || sl.quit; });
      if (sl.quit) return;
      lk.unlock();
      const int rc = sl.job();
      std::string e = rc ? g_err : std::string();  // (g_err is this worker's thread-local message)
      lk.lock();
      sl.rc = rc;
      sl.err = e;
      sl.busy = false;
      sl.cv.notify_all();
    }
  }
  void submit(int i, std::function<int()> f) {
    Slot& sl = slots[i];
    std::lock_guard<std::mutex> lk(sl.mu);
    sl.job = std::move(f);
    sl.busy = true;
    sl.cv.notify_all();
  }
  int wait(int i, std::string* err) {
    Slot& sl = slots[i];
    std::unique_lock<std::mutex> lk(sl.mu);
    sl.cv.wait(lk, [&] { return !sl.busy; });
    if (sl.rc && err) *err = sl.err;
    return sl.rc;
  }
  ~EnqueuePool() {
    if (!started) return;
    for (Slot& sl : slots) {
      {
        std::lock_guard<std::mutex> lk(sl.mu);
        sl.quit = true;
      }
      sl.cv.notify_all();
    }
    for (Slot& sl : slots)
      if (sl.th.joinable()) sl.th.join();
  }
};

struct mmf_handle {
  int device = 0;
  int eos_id = 49407;
  std::map<std::string, HostT> staged;
  std::vector<void*> groups[AG_COUNT];
  size_t group_bytes[AG_COUNT] = {};
  int cur_group = AG_TEXT;  // group of the weight uploads of the component being finalized
  Options opt;
  int ready = 0;
  // RoBERTa + heads
  float *r_word = nullptr, *r_pos = nullptr, *r_type0 = nullptr;
  LNp r_embln;
  EncLayer r_layers[12];
  // post-LN stream magnitude bound from the loaded LayerNorms, max_c |beta_c| + 4 |gamma_c|, and
  // the split stream it selects under text_hilo = -1 (finalize_text)
  float r_stream_mag = 0.f;
  int r_hilo_auto = 0;
  int r_precise = 0;  // bitmask of the GEMM kinds whose precise-mode weights (EncLayer qkv3 ...) are packed
  float *h_w1a = nullptr, *h_b1a = nullptr, *h_w2a = nullptr, *h_b2a = nullptr;
  float *h_w1m = nullptr, *h_b1m = nullptr, *h_w2m = nullptr, *h_b2m = nullptr;
  // EfficientNet
  float *e_stem_w = nullptr, *e_stem_b = nullptr;
  std::vector<EffBlock> e_blocks;
  Lin16 e_head;
  float *e_cls_w = nullptr, *e_cls_b = nullptr;
  // CLIP vision
  f16_t* v_patch_w = nullptr;
  float *v_cls = nullptr, *v_pos = nullptr;
  LNp v_pre, v_post;
  EncLayer v_layers[12];
  f16_t* v_proj = nullptr;
  // CLIP text
  float *t_tok = nullptr, *t_pos = nullptr;
  EncLayer t_layers[12];
  LNp t_final;
  f16_t* t_proj = nullptr;
  // fusion
  float *f_w0 = nullptr, *f_b0 = nullptr, *f_w3 = nullptr, *f_b3 = nullptr, *f_w5 = nullptr, *f_b5 = nullptr;
  // vault
  float* vault = nullptr;        // [N][512] unit rows
  float* vault_title = nullptr;  // [N][512] unit title text embeddings (or null)
  int vault_n = 0;
  // workspace capacity
  Workspace ws;
  int cap_b = 0, cap_lr = 0, cap_lc = 0;
  // per-kernel event timing (mmf_profile_begin/end)
  struct ProfRec { int ev; int kind; double flops, bytes; };
  bool prof = false;
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> ev_pool;
  int ev_used = 0;
  // fork/join streams of mmf_analyze_batch (text, effnet, clip-text towers beside the caller's)
  hipStream_t tower[3] = {nullptr, nullptr, nullptr};
  hipEvent_t fork_ev = nullptr, join_ev[3] = {nullptr, nullptr, nullptr};
  hipEvent_t text_ev = nullptr;  // RoBERTa tower done (option after_text)
  // option mt_enqueue (lazily started).  Invariant: while the workers enqueue, no tower writes to the
  // handle -- every per-launch choice is read from `opt` (set between calls, never during one) and
  // every workspace is reserved before the call (mmf_reserve); the towers' launch sequences only read
  // the handle and enqueue on their own streams.
  std::unique_ptr<EnqueuePool> pool;
  // mmf_resize_pil workspaces (grow-only, group AG_RESIZE)
  struct ResizeWs {
    ResizeJob* jobs = nullptr;
    uint8_t** outs = nullptr;
    int32_t *coef = nullptr, *bounds = nullptr;
    uint8_t* tmp = nullptr;
    size_t cap_jobs = 0, cap_coef = 0, cap_tmp = 0;
  } rs;

  ~mmf_handle() {
    pool.reset();  // workers joined before their streams go
    for (auto& g : groups)
      for (void* p : g) (void)hipFree(p);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < 3; ++i) {
      if (tower[i]) (void)hipStreamDestroy(tower[i]);
      if (join_ev[i]) (void)hipEventDestroy(join_ev[i]);
    }
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (text_ev) (void)hipEventDestroy(text_ev);
  }
};

namespace {

int dev_alloc(mmf_handle* h, void** p, size_t bytes, int group) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(MMF_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  h->groups[group].push_back(*p);
  h->group_bytes[group] += bytes;
  return 0;
}

// Free one group's buffers after the device has drained (any queued launch may still read them).
int free_group(mmf_handle* h, int group) {
  if (h->groups[group].empty()) return 0;
  HIPCHK(hipDeviceSynchronize());
  for (void* p : h->groups[group]) HIPCHK(hipFree(p));
  h->groups[group].clear();
  h->group_bytes[group] = 0;
  return 0;
}

// ---- per-kernel timing: two hipEvents around each launch while profiling is on ------------
// GEMM launches are profiled per (tile instantiation, epilogue, activation) -- one kernel symbol
// each, so the numbers line up with a rocprofv3 kernel trace of the same run.
constexpr int kGemmActs = 5, kGemmEpis = 5;
enum ProfKind {
  PK_GEMM0 = 0, PK_GEMM_LAST = kGemmConfigs * kGemmEpis * kGemmActs - 1, PK_ATTN, PK_LN, PK_EMBED, PK_IM2COL, PK_STEM, PK_DW, PK_SE,
  PK_GAP, PK_HEADS, PK_VAULT, PK_FUSION, PK_PW32, PK_COUNT
};
const char* prof_kind_name(int k) {
  static const char* names[PK_COUNT - PK_ATTN] = {"attention", "layernorm", "embed+ln", "clip_im2col", "effnet_stem",
                                                  "dwconv", "se", "gap_classifier", "text_heads", "vault", "fusion",
                                                  "pw32"};
  static char gemm_names[PK_GEMM_LAST + 1][64];
  if (k >= 0 && k <= PK_GEMM_LAST) {
    if (!gemm_names[k][0]) {
      const int epi = (k / kGemmActs) % kGemmEpis;
      snprintf(gemm_names[k], sizeof(gemm_names[k]), epi ? "%s act=%d epi=%d" : "%s act=%d",
               gemm_config_name(k / (kGemmActs * kGemmEpis)), k % kGemmActs, epi);
    }
    return gemm_names[k];
  }
  return (k >= PK_ATTN && k < PK_COUNT) ? names[k - PK_ATTN] : "?";
}

struct ProfScope {
  mmf_handle* h;
  hipStream_t s;
  int ev = -1;
  ProfScope(mmf_handle* h_, hipStream_t s_, int kind, double flops, double bytes) : h(h_), s(s_) {
    if (!h->prof) return;
    while ((int)h->ev_pool.size() < h->ev_used + 2) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      h->ev_pool.push_back(e);
    }
    ev = h->ev_used;
    h->ev_used += 2;
    (void)hipEventRecord(h->ev_pool[ev], s);
    h->prof_recs.push_back({ev, kind, flops, bytes});
  }
  ~ProfScope() {
    if (ev >= 0) (void)hipEventRecord(h->ev_pool[ev + 1], s);
  }
};

template <typename T>
int upload(mmf_handle* h, T** dst, const std::vector<T>& v) {
  void* p;
  CHK(dev_alloc(h, &p, v.size() * sizeof(T), h->cur_group));
  HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *dst = (T*)p;
  return 0;
}

int up_f32(mmf_handle* h, float** dst, const std::vector<float>& v) { return upload(h, dst, v); }
int up_f16(mmf_handle* h, f16_t** dst, const std::vector<float>& v) {
  std::vector<uint16_t> b(v.size());
  for (size_t i = 0; i < v.size(); ++i) b[i] = f2h_host(v[i]);
  return upload(h, dst, b);
}

// W [out][in] fp32 -> [W_hi | W_hi | W_lo] fp16 [out][3 in] (precise.hip: the K-concatenated weight)
int up_split3(mmf_handle* h, Lin16* dst, const std::vector<float>& w, const float* bias, int out, int in,
              int group = -1) {
  std::vector<uint16_t> b((size_t)out * 3 * in);
  for (int n = 0; n < out; ++n)
    for (int k = 0; k < in; ++k) {
      const float x = w[(size_t)n * in + k];
      const uint16_t hi = f2h_host(x);
      uint16_t* r = b.data() + (size_t)n * 3 * in;
      r[k] = hi;
      r[in + k] = hi;
      r[2 * in + k] = f2h_host(x - h2f_host(hi));
    }
  const int saved = h->cur_group;
  if (group >= 0) h->cur_group = group;
  const int r = upload(h, &dst->w, b);
  h->cur_group = saved;
  CHK(r);
  dst->b = const_cast<float*>(bias);
  dst->out = out;
  dst->in = 3 * in;
  return 0;
}

const HostT* get(mmf_handle* h, const std::string& name, size_t numel) {
  auto it = h->staged.find(name);
  if (it == h->staged.end()) {
    fail(MMF_EINVAL, "missing weight '%s'", name.c_str());
    return nullptr;
  }
  if (numel && it->second.numel() != numel) {
    fail(MMF_EINVAL, "weight '%s' has %zu elements, expected %zu", name.c_str(), it->second.numel(), numel);
    return nullptr;
  }
  return &it->second;
}
bool has(mmf_handle* h, const std::string& name) { return h->staged.count(name) != 0; }

#define GET(var, name, n)                       \
  const HostT* var = get(h, (name), (n));       \
  if (!var) return MMF_EINVAL;

int load_f32(mmf_handle* h, float** dst, const std::string& name, size_t n) {
  GET(t, name, n);
  return up_f32(h, dst, t->f);
}
// per-column vectors the lazy-LN epilogues DMA in 256-column blocks: zero-padded by 256
constexpr int kColPad = 256;
constexpr int kLnP = 8;  // lazy-LN partials per row a GEMM accepts (gemm.hip kLnPMax)
int up_f32_padded(mmf_handle* h, float** dst, std::vector<float> v) {
  v.resize(v.size() + kColPad, 0.f);
  return up_f32(h, dst, v);
}
int load_f32_padded(mmf_handle* h, float** dst, const std::string& name, size_t n) {
  GET(t, name, n);
  return up_f32_padded(h, dst, t->f);
}
int load_ln(mmf_handle* h, LNp* ln, const std::string& p, int n) {
  CHK(load_f32_padded(h, &ln->g, p + ".weight", n));
  return load_f32_padded(h, &ln->b, p + ".bias", n);
}
int load_lin(mmf_handle* h, Lin16* l, const std::string& p, int out, int in, bool bias, Lin16* split3 = nullptr,
             int split3_group = -1) {
  GET(w, p + ".weight", (size_t)out * in);
  CHK(up_f16(h, &l->w, w->f));
  if (bias) CHK(load_f32_padded(h, &l->b, p + ".bias", out));
  l->out = out;
  l->in = in;
  if (split3) CHK(up_split3(h, split3, w->f, l->b, out, in, split3_group));
  return 0;
}
// LN(x) W^T + b with LN = (gamma, beta) folded (gemm.hip lazy LN): w' = fp16(w diag(gamma)),
// u = sum_k w'[n][k] over the fp16 values (so acc - mean u is exactly sum_k w'(s_k - mean)),
// c = b + w beta, both in double
int fold_ln_lin(mmf_handle* h, Lin16* dst, float** u, const std::vector<float>& w, const std::vector<float>& b,
                int out, int in, const std::vector<float>& g, const std::vector<float>& beta) {
  std::vector<float> wf((size_t)out * in), uv(out), c(out);
  for (int n = 0; n < out; ++n) {
    double su = 0.0, sc = b[n];
    for (int k = 0; k < in; ++k) {
      const float x = w[(size_t)n * in + k] * g[k];
      wf[(size_t)n * in + k] = x;
      su += (double)h2f_host(f2h_host(x));
      sc += (double)w[(size_t)n * in + k] * beta[k];
    }
    uv[n] = (float)su;
    c[n] = (float)sc;
  }
  CHK(up_f16(h, &dst->w, wf));
  CHK(up_f32_padded(h, &dst->b, c));
  CHK(up_f32_padded(h, u, uv));
  dst->out = out;
  dst->in = in;
  return 0;
}
int fold_ln_named(mmf_handle* h, Lin16* dst, float** u, const std::string& lin, int out, int in,
                  const std::string& ln) {
  GET(w, lin + ".weight", (size_t)out * in);
  GET(b, lin + ".bias", out);
  GET(g, ln + ".weight", in);
  GET(be, ln + ".bias", in);
  return fold_ln_lin(h, dst, u, w->f, b->f, out, in, g->f, be->f);
}
// fused QKV: rows [q; k; v] of [3*H][H] + bias; with ln (non-empty) also the LN-folded copy; with
// heads also the per-head interleaved copy qkv_h (row 192 h + 64 part + d = row H part + 64 h + d)
int load_qkv(mmf_handle* h, EncLayer* L, const std::string& q, const std::string& k, const std::string& v, int H,
             const std::string& ln, bool heads = false, bool split3 = false) {
  Lin16* l = &L->qkv;
  std::vector<float> w((size_t)3 * H * H), b((size_t)3 * H);
  const std::string names[3] = {q, k, v};
  for (int i = 0; i < 3; ++i) {
    GET(tw, names[i] + ".weight", (size_t)H * H);
    GET(tb, names[i] + ".bias", (size_t)H);
    std::memcpy(w.data() + (size_t)i * H * H, tw->f.data(), sizeof(float) * H * H);
    std::memcpy(b.data() + (size_t)i * H, tb->f.data(), sizeof(float) * H);
  }
  CHK(up_f16(h, &l->w, w));
  CHK(up_f32_padded(h, &l->b, b));
  l->out = 3 * H;
  l->in = H;
  if (split3) CHK(up_split3(h, &L->qkv3, w, l->b, 3 * H, H, AG_TP0));
  if (heads) {
    std::vector<float> wh(w.size()), bh(b.size());
    for (int hd = 0; hd < H / 64; ++hd)
      for (int part = 0; part < 3; ++part)
        for (int d = 0; d < 64; ++d) {
          const size_t src = (size_t)part * H + hd * 64 + d, dst = (size_t)hd * 192 + part * 64 + d;
          std::memcpy(wh.data() + dst * H, w.data() + src * H, sizeof(float) * H);
          bh[dst] = b[src];
        }
    CHK(up_f16(h, &L->qkv_h.w, wh));
    CHK(up_f32_padded(h, &L->qkv_h.b, bh));
    L->qkv_h.out = 3 * H;
    L->qkv_h.in = H;
  }
  if (ln.empty()) return 0;
  GET(g, ln + ".weight", H);
  GET(be, ln + ".bias", H);
  return fold_ln_lin(h, &L->qkv_f, &L->qkv_u, w, b, 3 * H, H, g->f, be->f);
}

// BatchNorm (eval) folded into the preceding conv: w' = w * g/sqrt(v+eps), b' = beta - m*g/sqrt(v+eps)
int fold_bn(mmf_handle* h, const std::string& conv, const std::string& bn, int cout, size_t per_out,
            std::vector<float>* w, std::vector<float>* b) {
  GET(cw, conv + ".weight", (size_t)cout * per_out);
  GET(g, bn + ".weight", cout);
  GET(be, bn + ".bias", cout);
  GET(m, bn + ".running_mean", cout);
  GET(v, bn + ".running_var", cout);
  w->resize((size_t)cout * per_out);
  b->resize(cout);
  for (int o = 0; o < cout; ++o) {
    const double s = (double)g->f[o] / std::sqrt((double)v->f[o] + 1e-5);
    for (size_t i = 0; i < per_out; ++i) (*w)[(size_t)o * per_out + i] = (float)(cw->f[(size_t)o * per_out + i] * s);
    (*b)[o] = (float)((double)be->f[o] - (double)m->f[o] * s);
  }
  return 0;
}

std::vector<float> transpose(const std::vector<float>& a, int rows, int cols) {
  std::vector<float> t((size_t)rows * cols);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) t[(size_t)c * rows + r] = a[(size_t)r * cols + c];
  return t;
}

int finalize_text(mmf_handle* h) {
  const std::string p = "roberta.";
  CHK(load_f32(h, &h->r_word, p + "embeddings.word_embeddings.weight", (size_t)50265 * 768));
  CHK(load_f32(h, &h->r_pos, p + "embeddings.position_embeddings.weight", (size_t)514 * 768));
  {
    GET(t, p + "embeddings.token_type_embeddings.weight", 0);
    std::vector<float> t0(t->f.begin(), t->f.begin() + 768);
    CHK(up_f32(h, &h->r_type0, t0));
  }
  CHK(load_ln(h, &h->r_embln, p + "embeddings.LayerNorm", 768));
  {
    // RoBERTa's residual stream IS a LayerNorm output (post-LN): x_c = beta_c + gamma_c xhat_c, and
    // over C channels |xhat_c| <= sqrt(C - 1) (reached when one channel carries all of the row's
    // variance -- exactly the outlier-channel case), so |x_c| <= |beta_c| + sqrt(767) |gamma_c| is a
    // sound bound for every input.  Trained models put O(1e2-1e3) "outlier" values in a few
    // channels; stored in fp16 alone (2^-11 relative) their rounding shifts every next LayerNorm's
    // mean coherently across all channels (tests/test_gpu_outliers.py: 1.6e-3 at a 900-level
    // outlier vs 2.2e-4 on the plain draw), so above kHiloMag the split hi + lo stream (~22 bits)
    // is used.  (Round 3 bounded |xhat| by 4, which a dominating channel exceeds: VERDICT r3.)
    constexpr float kHiloMag = 64.f;
    const float kXhatMax = std::sqrt(767.f);
    float mag = 0.f;
    auto scan = [&](const std::string& ln) -> int {
      GET(g, ln + ".weight", 768);
      GET(b, ln + ".bias", 768);
      for (int c = 0; c < 768; ++c) mag = std::max(mag, std::fabs(b->f[c]) + kXhatMax * std::fabs(g->f[c]));
      return 0;
    };
    CHK(scan(p + "embeddings.LayerNorm"));
    for (int i = 0; i < 12; ++i) {
      const std::string l = p + "encoder.layer." + std::to_string(i) + ".";
      CHK(scan(l + "attention.output.LayerNorm"));
      CHK(scan(l + "output.LayerNorm"));
    }
    h->r_stream_mag = mag;
    h->r_hilo_auto = mag > kHiloMag ? 1 : 0;
  }
  // the precise mode's K-concatenated weights (+510 MB) are packed unless the layout is pinned to an
  // fp16 stream (text_hilo 0 / 1): the load-time calibration (engine.py) may select the mode
  // (each kind's K-concatenated weights in its own allocation group AG_TP0 + k, so that the engine's
  // calibration can release the kinds the selected mode does not read: option text_precise_packed)
  const bool sp = h->opt.text_hilo < 0 || h->opt.text_hilo >= 2;
  h->r_precise = 0;
  for (int k = 0; k < 4; ++k) CHK(free_group(h, AG_TP0 + k));
  for (int i = 0; i < 12; ++i) {
    const std::string l = p + "encoder.layer." + std::to_string(i) + ".";
    EncLayer& L = h->r_layers[i];
    L.qkv3 = L.o3 = L.fc13 = L.fc23 = Lin16{};
    CHK(load_qkv(h, &L, l + "attention.self.query", l + "attention.self.key", l + "attention.self.value", 768, "",
                 true, sp));
    CHK(load_lin(h, &L.o, l + "attention.output.dense", 768, 768, true, sp ? &L.o3 : nullptr, AG_TP0 + 1));
    CHK(load_ln(h, &L.ln1, l + "attention.output.LayerNorm", 768));
    CHK(load_lin(h, &L.fc1, l + "intermediate.dense", 3072, 768, true, sp ? &L.fc13 : nullptr, AG_TP0 + 2));
    CHK(load_lin(h, &L.fc2, l + "output.dense", 768, 3072, true, sp ? &L.fc23 : nullptr, AG_TP0 + 3));
    CHK(load_ln(h, &L.ln2, l + "output.LayerNorm", 768));
  }
  h->r_precise = sp ? 15 : 0;
  for (int hd = 0; hd < 2; ++hd) {
    const std::string n = hd ? "misinfo_head" : "ai_head";
    GET(w1, n + ".0.weight", (size_t)256 * 768);
    float** w1d = hd ? &h->h_w1m : &h->h_w1a;
    CHK(up_f32(h, w1d, transpose(w1->f, 256, 768)));
    CHK(load_f32(h, hd ? &h->h_b1m : &h->h_b1a, n + ".0.bias", 256));
    CHK(load_f32(h, hd ? &h->h_w2m : &h->h_w2a, n + ".3.weight", 512));
    CHK(load_f32(h, hd ? &h->h_b2m : &h->h_b2a, n + ".3.bias", 2));
  }
  return 0;
}

int finalize_effnet(mmf_handle* h) {
  const std::string p = "efficientnet.features.";
  std::vector<float> w, b;
  CHK(fold_bn(h, p + "0.0", p + "0.1", 32, 27, &w, &b));
  CHK(up_f32(h, &h->e_stem_w, w));
  CHK(up_f32(h, &h->e_stem_b, b));
  h->e_blocks.clear();
  for (int si = 0; si < 7; ++si) {
    const int* st = kStages[si];
    for (int j = 0; j < st[5]; ++j) {
      EffBlock B{};
      B.expand = st[0];
      B.k = st[1];
      B.stride = j == 0 ? st[2] : 1;
      B.cin = j == 0 ? st[3] : st[4];
      B.cout = st[4];
      B.cexp = B.cin * B.expand;
      B.csq = B.cin / 4 > 1 ? B.cin / 4 : 1;
      B.residual = (B.stride == 1 && B.cin == B.cout);
      const std::string bp = p + std::to_string(si + 1) + "." + std::to_string(j) + ".block.";
      int i = 0;
      if (B.expand != 1) {
        CHK(fold_bn(h, bp + "0.0", bp + "0.1", B.cexp, B.cin, &w, &b));
        CHK(up_f16(h, &B.e.w, w));
        CHK(up_f32(h, &B.e.w32, w));
        CHK(up_f32(h, &B.e.b, b));
        B.e.out = B.cexp;
        B.e.in = B.cin;
        i = 1;
      }
      CHK(fold_bn(h, bp + std::to_string(i) + ".0", bp + std::to_string(i) + ".1", B.cexp, (size_t)B.k * B.k, &w, &b));
      CHK(up_f32(h, &B.wd, w));
      {
        std::vector<float> t(w.size());
        const int kk = B.k * B.k;
        for (int c = 0; c < B.cexp; ++c)
          for (int q = 0; q < kk; ++q) t[(size_t)q * B.cexp + c] = w[(size_t)c * kk + q];
        CHK(up_f32(h, &B.wd_t, t));
      }
      CHK(up_f32(h, &B.bd, b));
      const std::string se = bp + std::to_string(i + 1) + ".";
      CHK(load_f32(h, &B.w1, se + "fc1.weight", (size_t)B.csq * B.cexp));
      CHK(load_f32(h, &B.b1, se + "fc1.bias", B.csq));
      {
        GET(w2, se + "fc2.weight", (size_t)B.cexp * B.csq);
        CHK(up_f32(h, &B.w2, transpose(w2->f, B.cexp, B.csq)));  // [csq][cexp] for coalesced fc2
      }
      CHK(load_f32(h, &B.b2, se + "fc2.bias", B.cexp));
      CHK(fold_bn(h, bp + std::to_string(i + 2) + ".0", bp + std::to_string(i + 2) + ".1", B.cout, B.cexp, &w, &b));
      CHK(up_f16(h, &B.p.w, w));
      CHK(up_f32(h, &B.p.w32, w));
      CHK(up_f32(h, &B.p.b, b));
      B.p.out = B.cout;
      B.p.in = B.cexp;
      h->e_blocks.push_back(B);
    }
  }
  CHK(fold_bn(h, p + "8.0", p + "8.1", 1280, 320, &w, &b));
  CHK(up_f16(h, &h->e_head.w, w));
  CHK(up_f32(h, &h->e_head.w32, w));
  CHK(up_f32(h, &h->e_head.b, b));
  h->e_head.out = 1280;
  h->e_head.in = 320;
  CHK(load_f32(h, &h->e_cls_w, "efficientnet.classifier.1.weight", 2 * 1280));
  CHK(load_f32(h, &h->e_cls_b, "efficientnet.classifier.1.bias", 2));
  return 0;
}

int finalize_clip_layers(mmf_handle* h, EncLayer* layers, const std::string& base, int H, int I) {
  for (int i = 0; i < 12; ++i) {
    const std::string l = base + std::to_string(i) + ".";
    EncLayer& L = layers[i];
    CHK(load_qkv(h, &L, l + "self_attn.q_proj", l + "self_attn.k_proj", l + "self_attn.v_proj", H, l + "layer_norm1"));
    CHK(load_lin(h, &L.o, l + "self_attn.out_proj", H, H, true));
    CHK(load_ln(h, &L.ln1, l + "layer_norm1", H));
    CHK(load_lin(h, &L.fc1, l + "mlp.fc1", I, H, true));
    CHK(fold_ln_named(h, &L.fc1_f, &L.fc1_u, l + "mlp.fc1", I, H, l + "layer_norm2"));
    CHK(load_lin(h, &L.fc2, l + "mlp.fc2", H, I, true));
    CHK(load_ln(h, &L.ln2, l + "layer_norm2", H));
  }
  return 0;
}

int finalize_clip_vision(mmf_handle* h) {
  const std::string p = "clip.vision_model.";
  {
    GET(w, p + "embeddings.patch_embedding.weight", (size_t)768 * 3072);
    CHK(up_f16(h, &h->v_patch_w, w->f));  // [768][3*32*32] = (c, ky, kx) columns
  }
  CHK(load_f32(h, &h->v_cls, p + "embeddings.class_embedding", 768));
  CHK(load_f32(h, &h->v_pos, p + "embeddings.position_embedding.weight", 50 * 768));
  CHK(load_ln(h, &h->v_pre, p + "pre_layrnorm", 768));
  CHK(finalize_clip_layers(h, h->v_layers, p + "encoder.layers.", 768, 3072));
  CHK(load_ln(h, &h->v_post, p + "post_layernorm", 768));
  GET(pw, "clip.visual_projection.weight", (size_t)512 * 768);
  return up_f16(h, &h->v_proj, pw->f);
}

int finalize_clip_text(mmf_handle* h) {
  const std::string p = "clip.text_model.";
  CHK(load_f32(h, &h->t_tok, p + "embeddings.token_embedding.weight", (size_t)49408 * 512));
  CHK(load_f32(h, &h->t_pos, p + "embeddings.position_embedding.weight", 77 * 512));
  CHK(finalize_clip_layers(h, h->t_layers, p + "encoder.layers.", 512, 2048));
  CHK(load_ln(h, &h->t_final, p + "final_layer_norm", 512));
  GET(pw, "clip.text_projection.weight", (size_t)512 * 512);
  return up_f16(h, &h->t_proj, pw->f);
}

int finalize_fusion(mmf_handle* h) {
  CHK(load_f32(h, &h->f_w0, "fusion_layer.0.weight", 64 * 5));
  CHK(load_f32(h, &h->f_b0, "fusion_layer.0.bias", 64));
  CHK(load_f32(h, &h->f_w3, "fusion_layer.3.weight", 32 * 64));
  CHK(load_f32(h, &h->f_b3, "fusion_layer.3.bias", 32));
  CHK(load_f32(h, &h->f_w5, "fusion_layer.5.weight", 2 * 32));
  return load_f32(h, &h->f_b5, "fusion_layer.5.bias", 2);
}

// ---------------------------------------------------------------------------------------------
// forward sequences
// ---------------------------------------------------------------------------------------------
GemmArgs gemm_args(const f16_t* A, int lda, const Lin16& l, int M) {
  GemmArgs g{};
  g.A = A;
  g.lda = lda;
  g.W = l.w;
  g.ldw = l.in;
  g.bias = l.b;
  g.M = M;
  g.N = l.out;
  g.K = l.in;
  g.ldc = l.out;
  g.ldr = l.out;
  return g;
}

// split-K workspace: `elems` floats of partial planes
GemmArgs with_ws(GemmArgs g, float* ws, size_t elems) {
  g.ws = ws;
  g.ws_elems = elems;
  return g;
}

int gemm(mmf_handle* h, GemmArgs g, hipStream_t s) {
  apply_options(h->opt, &g);
  const double M = g.M, N = g.N, K = g.K;
  const double out_b = (g.c32 ? 4.0 : 0.0) + (g.c16 ? 2.0 : 0.0) + (g.res32 ? 4.0 : 0.0) + (g.res16 ? 2.0 : 0.0);
  // epi 3 also runs the attention of its rows (4 L^2 64 flops per sequence and head, L = 128) and
  // writes ctx (N / 3 columns) instead of qkv
  const double att = g.epi == 3 ? 4.0 * (M / 128) * (N / 192) * 128.0 * 128.0 * 64.0 : 0.0;
  ProfScope ps(h, s, (gemm_config(g) * kGemmEpis + g.epi) * kGemmActs + g.act, 2.0 * M * N * K + att,
               2.0 * (M * K + N * K) + M * (g.epi == 3 ? N / 3 : N) * out_b * (g.epi == 4 && g.split_lo ? 3 : 1));
  HIPCHK(launch_gemm(g, s));
  return 0;
}

// Lazy LayerNorm (option lazy_ln, gemm.hip): a row stream's statistics as partials
struct LnStats {
  float2* p = nullptr;  // [rows padded to 256][P]
  int P = 0, tn = 0;
};
// consumer: LN(s) W^T + b with the LN folded into (w', u, c) -- s = raw rows with statistics st
GemmArgs ln_consumer(const f16_t* s_rows, int ld, const Lin16& folded, const float* u, const LnStats& st, int M) {
  GemmArgs g = gemm_args(s_rows, ld, folded, M);
  g.epi = 1;
  g.ln_in = st.p;
  g.ln_in_P = st.P;
  g.ln_in_tn = st.tn;
  g.ln_u = u;
  g.ln_eps = 1e-5f;
  return g;
}
// producer: stream += A W^T + b in place; the new stream's statistics go to `out`
GemmArgs ln_producer(const Options& o, const f16_t* A, int lda, const Lin16& l, f16_t* stream, int M, float2* out,
                     LnStats* produced) {
  GemmArgs g = gemm_args(A, lda, l, M);
  apply_options(o, &g);  // the tile (so the partials' width) depends on options
  g.res16 = stream;
  g.c16 = stream;
  g.ln_out = out;
  g.ln_eps = 1e-5f;
  g.epi = 2;
  produced->p = out;
  produced->tn = gemm_ln_tn(g);
  produced->P = (l.out + produced->tn - 1) / produced->tn;
  return g;
}

int attn(mmf_handle* h, const f16_t* qkv, int ld, const int32_t* mask, f16_t* out, int ldo, int B, int L, int H,
         int causal, hipStream_t s) {
  ProfScope ps(h, s, PK_ATTN, 4.0 * B * H * (double)L * L * 64, (double)B * L * H * 64 * 2 * 4);
  HIPCHK(launch_attention(qkv, ld, mask, out, ldo, B, L, H, causal, s));
  return 0;
}

int lnorm(mmf_handle* h, const float* x, int ldx, const LNp& p, float* y32, int ldy32, f16_t* y16, int ldy16,
          int rows, int C, hipStream_t s) {
  ProfScope ps(h, s, PK_LN, 8.0 * rows * C, (double)rows * C * (4 + (y32 ? 4 : 0) + (y16 ? 2 : 0)));
  HIPCHK(launch_layernorm(x, ldx, nullptr, 0, p.g, p.b, 1e-5f, y32, ldy32, y16, ldy16, rows, C, s));
  return 0;
}

// post-LN in fp32, in place: x = LN(x + y) (precise mode; layernorm_kernel reads a row before writing it)
int lnorm_add(mmf_handle* h, float* x, const float* y, const LNp& p, int rows, hipStream_t s) {
  ProfScope ps(h, s, PK_LN, 9.0 * rows * 768, (double)rows * 768 * 12);
  HIPCHK(launch_layernorm(x, 768, y, 768, p.g, p.b, 1e-5f, x, 768, nullptr, 0, rows, 768, s));
  return 0;
}

int add_ln(mmf_handle* h, float* x, int ldx, const f16_t* y, int ldy, const LNp& p, float* s32, float* o32,
           f16_t* o16, int ldo, int rows, int C, hipStream_t s) {
  ProfScope ps(h, s, PK_LN, 9.0 * rows * C, (double)rows * C * (4 + 2 + (s32 ? 4 : 0) + (o32 ? 4 : 0) + 2));
  HIPCHK(launch_add_ln(x, ldx, y, ldy, p.g, p.b, 1e-5f, s32, o32, o16, ldo, rows, C, s));
  return 0;
}

int add_ln(mmf_handle* h, f16_t* x, int ldx, const f16_t* y, int ldy, const LNp& p, f16_t* o16, int ldo, int rows,
           int C, hipStream_t s) {
  ProfScope ps(h, s, PK_LN, 9.0 * rows * C, (double)rows * C * (2 + 2 + 2 + 2));
  HIPCHK(launch_add_ln(x, ldx, y, ldy, p.g, p.b, 1e-5f, x, o16, ldo, rows, C, s));
  return 0;
}

int add_ln_hilo(mmf_handle* h, f16_t* hi, uint16_t* lo, int ld, const f16_t* y, int ldy, const LNp& p, int rows,
                hipStream_t s, int* ovf = nullptr, int L = 0) {
  ProfScope ps(h, s, PK_LN, 9.0 * rows * 768, (double)rows * 768 * (2 + 2 + 2 + 2 + 2));
  HIPCHK(launch_add_ln_hilo(hi, lo, ld, y, ldy, p.g, p.b, 1e-5f, rows, 768, s, ovf, L));
  return 0;
}

int check_cap(mmf_handle* h, int B, int Lr, int Lc) {
  if (B <= 0) return fail(MMF_EINVAL, "batch must be > 0 (got %d)", B);
  if (B > h->cap_b || Lr > h->cap_lr || Lc > h->cap_lc)
    return fail(MMF_EINVAL, "shape B=%d Lr=%d Lc=%d exceeds reserved B=%d Lr=%d Lc=%d (call mmf_reserve)", B, Lr, Lc,
                h->cap_b, h->cap_lr, h->cap_lc);
  return 0;
}

int text_mode(const mmf_handle* h) { return h->opt.text_hilo < 0 ? h->r_hilo_auto : h->opt.text_hilo; }

// RoBERTa precise mode (text_hilo = 2; precise.hip): fp32 stream, fp32 branch outputs, LayerNorm
// and attention, every GEMM on ~22-bit operands through the K-concatenated [hi | lo | hi] x
// [W_hi | W_hi | W_lo] product on the fp16 MFMA kernels.  All 12 layers run on every row; the heads
// read the CLS rows of the final stream.  DESIGN §4 states its cost.
int run_text_precise(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* ai, float* mi,
                     float* scores, int score_stride, hipStream_t s) {
  Workspace& w = h->ws;
  const int M = B * L;
  const int pm = h->opt.text_prec_mask & 15;  // kinds on hi / lo activations: [A_hi | A_lo] x [W_hi | W_hi] (K = 2 in)
  const int pw = pm & (h->opt.text_prec_mask >> 4);  // ... of them also on W_lo: + A_hi x W_lo (K = 3 in)
  if (pm & ~h->r_precise)
    return fail(MMF_EINVAL, "text_hilo = 2: text_prec_mask %d needs precise-mode weights that are not packed (packed: %d; "
                            "re-load the text model with text_hilo -1 or 2)", pm, h->r_precise);
  if (!w.p32 || w.t32_rows < (size_t)M) return fail(MMF_EINVAL, "text_hilo = 2: precise workspaces not reserved");
  float* x = w.r_x;  // the fp32 residual stream [M][768]
  float* y = w.r_y;  // branch outputs / ctx [M][768]
  {
    ProfScope ps(h, s, PK_EMBED, 10.0 * M * 768, (double)M * 768 * (4 + 4 + 4));
    HIPCHK(launch_roberta_embed(ids, h->r_word, h->r_pos, h->r_type0, h->r_embln.g, h->r_embln.b, 1e-5f, nullptr,
                                w.r_xb, B, L, 768, 1, s, x));
  }
  // GEMM kind k on hi / lo operands (bit k of text_prec_mask): the K-concatenated weight, K = 3 in;
  // otherwise the fp16 weight against the hi third of the same operand rows (K = in): fp16 x fp16
  // products, fp32 accumulation and output.  split3 writes the lo / second hi thirds only for a
  // consumer that reads them.
  auto lin = [&](const f16_t* A, int lda, const Lin16& fast, const Lin16& prec, int kind) {
    if (!(pm >> kind & 1)) return gemm_args(A, lda, fast, M);
    GemmArgs g = gemm_args(A, lda, prec, M);
    if (!(pw >> kind & 1)) g.K = 2 * fast.in;  // the first two thirds of the concatenated rows
    return g;
  };
  HIPCHK(launch_split3(x, 768, w.s3, M, 768, s, pm & 1));
  for (int i = 0; i < 12; ++i) {
    const EncLayer& Ly = h->r_layers[i];
    GemmArgs g = with_ws(lin(w.s3, 2304, Ly.qkv, Ly.qkv3, 0), w.sk_text, w.sk_elems);
    g.c32 = w.p32;
    g.ldc = 2304;
    CHK(gemm(h, g, s));
    {
      ProfScope ps(h, s, PK_ATTN, 4.0 * B * 12 * (double)L * L * 64, (double)M * (2304 + 768) * 4);
      // ctx straight into the out-projection's operand rows (no fp32 ctx / split3 pass)
      HIPCHK(launch_attention32(w.p32, 2304, 768, 1536, mask, y, 768, B, L, 12, s, w.s3, pm >> 1 & 1));
    }
    g = with_ws(lin(w.s3, 2304, Ly.o, Ly.o3, 1), w.sk_text, w.sk_elems);
    g.c32 = y;
    CHK(gemm(h, g, s));
    {  // x = LN1(x + y) and FFN-1's operand rows of it, one pass
      ProfScope ps(h, s, PK_LN, 9.0 * M * 768, (double)M * 768 * 14);
      HIPCHK(launch_layernorm_split3(x, y, Ly.ln1.g, Ly.ln1.b, 1e-5f, w.s3, pm >> 2 & 1, M, 768, s));
    }
    g = with_ws(lin(w.s3, 2304, Ly.fc1, Ly.fc13, 2), w.sk_text, w.sk_elems);
    g.act = 1;  // GELU-erf
    // the hidden straight into FFN-2's operand rows (epilogue 4: hi | lo | hi, no fp32 hidden and
    // no split3 pass: -8 B of HBM traffic per hidden element); the fp32 + split3 path where the
    // persistent tiles do not apply (small batches)
    GemmArgs ge = g;
    ge.epi = 4;
    ge.split_lo = pm >> 3 & 1;
    ge.c16 = w.h3;
    ge.ldc = 9216;
    if (gemm_epi_ok(ge)) {
      CHK(gemm(h, ge, s));
    } else {
      g.c32 = w.p32;
      g.ldc = 3072;
      CHK(gemm(h, g, s));
      HIPCHK(launch_split3(w.p32, 3072, w.h3, M, 3072, s, pm >> 3 & 1));
    }
    g = with_ws(lin(w.h3, 9216, Ly.fc2, Ly.fc23, 3), w.sk_text, w.sk_elems);
    g.c32 = y;
    CHK(gemm(h, g, s));
    if (i < 11) {  // x = LN2(x + y) and the next layer's QKV operand rows of it
      ProfScope ps(h, s, PK_LN, 9.0 * M * 768, (double)M * 768 * 14);
      HIPCHK(launch_layernorm_split3(x, y, Ly.ln2.g, Ly.ln2.b, 1e-5f, w.s3, pm & 1, M, 768, s));
    } else {
      CHK(lnorm_add(h, x, y, Ly.ln2, M, s));
    }
  }
  ProfScope ps(h, s, PK_HEADS, 2.0 * B * 2 * (768 * 256 + 256 * 2), (double)B * 768 * 4 + 2 * 768 * 256 * 4);
  HIPCHK(launch_text_heads(x, L * 768, h->h_w1a, h->h_b1a, h->h_w2a, h->h_b2a, h->h_w1m, h->h_b1m, h->h_w2m,
                           h->h_b2m, ai, mi, scores, score_stride, B, s));
  return 0;
}

// heads_ev: recorded once the encoder is done, before the heads (mmf_analyze_batch's after_text event:
// the waiting towers start while the two small head MLPs run)
int run_text(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* ai, float* mi,
             float* scores, int score_stride, hipStream_t s, hipEvent_t heads_ev = nullptr) {
  Workspace& w = h->ws;
  const int hilo = text_mode(h);
  if (hilo >= 2) {
    CHK(run_text_precise(h, ids, mask, B, L, ai, mi, scores, score_stride, s));
    if (heads_ev) HIPCHK(hipEventRecord(heads_ev, s));
    return 0;
  }
  uint16_t* rlo = hilo ? w.r_lo : nullptr;
  const int M = B * L;
  // overflow sentinel: a sequence whose fp16 stream or branch output leaves fp16's range gets NaN
  // scores (the masked softmax would hide it; engine.py's run-time trap then re-runs the batch in the
  // precise mode)
  int* ovf = w.r_ovf;
  HIPCHK(hipMemsetAsync(ovf, 0, (size_t)B * sizeof(int), s));
  {
    ProfScope ps(h, s, PK_EMBED, 10.0 * M * 768, (double)M * 768 * (4 + 4 + 2 + 2));
    HIPCHK(launch_roberta_embed(ids, h->r_word, h->r_pos, h->r_type0, h->r_embln.g, h->r_embln.b, 1e-5f, rlo,
                                w.r_xb, B, L, 768, 1, s, nullptr, ovf));
  }
  for (int i = 0; i < 12; ++i) {
    const EncLayer& Ly = h->r_layers[i];
    // last layer: only the CLS row feeds the heads (misinfo_forensics.py:95), so the rows below
    // run on B compact CLS rows (strided A / residual reads) instead of B*L rows
    const bool last = (i == 11);
    GemmArgs g;
    // (split-stream mode -- outlier-feature checkpoints, which sit at the parity bar: DESIGN §4 --
    // keeps the full last-layer attention, whose roundings were measured there)
    if (last && (h->opt.last_q1 & 1) && !rlo) {
      // ... and of its attention only the CLS queries are needed: K and V of every row (the fused
      // weight's rows 768..2303: 3 whole persistent rounds at M = 32768 instead of 4.5), Q of the
      // B CLS rows (skinny, split-K), one query per (sequence, head) (attention_q1_kernel) written
      // to the CLS rows of r_ctx
      Lin16 kv = Ly.qkv;
      kv.w += (size_t)768 * 768;
      kv.b += 768;
      kv.out = 1536;
      g = with_ws(gemm_args(w.r_xb, 768, kv, M), w.sk_text, w.sk_elems);
      g.c16 = w.r_qkv + 768;
      g.ldc = 2304;
      CHK(gemm(h, g, s));
      // Q of the CLS rows in fp32 (r_y is free until hilo_rows below); with the split stream the
      // lo word is added by a second skinny GEMM (q = Wq hi + bq + Wq lo: the ~22-bit row)
      Lin16 qq = Ly.qkv;
      qq.out = 768;
      float* qcls = w.r_y;
      g = with_ws(gemm_args(w.r_xb, L * 768, qq, B), w.sk_text, w.sk_elems);
      g.c32 = qcls;
      CHK(gemm(h, g, s));
      if (rlo) {
        g = with_ws(gemm_args(reinterpret_cast<const f16_t*>(rlo), L * 768, qq, B), w.sk_text, w.sk_elems);
        g.bias = nullptr;
        g.res32 = qcls;
        g.c32 = qcls;
        CHK(gemm(h, g, s));
      }
      ProfScope ps(h, s, PK_ATTN, 4.0 * B * 12 * (double)L * 64, (double)B * L * 768 * 2 * 2);
      HIPCHK(launch_attention_q1(qcls, 768, w.r_qkv, 2304, 768, 1536, mask, nullptr, w.r_ctx, L * 768, B, L, 12, s));
    } else if (h->opt.qkv_attn && L == 128 && M > 512) {
      // the attention of each (two sequences, head) tile inside the QKV GEMM's epilogue: ctx is
      // written directly (bit-identical to the two launches below, tests/test_gpu_parity.py)
      g = gemm_args(w.r_xb, 768, Ly.qkv_h, M);
      g.epi = 3;
      g.amask = mask;
      g.c16 = w.r_ctx;
      g.ldc = 768;
      CHK(gemm(h, g, s));
    } else {
      // (M <= 512, a single text or a few: split-K through the workspace, gemm_splitk_factor)
      g = with_ws(gemm_args(w.r_xb, 768, Ly.qkv, M), w.sk_text, w.sk_elems);
      g.c16 = w.r_qkv;
      CHK(gemm(h, g, s));
      CHK(attn(h, w.r_qkv, 2304, mask, w.r_ctx, 768, B, L, 12, 0, s));
    }
    if (!last) {
      // out-proj and FFN-2 write their fp16 branch output y; the residual add happens in fp32
      // inside add+LN (y lives in r_h, free until FFN-1, then in r_ctx, free after out-proj)
      f16_t* y = w.r_h;
      g = with_ws(gemm_args(w.r_ctx, 768, Ly.o, M), w.sk_text, w.sk_elems);
      g.c16 = y;
      CHK(gemm(h, g, s));
      CHK(add_ln_hilo(h, w.r_xb, rlo, 768, y, 768, Ly.ln1, M, s, ovf, L));
      g = with_ws(gemm_args(w.r_xb, 768, Ly.fc1, M), w.sk_text, w.sk_elems);
      g.act = 1;  // GELU-erf
      g.c16 = w.r_h;
      CHK(gemm(h, g, s));
      y = w.r_ctx;
      g = with_ws(gemm_args(w.r_h, 3072, Ly.fc2, M), w.sk_text, w.sk_elems);
      g.c16 = y;
      CHK(gemm(h, g, s));
      CHK(add_ln_hilo(h, w.r_xb, rlo, 768, y, 768, Ly.ln2, M, s, ovf, L));
      continue;
    }
    const int Mr = last ? B : M;            // rows after the attention
    const int rs = last ? L * 768 : 768;    // row stride of ctx at this point
    // the B CLS rows of the split residual stream, as fp32 (r_y, compact)
    HIPCHK(launch_hilo_rows(w.r_xb, rlo, rs, w.r_y, B, 768, s));
    g = with_ws(gemm_args(w.r_ctx, rs, Ly.o, Mr), w.sk_text, w.sk_elems);
    g.res32 = w.r_y;
    g.ldr = 768;
    g.c32 = w.r_y;
    CHK(gemm(h, g, s));
    CHK(lnorm(h, w.r_y, 768, Ly.ln1, last ? w.r_y : w.r_x, 768, w.r_xb, 768, Mr, 768, s));
    g = with_ws(gemm_args(w.r_xb, 768, Ly.fc1, Mr), w.sk_text, w.sk_elems);
    g.act = 1;  // GELU-erf
    g.c16 = w.r_h;
    CHK(gemm(h, g, s));
    g = with_ws(gemm_args(w.r_h, 3072, Ly.fc2, Mr), w.sk_text, w.sk_elems);
    g.res32 = last ? w.r_y : w.r_x;
    g.c32 = last ? w.r_x : w.r_y;
    CHK(gemm(h, g, s));
    CHK(lnorm(h, last ? w.r_x : w.r_y, 768, Ly.ln2, w.r_x, 768, w.r_xb, 768, Mr, 768, s));
  }
  // w.r_x now holds the B final CLS rows, compact
  if (heads_ev) HIPCHK(hipEventRecord(heads_ev, s));
  ProfScope ps(h, s, PK_HEADS, 2.0 * B * 2 * (768 * 256 + 256 * 2), (double)B * 768 * 4 + 2 * 768 * 256 * 4);
  HIPCHK(launch_text_heads(w.r_x, 768, h->h_w1a, h->h_b1a, h->h_w2a, h->h_b2a, h->h_w1m, h->h_b1m, h->h_w2m,
                           h->h_b2m, ai, mi, scores, score_stride, B, s, ovf));
  return 0;
}

// pre-LN CLIP encoder over x (residual stream, in place: fp32, or fp16 when opt.clip_res16) with
// xb = LN1_0(x) already computed
// Only one row per sequence is consumed after the last layer (CLS for the ViT, EOS for the text
// tower: TF clip:561-582, 650-651): the last layer's out-proj / MLP run on those B rows, gathered
// into compact buffers (xc fp32, ctxc fp16); on return xc holds them (before the final LN).
// independent of the batch size: rows must not change with the batch they run in (the lazy and
// materialised LayerNorms round differently), so sharding rows over GPUs keeps results bit-identical
// The exception is the latency regime: below kLazyMinRows rows (a ViT batch of <= 5 images, a text
// batch of <= 3 captions: analyze() one pair at a time) the 256-row lazy-LN tiles leave all but a
// few CUs idle (4-12 workgroups walking K = 768-3072: 20-37 us per GEMM at B = 1), so those batches
// run the materialised LayerNorms with split-K GEMMs; rows of batches >= 8 (the bench, shards) stay
// bit-identical across batch sizes (tests/test_gpu_parity.py), small batches match them to rounding.
constexpr int kLazyMinRows = 256;
bool clip_lazy(mmf_handle* h, int M) { return h->opt.lazy_ln && h->opt.clip_res16 && M >= kLazyMinRows; }

// One CLIP tower's encoder pass: its weights, workspaces and (lazy LN) the statistics of its stream
struct ClipEnc {
  EncLayer* layers;
  int H, I, heads;
  float* x;  // residual stream (fp32, or fp16 when opt.clip_res16: x16)
  f16_t *x16, *xb, *qkv, *ctx, *hid;
  const int32_t* mask;
  int causal, B, L, M;
  const int32_t* last_rows;
  float* xc;
  f16_t* ctxc;
  float* skws;
  size_t sk_elems;
  float2* const* st;
  bool lazy;
  LnStats cur;  // lazy LN: partials of the current stream
  int sti;      // which of the two partial buffers holds them
};

ClipEnc vit_enc(mmf_handle* h, int B) {
  Workspace& w = h->ws;
  const int M = B * 50;
  return ClipEnc{h->v_layers, 768, 3072, 12, w.v_x, h->opt.clip_res16 ? reinterpret_cast<f16_t*>(w.v_x) : nullptr,
                 w.v_xb, w.v_qkv, w.v_ctx, w.v_h, nullptr, 0, B, 50, M, nullptr, w.v_xc, w.v_ctxc, w.sk_vit,
                 w.sk_elems, w.v_st, clip_lazy(h, M), LnStats{w.v_st[0], 1, 768}, 0};
}
ClipEnc text_enc(mmf_handle* h, const int32_t* mask, int B, int L) {
  Workspace& w = h->ws;
  const int M = B * L;
  return ClipEnc{h->t_layers, 512, 2048, 8, w.t_x, h->opt.clip_res16 ? reinterpret_cast<f16_t*>(w.t_x) : nullptr,
                 w.t_xb, w.t_qkv, w.t_ctx, w.t_h, mask, 1, B, L, M, w.t_eos, w.t_xc, w.t_ctxc, w.sk_ctext,
                 w.sk_elems, w.t_st, clip_lazy(h, M), LnStats{w.t_st[0], 1, 512}, 0};
}

// the four GEMMs of a lazy-LN layer (not the last): QKV and FFN-1 read the raw stream with LN1 / LN2
// folded (consumers), out-proj and FFN-2 add into the stream and write its next partials (producers)
GemmArgs lazy_qkv(ClipEnc& E, int i) {
  const EncLayer& Ly = E.layers[i];
  GemmArgs g = ln_consumer(E.x16, E.H, Ly.qkv_f, Ly.qkv_u, E.cur, E.M);
  g.c16 = E.qkv;
  return g;
}
GemmArgs lazy_producer(mmf_handle* h, ClipEnc& E, const f16_t* A, int lda, const Lin16& l) {
  LnStats nxt;
  E.sti ^= 1;
  GemmArgs g = ln_producer(h->opt, A, lda, l, E.x16, E.M, E.st[E.sti], &nxt);
  E.cur = nxt;
  return g;
}
GemmArgs lazy_o(mmf_handle* h, ClipEnc& E, int i) { return lazy_producer(h, E, E.ctx, E.H, E.layers[i].o); }
GemmArgs lazy_fc1(ClipEnc& E, int i) {
  const EncLayer& Ly = E.layers[i];
  GemmArgs g = ln_consumer(E.x16, E.H, Ly.fc1_f, Ly.fc1_u, E.cur, E.M);
  g.act = 2;  // quick_gelu
  g.c16 = E.hid;
  return g;
}
GemmArgs lazy_fc2(mmf_handle* h, ClipEnc& E, int i) { return lazy_producer(h, E, E.hid, E.I, E.layers[i].fc2); }

int clip_attn(mmf_handle* h, const ClipEnc& E, hipStream_t s) {
  return attn(h, E.qkv, 3 * E.H, E.mask, E.ctx, E.H, E.B, E.L, E.heads, E.causal, s);
}

// pre-LN CLIP encoder layers [i0, i1) over E.x (residual stream, in place: fp32, or fp16 when
// opt.clip_res16) with xb = LN1_0(x) already computed (materialised mode) or its statistics in
// st[0] (lazy mode)
int run_clip_encoder(mmf_handle* h, ClipEnc& E, int i0, int i1, hipStream_t s) {
  const int M = E.M, H = E.H, I = E.I, B = E.B, L = E.L, heads = E.heads;
  float* const x = E.x;
  f16_t* const x16 = E.x16;
  f16_t *const xb = E.xb, *const qkv = E.qkv, *const ctx = E.ctx, *const hid = E.hid;
  float* const xc = E.xc;
  f16_t* const ctxc = E.ctxc;
  float* const skws = E.skws;
  const size_t sk_elems = E.sk_elems;
  const int32_t* const mask = E.mask;
  const int32_t* const last_rows = E.last_rows;
  const int causal = E.causal;
  EncLayer* const layers = E.layers;
  // lazy LN (gemm.hip; the caller's embedding wrote st[0] with the stream's statistics): the QKV /
  // FFN-1 GEMMs read the raw stream x16 with LN1 / LN2 folded, out-proj / FFN-2 add into it
  const bool lazy = E.lazy;
  for (int i = i0; i < i1; ++i) {
    const EncLayer& Ly = layers[i];
    GemmArgs g;
    if (i == 11 && (h->opt.last_q1 & 2)) {
      // only the pooled rows' queries are needed in the last layer: their stream rows -> xc (fp32,
      // also the residual below), LN1 -> Q (skinny GEMM on the unfolded weights), K and V of every
      // row (the fused weight's rows H..3H; lazy consumer or materialised), one query per
      // (sequence, head) straight into the compact ctxc
      HIPCHK(launch_gather_rows2(nullptr, x16 ? nullptr : x, x16, last_rows, L, H, nullptr, xc, B, s));
      f16_t* xq = hid;                   // hid ([M][I] fp16) is free until FFN-1
      float* qc = reinterpret_cast<float*>(hid + (size_t)B * H);  // fp32 queries
      CHK(lnorm(h, xc, H, Ly.ln1, nullptr, 0, xq, H, B, H, s));
      Lin16 qq = Ly.qkv;
      qq.out = H;
      g = with_ws(gemm_args(xq, H, qq, B), skws, sk_elems);
      g.c32 = qc;
      CHK(gemm(h, g, s));
      if (lazy) {
        Lin16 kvf = Ly.qkv_f;
        kvf.w += (size_t)H * H;
        kvf.b += H;  // (c and u are padded by 256 past 3H: the 256-column DMA stays in bounds)
        kvf.out = 2 * H;
        g = ln_consumer(x16, H, kvf, Ly.qkv_u + H, E.cur, M);
      } else {
        Lin16 kv = Ly.qkv;
        kv.w += (size_t)H * H;
        kv.b += H;
        kv.out = 2 * H;
        g = with_ws(gemm_args(xb, H, kv, M), skws, sk_elems);
      }
      g.c16 = qkv + H;
      g.ldc = 3 * H;
      CHK(gemm(h, g, s));
      {
        ProfScope ps(h, s, PK_ATTN, 4.0 * B * heads * (double)L * 64, (double)B * L * H * 2 * 2);
        HIPCHK(launch_attention_q1(qc, H, qkv, 3 * H, H, 2 * H, mask, causal ? last_rows : nullptr, ctxc, H, B, L,
                                   heads, s));
      }
    } else {
      g = lazy ? lazy_qkv(E, i) : with_ws(gemm_args(xb, H, Ly.qkv, M), skws, sk_elems);
      if (!lazy) g.c16 = qkv;
      CHK(gemm(h, g, s));
      CHK(clip_attn(h, E, s));
    }
    if (i == 11) {
      if (!(h->opt.last_q1 & 2)) HIPCHK(launch_gather_rows2(ctx, x16 ? nullptr : x, x16, last_rows, L, H, ctxc, xc, B, s));
      g = with_ws(gemm_args(ctxc, H, Ly.o, B), skws, sk_elems);
      g.res32 = xc;
      g.c32 = xc;
      CHK(gemm(h, g, s));
      CHK(lnorm(h, xc, H, Ly.ln2, nullptr, 0, xb, H, B, H, s));
      g = with_ws(gemm_args(xb, H, Ly.fc1, B), skws, sk_elems);
      g.act = 2;  // quick_gelu
      g.c16 = hid;
      CHK(gemm(h, g, s));
      g = with_ws(gemm_args(hid, I, Ly.fc2, B), skws, sk_elems);
      g.res32 = xc;
      g.c32 = xc;
      CHK(gemm(h, g, s));
      break;
    }
    if (lazy) {
      CHK(gemm(h, lazy_o(h, E, i), s));
      CHK(gemm(h, lazy_fc1(E, i), s));
      CHK(gemm(h, lazy_fc2(h, E, i), s));
      continue;
    }
    // out-proj / FFN-2 write their fp16 branch output y (out-proj into `hid`, free until FFN-1;
    // FFN-2 into `ctx`, free after out-proj); add+LN adds it to the fp32 residual stream x in place
    // (skinny M <= 512: split-K through the tower's workspace, gemm_splitk_factor)
    g = with_ws(gemm_args(ctx, H, Ly.o, M), skws, sk_elems);
    g.c16 = hid;
    CHK(gemm(h, g, s));
    CHK(x16 ? add_ln(h, x16, H, hid, H, Ly.ln2, xb, H, M, H, s)
            : add_ln(h, x, H, hid, H, Ly.ln2, x, nullptr, xb, H, M, H, s));
    g = with_ws(gemm_args(xb, H, Ly.fc1, M), skws, sk_elems);
    g.act = 2;  // quick_gelu
    g.c16 = hid;
    CHK(gemm(h, g, s));
    g = with_ws(gemm_args(hid, I, Ly.fc2, M), skws, sk_elems);
    g.c16 = ctx;
    CHK(gemm(h, g, s));
    // layer i + 1 < 12 always holds here (layer 11 takes the compact branch above)
    CHK(x16 ? add_ln(h, x16, H, ctx, H, layers[i + 1].ln1, xb, H, M, H, s)
            : add_ln(h, x, H, ctx, H, layers[i + 1].ln1, x, nullptr, xb, H, M, H, s));
  }
  return 0;
}

int clip_image_embed(mmf_handle* h, const uint8_t* img, int B, hipStream_t s) {
  Workspace& w = h->ws;
  {
    ProfScope ps(h, s, PK_IM2COL, 2.0 * B * 49 * 3072, (double)B * 49 * 3072 * (1 + 2));
    HIPCHK(launch_clip_im2col(img, w.v_col, B, s));
  }
  Lin16 pe;
  pe.w = h->v_patch_w;
  pe.out = 768;
  pe.in = 3072;
  GemmArgs g = gemm_args(w.v_col, 3072, pe, B * 49);
  g.c32 = w.v_patch;
  CHK(gemm(h, g, s));
  ProfScope ps(h, s, PK_EMBED, 16.0 * B * 50 * 768, (double)B * 50 * 768 * (4 + 4 + 2));
  HIPCHK(launch_clip_vision_assemble(w.v_patch, h->v_cls, h->v_pos, h->v_pre.g, h->v_pre.b, h->v_layers[0].ln1.g,
                                     h->v_layers[0].ln1.b, 1e-5f, h->opt.clip_res16 ? nullptr : w.v_x,
                                     h->opt.clip_res16 ? reinterpret_cast<f16_t*>(w.v_x) : nullptr, w.v_xb,
                                     clip_lazy(h, B * 50) ? w.v_st[0] : nullptr, B, s));
  return 0;
}

int clip_image_tail(mmf_handle* h, int B, float* emb, hipStream_t s) {
  Workspace& w = h->ws;
  HIPCHK(launch_gather_ln(w.v_xc, nullptr, 1, h->v_post.g, h->v_post.b, 1e-5f, w.v_cls, nullptr, B, 768, s));
  Lin16 pj;
  pj.w = h->v_proj;
  pj.out = 512;
  pj.in = 768;
  GemmArgs g = with_ws(gemm_args(w.v_cls, 768, pj, B), w.sk_vit, w.sk_elems);
  g.c32 = emb;
  CHK(gemm(h, g, s));
  HIPCHK(launch_l2norm(emb, B, 512, s));
  return 0;
}

int run_clip_image(mmf_handle* h, const uint8_t* img, int B, float* emb, hipStream_t s) {
  CHK(clip_image_embed(h, img, B, s));
  ClipEnc E = vit_enc(h, B);
  CHK(run_clip_encoder(h, E, 0, 12, s));
  return clip_image_tail(h, B, emb, s);
}

int clip_text_embed(mmf_handle* h, const int32_t* ids, int B, int L, hipStream_t s) {
  Workspace& w = h->ws;
  {
    ProfScope ps(h, s, PK_EMBED, 10.0 * B * L * 512, (double)B * L * 512 * (4 + 4 + 4 + 2));
    HIPCHK(launch_clip_text_embed(ids, h->t_tok, h->t_pos, h->t_layers[0].ln1.g, h->t_layers[0].ln1.b, 1e-5f,
                                  h->opt.clip_res16 ? nullptr : w.t_x,
                                  h->opt.clip_res16 ? reinterpret_cast<f16_t*>(w.t_x) : nullptr, w.t_xb,
                                  clip_lazy(h, B * L) ? w.t_st[0] : nullptr, B, L, 512, s));
  }
  HIPCHK(launch_eos_index(ids, w.t_eos, B, L, h->eos_id, s));
  return 0;
}

int clip_text_tail(mmf_handle* h, int B, float* emb, hipStream_t s) {
  Workspace& w = h->ws;
  HIPCHK(launch_gather_ln(w.t_xc, nullptr, 1, h->t_final.g, h->t_final.b, 1e-5f, w.t_pool, nullptr, B, 512, s));
  Lin16 pj;
  pj.w = h->t_proj;
  pj.out = 512;
  pj.in = 512;
  GemmArgs g = with_ws(gemm_args(w.t_pool, 512, pj, B), w.sk_ctext, w.sk_elems);
  g.c32 = emb;
  CHK(gemm(h, g, s));
  HIPCHK(launch_l2norm(emb, B, 512, s));
  return 0;
}

int run_clip_text(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* emb, hipStream_t s) {
  CHK(clip_text_embed(h, ids, B, L, s));
  ClipEnc E = text_enc(h, mask, B, L);
  CHK(run_clip_encoder(h, E, 0, 12, s));
  return clip_text_tail(h, B, emb, s);
}

// EfficientNet-B0 activation elements per image: block input/output, expanded, depthwise output,
// SE pool partials (nchunks x channels) maxima over the network
struct EffSizes { size_t io, exp, dw, pool; };
EffSizes eff_sizes() {
  EffSizes z{(size_t)112 * 112 * 32, 0, 0, 0};
  int H = 112;
  for (int si = 0; si < 7; ++si)
    for (int j = 0; j < kStages[si][5]; ++j) {
      const int e = kStages[si][0], st = j == 0 ? kStages[si][2] : 1;
      const int cin = j == 0 ? kStages[si][3] : kStages[si][4], cout = kStages[si][4], cexp = cin * e;
      const int Ho = (H - 1) / st + 1;
      z.exp = std::max(z.exp, (size_t)H * H * cexp);
      z.dw = std::max(z.dw, (size_t)Ho * Ho * cexp);
      z.io = std::max(z.io, (size_t)Ho * Ho * cout);
      z.pool = std::max(z.pool, (size_t)dwconv_nchunks(H, H, cexp, st) * cexp);
      H = Ho;
    }
  z.exp = std::max(z.exp, (size_t)7 * 7 * 1280);
  return z;
}

// The fp32 tower (option effnet_fp32): same network, same folded weights (fp32 copies of the 1x1
// convs), activations fp32 throughout -- no fusion, one launch per layer.
int run_effnet32(mmf_handle* h, const uint8_t* img, const float* xf32, int B, float* logits, float* score,
                 int score_stride, hipStream_t s, int img0 = 0) {
  Workspace& w = h->ws;
  if (w.e32_cap_b < img0 + B) return fail(MMF_EINVAL, "effnet_fp32: fp32 tower workspaces not reserved");
  // a chunk starting at image img0 works in its own slice of every workspace (mmf_effnet_forward)
  const EffSizes es = eff_sizes();
  const size_t b0 = (size_t)img0;
  float* const e32_exp = w.e32_exp + b0 * es.exp;
  float* const e32_dw = w.e32_dw + b0 * es.dw;
  float* const e_pool = w.e_pool + b0 * es.pool;
  float* const e_scale = w.e_scale + b0 * 1280;
  float* cur = w.e32_a + b0 * es.io;
  float* nxt = w.e32_b + b0 * es.io;
  {
    ProfScope ps(h, s, PK_STEM, 2.0 * B * 112 * 112 * 32 * 27, (double)B * (224 * 224 * 3 + 112 * 112 * 32 * 4));
    HIPCHK(launch_effnet_stem32(img, xf32, h->e_stem_w, h->e_stem_b, cur, B, s));
  }
  int H = 112, W = 112;
  for (const EffBlock& b : h->e_blocks) {
    const int Ho = (H - 1) / b.stride + 1, Wo = (W - 1) / b.stride + 1;
    const float* src = cur;
    if (b.expand != 1) {
      ProfScope ps(h, s, PK_PW32, 2.0 * B * H * W * b.cin * b.cexp, 4.0 * B * H * W * (b.cin + b.cexp));
      HIPCHK(launch_pw32(cur, b.e.w32, b.e.b, nullptr, 1, nullptr, e32_exp, B * H * W, b.cexp, b.cin, 3 /* SiLU */, s,
                             h->opt.pw32_mfma));
      src = e32_exp;
    }
    {
      ProfScope ps(h, s, PK_DW, 2.0 * B * Ho * Wo * b.cexp * b.k * b.k, 4.0 * B * b.cexp * ((double)H * W + Ho * Wo));
      HIPCHK(launch_dw32(src, b.wd_t, b.bd, e32_dw, B, H, W, b.cexp, b.k, b.stride, s));
    }
    {
      ProfScope ps(h, s, PK_SE, 4.0 * B * b.cexp * b.csq, 4.0 * B * b.cexp * ((double)Ho * Wo + 2));
      // as many pool chunks as the fp16 tower uses for this layer (fits e_pool by construction)
      const int nch = std::min(dwconv_nchunks(H, W, b.cexp, b.stride), Ho * Wo);
      HIPCHK(launch_sum32(e32_dw, B, Ho * Wo, b.cexp, nch, e_pool, s));
      HIPCHK(launch_se(e_pool, nch, 1.0f / (float)(Ho * Wo), b.w1, b.b1, b.w2, b.b2, e_scale, B, b.cexp, b.csq, s,
                       true));
    }
    {
      ProfScope ps(h, s, PK_PW32, 2.0 * B * Ho * Wo * b.cexp * b.cout,
                   4.0 * B * Ho * Wo * (b.cexp + b.cout * (b.residual ? 2 : 1)));
      HIPCHK(launch_pw32(e32_dw, b.p.w32, b.p.b, e_scale, Ho * Wo, b.residual ? cur : nullptr, nxt, B * Ho * Wo,
                         b.cout, b.cexp, 0, s, h->opt.pw32_mfma));
    }
    std::swap(cur, nxt);
    H = Ho;
    W = Wo;
  }
  {
    ProfScope ps(h, s, PK_PW32, 2.0 * B * H * W * 320 * 1280, 4.0 * B * H * W * (320 + 1280));
    HIPCHK(launch_pw32(cur, h->e_head.w32, h->e_head.b, nullptr, 1, nullptr, e32_exp, B * H * W, 1280, 320, 3, s,
                       h->opt.pw32_mfma));
  }
  ProfScope ps(h, s, PK_GAP, (double)B * H * W * 1280 + 4.0 * B * 1280, (double)B * H * W * 1280 * 4);
  HIPCHK(launch_gap32(e32_exp, H * W, 1280, h->e_cls_w, h->e_cls_b, logits, score, score_stride, B, s));
  return 0;
}

// The EfficientNet activation workspaces hold max_batch images at the largest per-image size of each
// buffer; a batch chunk that starts at image b0 works in the disjoint slice b0 * (per-image max) on,
// so chunks of one batch can run concurrently on different streams (mmf_effnet_forward).
struct EffWs {
  f16_t *e_a, *e_b, *e_exp, *e_dw;
  float *e_pool, *e_scale;
};
EffWs eff_ws(mmf_handle* h, int b0) {
  const Workspace& w = h->ws;
  const EffSizes es = eff_sizes();
  const size_t b = (size_t)b0;
  return EffWs{w.e_a + b * es.io, w.e_b + b * es.io, w.e_exp + b * es.exp, w.e_dw + b * es.dw,
               w.e_pool + b * es.pool, w.e_scale + b * 1280};
}

int run_effnet(mmf_handle* h, const uint8_t* img, const float* xf32, int B, float* logits, float* score, int score_stride,
               hipStream_t s, int img0 = 0) {
  if (h->opt.effnet_fp32) return run_effnet32(h, img, xf32, B, logits, score, score_stride, s, img0);
  const EffWs w = eff_ws(h, img0);
  f16_t* cur = w.e_a;
  f16_t* nxt = w.e_b;
  // option fuse_stem = 0: separate stem launch + stage-1 depthwise (A/B and parity tests)
  const EffBlock& b0 = h->e_blocks.front();
  const bool fuse_stem = h->opt.fuse_stem && b0.expand == 1 && b0.cexp == 32 && b0.k == 3 && b0.stride == 1;
  if (!fuse_stem) {
    ProfScope ps(h, s, PK_STEM, 2.0 * B * 112 * 112 * 32 * 27, (double)B * (224 * 224 * 3 + 112 * 112 * 32 * 2));
    if (xf32) HIPCHK(launch_effnet_stem_f32(xf32, h->e_stem_w, h->e_stem_b, cur, B, s));
    else HIPCHK(launch_effnet_stem(img, h->e_stem_w, h->e_stem_b, cur, B, s));
  }
  int H = 112, W = 112;
  for (const EffBlock& b : h->e_blocks) {
    const f16_t* src = cur;
    int nch = 0;
    const int Ho = (H - 1) / b.stride + 1, Wo = (W - 1) / b.stride + 1;
    // option fuse_expand = 0: separate expand launch (A/B)
    const bool fuse = b.expand != 1 && h->opt.fuse_expand && expand_dw_applicable(b.cin, b.cexp, b.k);
    if (&b == &b0 && fuse_stem) {
      // stem output recomputed per 18x18 halo tile: 1.27x the stem MACs, image patch read once
      ProfScope ps(h, s, PK_DW, 2.0 * B * 112 * 112 * 32 * (9 + 27 * 1.27),
                   (double)B * (224 * 224 * 3 * 1.34 + 112 * 112 * 32 * 2));
      HIPCHK(launch_effnet_stem_dw(img, xf32, h->e_stem_w, h->e_stem_b, b.wd, b.bd, w.e_dw, w.e_pool, B, &nch, s));
    } else if (fuse) {
      ProfScope ps(h, s, PK_DW, 2.0 * B * Ho * Wo * b.cexp * b.k * b.k + 2.0 * B * H * W * b.cin * b.cexp,
                   (double)B * 2 * ((double)H * W * b.cin * (b.cexp / 48) + (double)Ho * Wo * b.cexp));
      HIPCHK(launch_expand_dw(cur, b.cin, b.e.w, b.e.b, b.wd, b.bd, w.e_dw, w.e_pool, B, H, W, b.cexp, b.k, b.stride,
                              &nch, s));
    } else if (b.expand != 1) {
      GemmArgs g = gemm_args(cur, b.cin, b.e, B * H * W);
      g.act = 3;  // SiLU
      g.c16 = w.e_exp;
      CHK(gemm(h, g, s));
      src = w.e_exp;
    }
    if (!fuse && !(&b == &b0 && fuse_stem)) {
      ProfScope ps(h, s, PK_DW, 2.0 * B * Ho * Wo * b.cexp * b.k * b.k,
                   (double)B * b.cexp * 2 * ((double)H * W + (double)Ho * Wo));
      HIPCHK(launch_dwconv(src, b.wd, b.bd, w.e_dw, w.e_pool, B, H, W, b.cexp, b.k, b.stride, &nch, s,
                            1 | (h->opt.dw_cw32 ? 8 : 0)));
    }
    ProfScope ps(h, s, PK_SE, 4.0 * B * b.cexp * b.csq, (double)B * b.cexp * 4 * (nch + 1));
    HIPCHK(launch_se(w.e_pool, nch, 1.0f / (float)(Ho * Wo), b.w1, b.b1, b.w2, b.b2, w.e_scale, B, b.cexp, b.csq, s));
    GemmArgs g = gemm_args(w.e_dw, b.cexp, b.p, B * Ho * Wo);
    g.ascale = w.e_scale;
    g.rows_per_batch = Ho * Wo;
    if (b.residual) g.res16 = cur;
    g.c16 = nxt;
    CHK(gemm(h, g, s));
    f16_t* t = cur;
    cur = nxt;
    nxt = t;
    H = Ho;
    W = Wo;
  }
  GemmArgs g = gemm_args(cur, 320, h->e_head, B * H * W);
  g.act = 3;
  g.c16 = w.e_exp;
  CHK(gemm(h, g, s));
  ProfScope ps(h, s, PK_GAP, (double)B * H * W * 1280 + 4.0 * B * 1280, (double)B * H * W * 1280 * 2);
  HIPCHK(launch_gap_classifier(w.e_exp, H * W, 1280, h->e_cls_w, h->e_cls_b, logits, score, score_stride, B, s));
  return 0;
}

// fork/join streams of the multi-tower entry points, created on first use
int ensure_towers(mmf_handle* h) {
  if (h->tower[0]) return 0;
  for (int i = 0; i < 3; ++i) {
    HIPCHK(hipStreamCreateWithFlags(&h->tower[i], hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&h->join_ev[i], hipEventDisableTiming));
  }
  HIPCHK(hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->text_ev, hipEventDisableTiming));
  return 0;
}

// after the towers joined: CLIP cosine, vault top-5, fusion (mmf_analyze_batch's last part)
int analyze_tail(mmf_handle* h, int B, float* scores5, float* text_sim, float* probs2, int32_t* verdict, float* conf,
                 int32_t* rule, float* top_sims, int32_t* top_idx, hipStream_t s) {
  Workspace& w = h->ws;
  HIPCHK(launch_rowdot(w.v_emb, w.t_emb, scores5 + 3, 5, B, 512, s));
  if (h->ready & 32) {
    ProfScope ps(h, s, PK_VAULT, 2.0 * B * h->vault_n * 512, (double)h->vault_n * 512 * 4 + (double)B * h->vault_n * 8);
    HIPCHK(launch_vault_sims(w.v_emb, h->vault, w.s_sims, B, h->vault_n, 512, s, h->opt.vault_ref));
    HIPCHK(launch_vault_topk(w.s_sims, B, h->vault_n, 5, 0.85f, top_sims, top_idx, scores5 + 4, 5, w.t_emb,
                             h->vault_title, 512, text_sim, s, h->opt.vault_ref));
  } else {
    HIPCHK(launch_fill_strided(scores5 + 4, 5, B, 0.f, s));
    if (text_sim) HIPCHK(hipMemsetAsync(text_sim, 0, (size_t)B * 4, s));
    if (top_sims) HIPCHK(hipMemsetAsync(top_sims, 0, (size_t)B * 5 * 4, s));
    if (top_idx) HIPCHK(hipMemsetAsync(top_idx, 0xff, (size_t)B * 5 * 4, s));
  }
  ProfScope ps(h, s, PK_FUSION, 2.0 * B * (5 * 64 + 64 * 32 + 32 * 2), (double)B * (5 + 2 + 3) * 4);
  HIPCHK(launch_fusion(scores5, h->f_w0, h->f_b0, h->f_w3, h->f_b3, h->f_w5, h->f_b5, probs2, verdict, conf, rule, B,
                       s));
  return 0;
}


// Workspaces of the precision modes, allocated while the mode is selected and freed when it is left
// (mmf_reserve, mmf_set_option, mmf_finalize) -- never from inside a launch sequence, which worker
// threads may be enqueueing (option mt_enqueue): the fp32 EfficientNet tower (effnet_fp32, ~10 MB per
// image) and the RoBERTa precise mode (text_hilo = 2, 40 KB per token row).
int ensure_mode_ws(mmf_handle* h) {
  if (!h->cap_b) return 0;
  Workspace& w = h->ws;
  const size_t rows = (size_t)h->cap_b * h->cap_lr;
  void* p;
  if (text_mode(h) >= 2) {
    if (w.t32_rows < rows) {
      CHK(free_group(h, AG_TEXT32));
      CHK(dev_alloc(h, &p, rows * 3072 * 4, AG_TEXT32)); w.p32 = (float*)p;
      CHK(dev_alloc(h, &p, rows * 2304 * 2, AG_TEXT32)); w.s3 = (f16_t*)p;
      CHK(dev_alloc(h, &p, rows * 9216 * 2, AG_TEXT32)); w.h3 = (f16_t*)p;
      w.t32_rows = rows;
    }
  } else if (w.t32_rows) {
    CHK(free_group(h, AG_TEXT32));
    w.p32 = nullptr;
    w.s3 = w.h3 = nullptr;
    w.t32_rows = 0;
  }
  if (h->opt.effnet_fp32) {
    if (w.e32_cap_b < h->cap_b) {
      CHK(free_group(h, AG_EFF32));
      const EffSizes es = eff_sizes();
      const size_t nb = (size_t)h->cap_b * 4;
      CHK(dev_alloc(h, &p, nb * es.io, AG_EFF32)); w.e32_a = (float*)p;
      CHK(dev_alloc(h, &p, nb * es.io, AG_EFF32)); w.e32_b = (float*)p;
      CHK(dev_alloc(h, &p, nb * es.exp, AG_EFF32)); w.e32_exp = (float*)p;
      CHK(dev_alloc(h, &p, nb * es.dw, AG_EFF32)); w.e32_dw = (float*)p;
      w.e32_cap_b = h->cap_b;
    }
  } else if (w.e32_cap_b) {
    CHK(free_group(h, AG_EFF32));
    w.e32_a = w.e32_b = w.e32_exp = w.e32_dw = nullptr;
    w.e32_cap_b = 0;
  }
  return 0;
}

int ensure_sims(mmf_handle* h) {
  if (!h->vault_n || !h->cap_b) return 0;
  if (h->ws.s_cap_n >= h->vault_n) return 0;
  CHK(free_group(h, AG_SIMS));
  void* p;
  CHK(dev_alloc(h, &p, (size_t)h->cap_b * h->vault_n * sizeof(float), AG_SIMS));
  h->ws.s_sims = (float*)p;
  h->ws.s_cap_n = h->vault_n;
  return 0;
}

}  // namespace

// =============================================================================================
extern "C" {

const char* mmf_last_error(void) { return g_err.c_str(); }
const char* mmf_version(void) { return "mmf_hip 0.1.0 gfx950"; }

int mmf_create(int device, mmf_handle** out) {
  if (!out) return fail(MMF_EINVAL, "out is NULL");
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(MMF_EINVAL, "device %d out of range (%d devices)", device, n);
  HIPCHK(hipSetDevice(device));
  mmf_handle* h = new (std::nothrow) mmf_handle();
  if (!h) return fail(MMF_ENOMEM, "out of host memory");
  h->device = device;
  h->opt = process_options();
  *out = h;
  g_err.clear();
  return 0;
}

void mmf_destroy(mmf_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  delete h;
}

int mmf_load_tensor(mmf_handle* h, const char* name, int dtype, int ndim, const int64_t* shape, const void* data) {
  if (!h || !name || (!data && ndim > 0) || ndim < 0 || ndim > 8) return fail(MMF_EINVAL, "bad argument");
  HostT t;
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    if (shape[i] < 0) return fail(MMF_EINVAL, "negative dim in '%s'", name);
    t.shape.push_back(shape[i]);
    n *= (size_t)shape[i];
  }
  if (dtype == MMF_DTYPE_I64) return 0;  // integer buffers (num_batches_tracked) carry no arithmetic
  if (dtype != MMF_DTYPE_F32) return fail(MMF_EINVAL, "unsupported dtype %d for '%s'", dtype, name);
  t.f.resize(n);
  if (n) std::memcpy(t.f.data(), data, n * sizeof(float));
  h->staged[name] = std::move(t);
  return 0;
}

int mmf_finalize(mmf_handle* h, int clip_eos_token_id) {
  if (!h) return fail(MMF_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  h->eos_id = clip_eos_token_id;
  int ready = h->ready;  // incremental: components not re-staged keep their packed weights
  std::string missing;
  // a re-staged component replaces its packed weights: its previous buffers are freed first
  auto attempt = [&](int bit, int group, const char* key, int (*fn)(mmf_handle*)) -> int {
    if (!has(h, key)) return 0;
    ready &= ~bit;
    h->ready = ready;
    CHK(free_group(h, group));
    h->cur_group = group;
    int r = fn(h);
    if (r) return r;
    ready |= bit;
    return 0;
  };
  CHK(attempt(1, AG_TEXT, "roberta.embeddings.word_embeddings.weight", finalize_text));
  CHK(attempt(2, AG_EFF, "efficientnet.features.0.0.weight", finalize_effnet));
  CHK(attempt(4, AG_VIS, "clip.vision_model.embeddings.patch_embedding.weight", finalize_clip_vision));
  CHK(attempt(8, AG_CTEXT, "clip.text_model.embeddings.token_embedding.weight", finalize_clip_text));
  CHK(attempt(16, AG_FUSION, "fusion_layer.0.weight", finalize_fusion));
  h->ready = ready;
  h->staged.clear();
  HIPCHK(hipDeviceSynchronize());
  return ensure_mode_ws(h);
}

int mmf_ready(mmf_handle* h) { return h ? h->ready : 0; }

int mmf_reserve(mmf_handle* h, int B, int Lr, int Lc) {
  if (!h || B <= 0 || Lr <= 0 || Lr > 512 || Lc <= 0 || Lc > 77)
    return fail(MMF_EINVAL, "mmf_reserve: bad shape B=%d Lr=%d Lc=%d", B, Lr, Lc);
  HIPCHK(hipSetDevice(h->device));
  CHK(free_group(h, AG_WS));
  CHK(free_group(h, AG_SIMS));
  CHK(free_group(h, AG_EFF32));
  CHK(free_group(h, AG_TEXT32));
  h->ws = Workspace();
  h->cap_b = h->cap_lr = h->cap_lc = 0;
  Workspace& w = h->ws;
  auto A = [&](void** p, size_t bytes) { return dev_alloc(h, p, bytes, AG_WS); };
  const size_t Mr = (size_t)B * Lr, Mv = (size_t)B * 50, Mt = (size_t)B * Lc;
  CHK(A((void**)&w.r_x, Mr * 768 * 4));
  CHK(A((void**)&w.r_y, Mr * 768 * 4));
  CHK(A((void**)&w.r_xb, Mr * 768 * 2));
  CHK(A((void**)&w.r_lo, Mr * 768 * 2));
  CHK(A((void**)&w.r_ovf, (size_t)B * 4));
  CHK(A((void**)&w.r_qkv, Mr * 2304 * 2));
  CHK(A((void**)&w.r_ctx, Mr * 768 * 2));
  CHK(A((void**)&w.r_h, Mr * 3072 * 2));
  CHK(A((void**)&w.v_col, (size_t)B * 49 * 3072 * 2));
  CHK(A((void**)&w.v_patch, (size_t)B * 49 * 768 * 4));
  CHK(A((void**)&w.v_x, Mv * 768 * 4));
  CHK(A((void**)&w.v_xb, Mv * 768 * 2));
  CHK(A((void**)&w.v_qkv, Mv * 2304 * 2));
  CHK(A((void**)&w.v_ctx, Mv * 768 * 2));
  CHK(A((void**)&w.v_h, Mv * 3072 * 2));
  CHK(A((void**)&w.v_cls, (size_t)B * 768 * 2));
  CHK(A((void**)&w.v_emb, (size_t)B * 512 * 4));
  CHK(A((void**)&w.t_x, Mt * 512 * 4));
  CHK(A((void**)&w.t_xb, Mt * 512 * 2));
  CHK(A((void**)&w.t_qkv, Mt * 1536 * 2));
  CHK(A((void**)&w.t_ctx, Mt * 512 * 2));
  CHK(A((void**)&w.t_h, Mt * 2048 * 2));
  CHK(A((void**)&w.t_pool, (size_t)B * 512 * 2));
  CHK(A((void**)&w.t_emb, (size_t)B * 512 * 4));
  CHK(A((void**)&w.t_eos, (size_t)B * 4));
  CHK(A((void**)&w.v_xc, (size_t)B * 768 * 4));
  CHK(A((void**)&w.v_ctxc, (size_t)B * 768 * 2));
  CHK(A((void**)&w.t_xc, (size_t)B * 512 * 4));
  CHK(A((void**)&w.t_ctxc, (size_t)B * 512 * 2));
  {
    auto stats_rows = [](size_t rows) { return (rows + 255) / 256 * 256 * kLnP * sizeof(float2); };
    for (int i = 0; i < 2; ++i) {
      CHK(A((void**)&w.v_st[i], stats_rows(Mv)));
      CHK(A((void**)&w.t_st[i], stats_rows(Mt)));
    }
  }
  // max over the skinny-M GEMMs (compact last layers: B rows; whole encoders of small batches: up to
  // the 512 rows gemm_config sends to the split-K path) of (K / 256) * N = 9216 per row
  w.sk_elems = (size_t)std::max(B, 512) * 9216;
  for (float** sk : {&w.sk_text, &w.sk_vit, &w.sk_ctext}) CHK(A((void**)sk, w.sk_elems * 4));
  // EfficientNet activation sizes per image
  const EffSizes es = eff_sizes();
  const size_t max_io = es.io, max_exp = es.exp, max_dw = es.dw, max_pool = es.pool, max_c = 1280;
  CHK(A((void**)&w.e_a, (size_t)B * max_io * 2));
  CHK(A((void**)&w.e_b, (size_t)B * max_io * 2));
  CHK(A((void**)&w.e_exp, (size_t)B * max_exp * 2));
  CHK(A((void**)&w.e_dw, (size_t)B * max_dw * 2));
  CHK(A((void**)&w.e_pool, (size_t)B * max_pool * 4));
  CHK(A((void**)&w.e_scale, (size_t)B * max_c * 4));
  h->cap_b = B;
  h->cap_lr = Lr;
  h->cap_lc = Lc;
  CHK(ensure_sims(h));
  return ensure_mode_ws(h);
}

int mmf_text_forward(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* ai, float* mi,
                     float* scores2, void* stream) {
  if (!h || !ids || !mask) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 1)) return fail(MMF_EINVAL, "text model (RoBERTa + heads) not loaded");
  if (L > 512) return fail(MMF_EINVAL, "RoBERTa length %d > 512 (position table ends at 514)", L);
  CHK(check_cap(h, B, L, 1));
  HIPCHK(hipSetDevice(h->device));
  return run_text(h, ids, mask, B, L, ai, mi, scores2, 2, (hipStream_t)stream);
}

int mmf_effnet_forward(mmf_handle* h, const uint8_t* img, int B, float* logits, float* score, void* stream) {
  if (!h || !img) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 2)) return fail(MMF_EINVAL, "EfficientNet not loaded");
  CHK(check_cap(h, B, 1, 1));
  HIPCHK(hipSetDevice(h->device));
  const hipStream_t s = (hipStream_t)stream;
  // option effnet_chunks: the batch split into that many image chunks on concurrent streams (each
  // chunk's kernels fill the other's launch tails; per-image results are unchanged: every layer is
  // per image, and the GEMM rows do not depend on M)
  const int nc = std::min(std::max(h->opt.effnet_chunks, 1), 4);
  if (nc == 1 || B < 32 * nc) return run_effnet(h, img, nullptr, B, logits, score, 1, s);
  CHK(ensure_towers(h));
  HIPCHK(hipEventRecord(h->fork_ev, s));
  int b0 = 0;
  for (int c = 0; c < nc; ++c) {
    const int bc = B / nc + (c < B % nc ? 1 : 0);
    const hipStream_t cs = c ? h->tower[c - 1] : s;
    if (c) HIPCHK(hipStreamWaitEvent(cs, h->fork_ev, 0));
    CHK(run_effnet(h, img + (size_t)b0 * 224 * 224 * 3, nullptr, bc, logits ? logits + (size_t)b0 * 2 : nullptr,
                   score ? score + b0 : nullptr, 1, cs, b0));
    b0 += bc;
  }
  for (int c = 1; c < nc; ++c) {
    HIPCHK(hipEventRecord(h->join_ev[c - 1], h->tower[c - 1]));
    HIPCHK(hipStreamWaitEvent(s, h->join_ev[c - 1], 0));
  }
  return 0;
}

int mmf_effnet_forward_f32(mmf_handle* h, const float* x, int B, float* logits, float* score, void* stream) {
  if (!h || !x) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 2)) return fail(MMF_EINVAL, "EfficientNet not loaded");
  CHK(check_cap(h, B, 1, 1));
  HIPCHK(hipSetDevice(h->device));
  return run_effnet(h, nullptr, x, B, logits, score, 1, (hipStream_t)stream);
}

int mmf_clip_image(mmf_handle* h, const uint8_t* img, int B, float* emb, void* stream) {
  if (!h || !img || !emb) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 4)) return fail(MMF_EINVAL, "CLIP vision tower not loaded");
  CHK(check_cap(h, B, 1, 1));
  HIPCHK(hipSetDevice(h->device));
  return run_clip_image(h, img, B, emb, (hipStream_t)stream);
}

int mmf_clip_text(mmf_handle* h, const int32_t* ids, const int32_t* mask, int B, int L, float* emb, void* stream) {
  if (!h || !ids || !mask || !emb) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 8)) return fail(MMF_EINVAL, "CLIP text tower not loaded");
  if (L > 77) return fail(MMF_EINVAL, "CLIP text length %d > 77", L);
  CHK(check_cap(h, B, 1, L));
  HIPCHK(hipSetDevice(h->device));
  return run_clip_text(h, ids, mask, B, L, emb, (hipStream_t)stream);
}

namespace {
int set_vault_rows(mmf_handle* h, std::vector<float>& u, int N) {
  h->ready &= ~32;
  CHK(free_group(h, AG_TITLES));  // titles belong to the previous vault
  h->vault_title = nullptr;
  CHK(free_group(h, AG_VAULT));
  h->cur_group = AG_VAULT;
  CHK(up_f32(h, &h->vault, u));
  h->vault_n = N;
  h->ready |= 32;
  h->ws.s_cap_n = 0;
  return ensure_sims(h);
}
}  // namespace

int mmf_clip_consistency(mmf_handle* h, const uint8_t* img, const int32_t* ids, const int32_t* mask, int B, int L,
                         float* img_emb, float* txt_emb, float* sim, void* stream) {
  if (!h || !img || !ids || !mask || !sim) return fail(MMF_EINVAL, "null argument");
  if ((h->ready & 12) != 12) return fail(MMF_EINVAL, "CLIP towers not loaded");
  if (L > 77) return fail(MMF_EINVAL, "CLIP text length %d > 77", L);
  CHK(check_cap(h, B, 1, L));
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  float* ie = img_emb ? img_emb : h->ws.v_emb;
  float* te = txt_emb ? txt_emb : h->ws.t_emb;
  CHK(ensure_towers(h));
  const int concurrent = h->opt.concurrent && !h->prof;
  hipStream_t st = s;
  if (concurrent) {  // the text tower beside the vision tower (disjoint workspaces)
    HIPCHK(hipEventRecord(h->fork_ev, s));
    HIPCHK(hipStreamWaitEvent(h->tower[2], h->fork_ev, 0));
    st = h->tower[2];
  }
  if (concurrent && h->opt.mt_enqueue > 0 && B <= h->opt.mt_enqueue) {  // as in mmf_analyze_batch
    if (!h->pool) {
      h->pool.reset(new EnqueuePool());
      h->pool->start(h->device);
    }
    h->pool->submit(1, [=] { return run_clip_text(h, ids, mask, B, L, te, st); });
    const int rc = run_clip_image(h, img, B, ie, s);
    std::string e;
    const int wrc = h->pool->wait(1, &e);
    CHK(rc);
    if (wrc) return fail(wrc, "%s", e.c_str());
  } else {
    CHK(run_clip_text(h, ids, mask, B, L, te, st));
    CHK(run_clip_image(h, img, B, ie, s));
  }
  if (concurrent) {
    HIPCHK(hipEventRecord(h->join_ev[2], h->tower[2]));
    HIPCHK(hipStreamWaitEvent(s, h->join_ev[2], 0));
  }
  HIPCHK(launch_rowdot(ie, te, sim, 1, B, 512, s));
  return 0;
}

int mmf_set_vault(mmf_handle* h, const float* V, int N, int D) {
  if (!h || !V || N <= 0 || D != 512) return fail(MMF_EINVAL, "mmf_set_vault: need N > 0 rows of D = 512");
  HIPCHK(hipSetDevice(h->device));
  std::vector<float> u((size_t)N * D);
  for (int i = 0; i < N; ++i) {
    double s = 0;
    for (int d = 0; d < D; ++d) s += (double)V[(size_t)i * D + d] * V[(size_t)i * D + d];
    const float nrm = (float)std::sqrt(s);  // a zero row gives 0/0 = NaN, as numpy does
    for (int d = 0; d < D; ++d) u[(size_t)i * D + d] = V[(size_t)i * D + d] / nrm;
  }
  return set_vault_rows(h, u, N);
}

int mmf_set_vault_normalized(mmf_handle* h, const float* Vhat, int N, int D) {
  if (!h || !Vhat || N <= 0 || D != 512) return fail(MMF_EINVAL, "mmf_set_vault_normalized: need N > 0 rows of D = 512");
  HIPCHK(hipSetDevice(h->device));
  std::vector<float> u(Vhat, Vhat + (size_t)N * D);
  return set_vault_rows(h, u, N);
}

int mmf_set_vault_titles(mmf_handle* h, const int32_t* ids, const int32_t* mask, int N, int L, void* stream) {
  if (!h || !ids || !mask) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 32) || N != h->vault_n) return fail(MMF_EINVAL, "set the vault (N=%d) first", h->vault_n);
  if (!(h->ready & 8)) return fail(MMF_EINVAL, "CLIP text tower not loaded");
  if (L > h->cap_lc || h->cap_b <= 0) return fail(MMF_EINVAL, "reserve CLIP length >= %d first", L);
  HIPCHK(hipSetDevice(h->device));
  CHK(free_group(h, AG_TITLES));
  h->vault_title = nullptr;
  float* t;
  CHK(dev_alloc(h, (void**)&t, (size_t)N * 512 * 4, AG_TITLES));
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < N; i += h->cap_b) {
    const int n = std::min(h->cap_b, N - i);
    CHK(run_clip_text(h, ids + (size_t)i * L, mask + (size_t)i * L, n, L, t + (size_t)i * 512, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  h->vault_title = t;
  return 0;
}

int mmf_vault_topk(mmf_handle* h, const float* q, int B, int k, float thresh, float* sims, int32_t* idx, float* disc,
                   const float* temb, float* tsim, void* stream) {
  if (!h || !q) return fail(MMF_EINVAL, "null argument");
  if (!(h->ready & 32)) return fail(MMF_EINVAL, "vault not loaded");
  if (k < 1 || k > h->vault_n) return fail(MMF_EINVAL, "top_k must be in [1, N=%d]", h->vault_n);
  if (k > 8 && h->vault_n > 16384) return fail(MMF_EINVAL, "top_k > 8 needs a vault of <= 16384 rows");
  CHK(check_cap(h, B, 1, 1));
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(launch_vault_sims(q, h->vault, h->ws.s_sims, B, h->vault_n, 512, s, h->opt.vault_ref));
  HIPCHK(launch_vault_topk(h->ws.s_sims, B, h->vault_n, k, thresh, sims, idx, disc, 1, temb, h->vault_title, 512,
                           tsim, s, h->opt.vault_ref));
  return 0;
}

int mmf_fusion(mmf_handle* h, const float* x5, int B, float* probs, int32_t* verdict, float* conf, int32_t* rule,
               void* stream) {
  if (!h || !x5 || !probs || B <= 0) return fail(MMF_EINVAL, "bad argument");
  if (!(h->ready & 16)) return fail(MMF_EINVAL, "fusion layer not loaded");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(launch_fusion(x5, h->f_w0, h->f_b0, h->f_w3, h->f_b3, h->f_w5, h->f_b5, probs, verdict, conf, rule, B,
                       (hipStream_t)stream));
  return 0;
}

int mmf_analyze_batch(mmf_handle* h, const int32_t* rob_ids, const int32_t* rob_mask, int Lr, const int32_t* clip_ids,
                      const int32_t* clip_mask, int Lc, const uint8_t* img_eff, const uint8_t* img_clip, int B,
                      float* scores5, float* text_sim, float* probs2, int32_t* verdict, float* conf, int32_t* rule,
                      float* top_sims, int32_t* top_idx, void* stream) {
  if (!h || !rob_ids || !rob_mask || !clip_ids || !clip_mask || !img_eff || !scores5 || !probs2)
    return fail(MMF_EINVAL, "null argument");
  if ((h->ready & 31) != 31) return fail(MMF_EINVAL, "not all models loaded (ready mask %d)", h->ready);
  if (Lr > 512 || Lc > 77) return fail(MMF_EINVAL, "lengths Lr=%d (<=512) Lc=%d (<=77)", Lr, Lc);
  CHK(check_cap(h, B, Lr, Lc));
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  if (!img_clip) img_clip = img_eff;
  Workspace& w = h->ws;
  // the per-kernel profiling pass runs the towers sequentially so event intervals are clean
  const int concurrent = h->opt.concurrent && !h->prof;
  if (concurrent) CHK(ensure_towers(h));
  // fork: the four towers only share read-only inputs and write disjoint workspaces/outputs
  hipStream_t st_text = s, st_eff = s, st_ctxt = s;
  if (concurrent) {
    HIPCHK(hipEventRecord(h->fork_ev, s));
    for (int i = 0; i < 3; ++i) HIPCHK(hipStreamWaitEvent(h->tower[i], h->fork_ev, 0));
    st_text = h->tower[0];
    st_eff = h->tower[1];
    st_ctxt = h->tower[2];
  }
  // diag_skip (diagnostic only, never set by the API or bench.py): towers left out to measure each
  // tower's marginal cost in the concurrent step (bit 1 text, 2 EfficientNet, 4 CLIP text, 8 ViT)
  const int skip = h->opt.diag_skip;
  if (concurrent && h->opt.mt_enqueue > 0 && B <= h->opt.mt_enqueue) {
    // small batches: three host threads enqueue the text, CLIP-text and EfficientNet towers while
    // this thread enqueues the ViT, so every chain starts at once (each stream keeps its own order)
    if (!h->pool) {
      h->pool.reset(new EnqueuePool());
      h->pool->start(h->device);
    }
    float* t_emb = w.t_emb;
    const bool on[3] = {!(skip & 1), !(skip & 4), !(skip & 2)};
    if (on[0]) h->pool->submit(0, [=] { return run_text(h, rob_ids, rob_mask, B, Lr, nullptr, nullptr, scores5, 5, st_text); });
    if (on[1]) h->pool->submit(1, [=] { return run_clip_text(h, clip_ids, clip_mask, B, Lc, t_emb, st_ctxt); });
    if (on[2]) h->pool->submit(2, [=] { return run_effnet(h, img_eff, nullptr, B, nullptr, scores5 + 2, 5, st_eff, 0); });
    const int rc = (skip & 8) ? 0 : run_clip_image(h, img_clip, B, w.v_emb, s);
    int wrc = 0;
    std::string werr;
    for (int i = 0; i < 3; ++i) {
      if (!on[i]) continue;
      std::string e;
      const int r = h->pool->wait(i, &e);
      if (r && !wrc) {
        wrc = r;
        werr = e;
      }
    }
    CHK(rc);
    if (wrc) return fail(wrc, "%s", werr.c_str());
  } else {
    // option after_text: the chosen towers' streams wait for the RoBERTa tower (its persistent GEMMs
    // then own every CU instead of sharing them with the other towers' launches)
    // (releasing them before RoBERTa's last layer or two, and EfficientNet chained behind a CLIP tower or
    // split over two streams, measured slower: DESIGN.md §1 round 5)
    const int after = concurrent && !(skip & 1) ? h->opt.after_text : 0;
    if (!(skip & 1)) CHK(run_text(h, rob_ids, rob_mask, B, Lr, nullptr, nullptr, scores5, 5, st_text, after ? h->text_ev : nullptr));
    if (after) {
      if (after & 2) HIPCHK(hipStreamWaitEvent(st_eff, h->text_ev, 0));
      if (after & 4) HIPCHK(hipStreamWaitEvent(st_ctxt, h->text_ev, 0));
      if (after & 8) HIPCHK(hipStreamWaitEvent(s, h->text_ev, 0));
    }
    if (!(skip & 4)) CHK(run_clip_text(h, clip_ids, clip_mask, B, Lc, w.t_emb, st_ctxt));
    if (!(skip & 2)) CHK(run_effnet(h, img_eff, nullptr, B, nullptr, scores5 + 2, 5, st_eff));
    if (!(skip & 8)) CHK(run_clip_image(h, img_clip, B, w.v_emb, s));
  }
  if (concurrent) {
    for (int i = 0; i < 3; ++i) {
      HIPCHK(hipEventRecord(h->join_ev[i], h->tower[i]));
      HIPCHK(hipStreamWaitEvent(s, h->join_ev[i], 0));
    }
  }
  return analyze_tail(h, B, scores5, text_sim, probs2, verdict, conf, rule, top_sims, top_idx, s);
}

int mmf_profile_begin(mmf_handle* h) {
  if (!h) return fail(MMF_EINVAL, "null handle");
  h->prof = true;
  h->prof_recs.clear();
  h->ev_used = 0;
  return 0;
}

int mmf_profile_end(mmf_handle* h, int max_kinds, int* counts, double* ms, double* flops, double* bytes) {
  if (!h || max_kinds < PK_COUNT || !counts || !ms || !flops || !bytes)
    return fail(MMF_EINVAL, "mmf_profile_end needs arrays of >= %d kinds", (int)PK_COUNT);
  h->prof = false;
  for (int k = 0; k < max_kinds; ++k) {
    counts[k] = 0;
    ms[k] = flops[k] = bytes[k] = 0.0;
  }
  if (!h->prof_recs.empty()) HIPCHK(hipEventSynchronize(h->ev_pool[h->prof_recs.back().ev + 1]));
  for (const auto& r : h->prof_recs) {
    if (r.kind < 0 || r.kind >= PK_COUNT) continue;
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, h->ev_pool[r.ev], h->ev_pool[r.ev + 1]));
    counts[r.kind] += 1;
    ms[r.kind] += t;
    flops[r.kind] += r.flops;
    bytes[r.kind] += r.bytes;
  }
  h->prof_recs.clear();
  h->ev_used = 0;
  return PK_COUNT;
}

const char* mmf_profile_kind_name(int kind) { return prof_kind_name(kind); }

int mmf_set_option(mmf_handle* h, const char* name, int value) {
  if (!name) return fail(MMF_EINVAL, "null option name");
  if (h && !strcmp(name, "text_precise_packed")) {
    // release the precise-mode weights of the GEMM kinds not in `value` (the engine's calibration, once
    // it has selected a mode that does not read them); packing happens only at weight load
    if (value & ~h->r_precise & 15)
      return fail(MMF_EINVAL, "text_precise_packed %d: only a subset of the packed kinds (%d) can be kept; re-load the "
                              "text model to re-pack", value, h->r_precise);
    if (text_mode(h) >= 2 && (h->opt.text_prec_mask & 15 & ~value))
      return fail(MMF_EINVAL, "text_precise_packed %d: the selected precise mode (text_prec_mask %d) reads them", value,
                  h->opt.text_prec_mask);
    (void)hipSetDevice(h->device);
    for (int k = 0; k < 4; ++k) {
      if (!((h->r_precise >> k) & 1) || ((value >> k) & 1)) continue;
      CHK(free_group(h, AG_TP0 + k));
      for (EncLayer& L : h->r_layers) (k == 0 ? L.qkv3 : k == 1 ? L.o3 : k == 2 ? L.fc13 : L.fc23) = Lin16{};
    }
    h->r_precise = value & 15;
    return 0;
  }
  Options& o = h ? h->opt : process_options();
  for (const OptName& n : kOptNames)
    if (!strcmp(n.name, name)) {
      if (h && (h->ready & 1)) {
        const bool prec = !strcmp(name, "text_hilo") ? value >= 2 : o.text_hilo >= 2;
        const int pm = (!strcmp(name, "text_prec_mask") ? value : o.text_prec_mask) & 15;
        if ((!strcmp(name, "text_hilo") || !strcmp(name, "text_prec_mask")) && prec && (pm & ~h->r_precise))
          return fail(MMF_EINVAL, "text_hilo = 2 with text_prec_mask %d needs precise-mode weights that are not packed "
                                  "(packed: %d; re-load the text model with text_hilo -1 or 2)", pm, h->r_precise);
      }
      o.*(n.field) = value;
      if (h) {
        (void)hipSetDevice(h->device);
        return ensure_mode_ws(h);  // (precision modes: their workspaces follow the selection)
      }
      return 0;
    }
  return fail(MMF_EINVAL, "unknown option '%s'", name);
}

const char* mmf_option_name(int i) {
  constexpr int n = (int)(sizeof(kOptNames) / sizeof(kOptNames[0]));
  return (i >= 0 && i < n) ? kOptNames[i].name : nullptr;
}

int mmf_get_option(mmf_handle* h, const char* name, int* value) {
  if (!name || !value) return fail(MMF_EINVAL, "null argument");
  if (h && !strcmp(name, "text_hilo_effective")) {  // read-only: the stream layout run_text uses
    *value = h->opt.text_hilo < 0 ? h->r_hilo_auto : h->opt.text_hilo;
    return 0;
  }
  if (h && !strcmp(name, "text_precise_packed")) {  // kinds whose precise-mode weights are packed
    *value = h->r_precise;
    return 0;
  }
  const Options& o = h ? h->opt : process_options();
  for (const OptName& n : kOptNames)
    if (!strcmp(n.name, name)) {
      *value = o.*(n.field);
      return 0;
    }
  return fail(MMF_EINVAL, "unknown option '%s'", name);
}

namespace {
// Pillow's support / taps / bounds on the host (the same double arithmetic as Resample.c) for the
// window bookkeeping; the coefficients themselves are computed on the device (resize.hip)
struct AxisPlan { double scale, support; int ks; };
AxisPlan axis_plan(int in_size, int out_size, int filt) {
  AxisPlan a;
  a.scale = (double)(float)in_size / out_size;
  const double fs = a.scale < 1.0 ? 1.0 : a.scale;
  a.support = (filt ? 2.0 : 1.0) * fs;
  a.ks = (int)std::ceil(a.support) * 2 + 1;
  return a;
}
void tap_range(const AxisPlan& a, int in_size, int xx, int* lo, int* hi) {
  const double center = (xx + 0.5) * a.scale;
  int xmin = (int)(center - a.support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + a.support + 0.5);
  if (xmax > in_size) xmax = in_size;
  *lo = xmin;
  *hi = xmax;
}
// one job = one image in one geometry: geom 0 = EfficientNet squash (bilinear), 1 = CLIP
// shortest-edge + centre crop (bicubic); returns false when a pass needs more than kResizeKMax taps
bool plan_job(int w, int h, int geom, ResizeJob* J) {
  *J = ResizeJob{};
  J->w = w;
  J->h = h;
  J->filt = geom;
  if (w == 224 && h == 224) {
    J->ow = J->oh = 224;
  } else if (geom == 0) {
    J->ow = J->oh = 224;
  } else {
    const int shrt = w <= h ? w : h, lng = w <= h ? h : w;
    const int new_long = (int)(224.0 * lng / shrt);
    J->ow = w <= h ? 224 : new_long;
    J->oh = w <= h ? new_long : 224;
    J->cx = (J->ow - 224) / 2;
    J->cy = (J->oh - 224) / 2;
  }
  J->need_h = J->ow != w;
  J->need_v = J->oh != h;
  J->ksh = J->need_h ? axis_plan(w, J->ow, J->filt).ks : 1;
  J->ksv = J->need_v ? axis_plan(h, J->oh, J->filt).ks : 1;
  if (J->ksh > kResizeKMax || J->ksv > kResizeKMax) return false;
  if (J->need_v) {
    const AxisPlan a = axis_plan(h, J->oh, J->filt);
    int lo, hi;
    tap_range(a, h, J->cy, &lo, &hi);
    J->y0 = lo;
    tap_range(a, h, J->cy + 223, &lo, &hi);
    J->y1 = hi;
  } else {
    J->y0 = J->cy;
    J->y1 = J->cy + 224;
  }
  return true;
}
}  // namespace

int mmf_jpeg_reconstruct(mmf_handle* h, const uint8_t* packed, const uint32_t* block_off, const int64_t* pk_off,
                         const uint16_t* qt, const int64_t* coef_blocks, const int32_t* infos, const int64_t* out_offsets,
                         int B, int max_blocks, int max_pixels, uint8_t* samples, uint8_t* out_rgbx, void* stream) {
  if (!h || B < 0) return fail(MMF_EINVAL, "null argument");
  if (B == 0) return 0;
  if (!packed || !block_off || !pk_off || !qt || !coef_blocks || !infos || !out_offsets || !samples || !out_rgbx)
    return fail(MMF_EINVAL, "null argument");
  if (max_blocks <= 0 || max_pixels <= 0) return fail(MMF_EINVAL, "max_blocks / max_pixels must be positive");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(launch_jpeg_reconstruct(packed, block_off, pk_off, qt, coef_blocks, infos, out_offsets, B, max_blocks,
                                 max_pixels, samples, out_rgbx, (hipStream_t)stream));
  return 0;
}

int mmf_resize_pil(mmf_handle* h, const uint8_t* src, const int64_t* offsets, const int32_t* wh, int B,
                   int pixel_bytes, uint8_t* out_effnet, uint8_t* out_clip, void* stream) {
  if (!h || !src || !offsets || !wh || B < 0) return fail(MMF_EINVAL, "null argument");
  if (pixel_bytes != 3 && pixel_bytes != 4) return fail(MMF_EINVAL, "pixel_bytes must be 3 (RGB) or 4 (RGBX)");
  if (!out_effnet && !out_clip) return 0;
  HIPCHK(hipSetDevice(h->device));
  std::vector<ResizeJob> jobs;
  std::vector<uint8_t*> outs;
  long long tmp = 0;
  int coef = 0, max_rows = 0;
  for (int i = 0; i < B; ++i) {
    const int w = wh[2 * i], ht = wh[2 * i + 1];
    if (w <= 0 || ht <= 0) return fail(MMF_EINVAL, "image %d has size %dx%d", i, w, ht);
    for (int geom = 0; geom < 2; ++geom) {
      uint8_t* o = geom ? out_clip : out_effnet;
      if (!o) continue;
      ResizeJob J;
      if (!plan_job(w, ht, geom, &J))
        return fail(MMF_ERANGE, "image %d (%dx%d): downscale beyond %d taps per output pixel", i, w, ht, kResizeKMax);
      J.src_off = offsets[i];
      J.ps = pixel_bytes;
      J.tmp_off = tmp;
      J.coef_off = coef;
      tmp += (long long)(J.y1 - J.y0) * 224 * 3;
      coef += 224 * (J.ksh + J.ksv);
      max_rows = std::max(max_rows, J.y1 - J.y0);
      jobs.push_back(J);
      outs.push_back(o + (size_t)i * 224 * 224 * 3);
    }
  }
  auto& R = h->rs;
  const size_t nj = jobs.size();
  if (nj > R.cap_jobs || (size_t)coef > R.cap_coef || (size_t)tmp > R.cap_tmp) {
    CHK(free_group(h, AG_RESIZE));
    R.cap_jobs = std::max(nj, R.cap_jobs);
    R.cap_coef = std::max((size_t)coef, R.cap_coef);
    R.cap_tmp = std::max((size_t)tmp, R.cap_tmp);
    void* p;
    CHK(dev_alloc(h, &p, R.cap_jobs * sizeof(ResizeJob), AG_RESIZE)); R.jobs = (ResizeJob*)p;
    CHK(dev_alloc(h, &p, R.cap_jobs * sizeof(uint8_t*), AG_RESIZE)); R.outs = (uint8_t**)p;
    CHK(dev_alloc(h, &p, R.cap_jobs * 2 * 224 * 2 * sizeof(int32_t), AG_RESIZE)); R.bounds = (int32_t*)p;
    CHK(dev_alloc(h, &p, R.cap_coef * sizeof(int32_t), AG_RESIZE)); R.coef = (int32_t*)p;
    CHK(dev_alloc(h, &p, R.cap_tmp, AG_RESIZE)); R.tmp = (uint8_t*)p;
  }
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(R.jobs, jobs.data(), nj * sizeof(ResizeJob), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(R.outs, outs.data(), nj * sizeof(uint8_t*), hipMemcpyHostToDevice, s));
  HIPCHK(launch_resize_pil(src, R.jobs, (int)nj, max_rows, R.coef, R.bounds, R.tmp, R.outs, s));
  HIPCHK(hipStreamSynchronize(s));  // the host job tables above are released on return
  return 0;
}

int mmf_resize_supported(int width, int height) {
  if (width <= 0 || height <= 0) return 0;
  ResizeJob J;
  return plan_job(width, height, 0, &J) && plan_job(width, height, 1, &J) ? 1 : 0;
}

int64_t mmf_device_bytes(mmf_handle* h) {
  if (!h) return 0;
  int64_t t = 0;
  for (size_t b : h->group_bytes) t += (int64_t)b;
  return t;
}

int mmf_gemm_f16(const void* A, int lda, const void* W, int ldw, const float* bias, const float* residual, float* c32,
                  void* c16, int ldc, int M, int N, int K, int act, void* stream) {
  GemmArgs g{};
  g.A = (const f16_t*)A;
  g.lda = lda;
  g.W = (const f16_t*)W;
  g.ldw = ldw;
  g.bias = bias;
  g.res32 = residual;
  g.ldr = ldc;
  g.c32 = c32;
  g.c16 = (f16_t*)c16;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.act = act;
  apply_options(process_options(), &g);
  if (!A || !W || (!c32 && !c16)) return fail(MMF_EINVAL, "null argument");
  hipError_t e = launch_gemm(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MMF_EIO, "gemm: %s", hipGetErrorString(e));
  return 0;
}

int mmf_gemm_f16_ex(const void* A, int lda, const void* W, int ldw, const float* bias, const void* res16,
                     const float* ascale, int rows_per_batch, void* c16, int ldc, int M, int N, int K, int act,
                     void* stream) {
  GemmArgs g{};
  g.A = (const f16_t*)A;
  g.lda = lda;
  g.W = (const f16_t*)W;
  g.ldw = ldw;
  g.bias = bias;
  g.res16 = (const f16_t*)res16;
  g.ldr = ldc;
  g.ascale = ascale;
  g.rows_per_batch = rows_per_batch;
  g.c16 = (f16_t*)c16;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.act = act;
  apply_options(process_options(), &g);
  if (!A || !W || !c16) return fail(MMF_EINVAL, "null argument");
  if (ascale && rows_per_batch <= 0) return fail(MMF_EINVAL, "rows_per_batch must be > 0 with ascale");
  hipError_t e = launch_gemm(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MMF_EIO, "gemm: %s", hipGetErrorString(e));
  return 0;
}

int mmf_gemm_f16_split(const void* A, int lda, const void* W, int ldw, const float* bias, void* c16, int ldc, int M,
                       int N, int K, int act, int split_lo, void* stream) {
  GemmArgs g{};
  g.A = (const f16_t*)A;
  g.lda = lda;
  g.W = (const f16_t*)W;
  g.ldw = ldw;
  g.bias = bias;
  g.c16 = (f16_t*)c16;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.act = act;
  g.epi = 4;
  g.split_lo = split_lo ? 1 : 0;
  apply_options(process_options(), &g);
  if (!A || !W || !c16 || !bias) return fail(MMF_EINVAL, "null argument");
  if (!gemm_epi_ok(g)) return fail(MMF_EINVAL, "split-operand epilogue not applicable (M=%d N=%d K=%d ldc=%d act=%d)", M, N, K, ldc, act);
  hipError_t e = launch_gemm(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MMF_EIO, "gemm: %s", hipGetErrorString(e));
  return 0;
}

int mmf_attention_f16(const void* qkv, const int32_t* mask, void* out, int B, int L, int H, int causal,
                       void* stream) {
  if (!qkv || !out) return fail(MMF_EINVAL, "null argument");
  hipError_t e = launch_attention((const f16_t*)qkv, 3 * H * 64, mask, (f16_t*)out, H * 64, B, L, H, causal,
                                  (hipStream_t)stream);
  if (e != hipSuccess) return fail(MMF_EIO, "attention: %s", hipGetErrorString(e));
  return 0;
}

}  // extern "C"
