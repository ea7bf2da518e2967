// Internal structures of libmde_hip's engine: the loaded packed weights
// (mde_engine), the execution context with its activation arena
// (mde_context) and the forward-schedule runner shared by the model
// families (engine.hip: Depth Anything V2; depth_pro.hip: Depth Pro).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/mde.h"
#include "mde_ops.h"
#include "pack_format.h"
#include "tuning.h"

namespace mde {

struct DevTensor {
  void* ptr = nullptr;
  int dtype = 0;
  int ndim = 0;
  int dims[4] = {0, 0, 0, 0};
};

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Depth Anything V2 activations (engine.hip plan_arena_dav2)
struct DAV2Buf {
  h16 *P, *Hn, *Q, *K, *Vt, *O, *Mh;
  float* X;   // fp32 residual stream [B*T][D] (null when Xh is used)
  h16* Xh;    // f16 residual stream (packed precision "fp16", cfg.resid_f16), else null
  h16 *tap[4], *pj[4], *l1, *l2, *l4, *rn[4];
  h16 *tb, *sb, *ub, *vb, *p4, *p3, *p2, *c1;
  float* ws;        // fc2 split-K partials [4][B*T][D] (small-batch contexts only, else null)
  float* aws;       // attention split-KV partials (batches whose grid splits, else null)
  size_t aws_bytes;
  float* st;        // folded-LN partials [B*T][D/32][2] (f16 residual + folded pack, else null)
  float* sws;       // E_STORE split-K partials (GemmParams::partial_cap = kSplitWsFloats)
  // exact-fp32 encoder (PackConfig::enc_f32, fp32.hip): fp32 patch rows, LN
  // output, q / k / v [B*H][Tpad][64], attention output, MLP hidden (else null)
  float *P32, *Hn32, *Q32, *K32, *V32, *O32, *Mh32;
  // exact-fp32 DPT head (packs with head.c1.w32, fp32.hip): fp32 NHWC maps
  // mirroring the f16 ones above, the x2-upsampled fusion output, output_conv1,
  // its upsample to the input size and the head's hidden map (else null)
  float *tap32[4], *pj32[4], *l1_32, *l2_32, *l4_32, *rn32[4];
  float *tb32, *sb32, *ub32, *vb32, *p4_32, *p3_32, *p2_32, *up1_32, *c1_32, *up2_32, *hid32;
};

// fp32 elements of a context's E_STORE split-K workspace (launch_gemm bounds
// slices x M x N by it; the largest split the policy picks is ~4.2 M)
constexpr size_t kSplitWsFloats = size_t(5) << 20;
// the allocation behind it: the fused split-K slots are whole 64^2 tiles
// (padding beyond M x N), then kTileCnt arrival counters (int, zeroed with the
// arena; GemmParams::tile_cnt)
constexpr size_t kSplitSlotFloats = size_t(6) << 20;
constexpr int kTileCnt = 16384;
constexpr size_t kSplitWsAlloc = kSplitSlotFloats + kTileCnt;
inline int* split_counters(float* sws) { return sws ? reinterpret_cast<int*>(sws + kSplitSlotFloats) : nullptr; }
// fc2 split-K partials of a small-batch context: [4][rows rounded up to 128][D]
// (the fused form's 128^2 slots of D % 128 == 0 encoders fit)
inline size_t fc2_ws_floats(size_t rows, int D) { return 4 * align_up(rows, 128) * (size_t)D; }

// Depth Pro activations (depth_pro.hip plan_arena_dp).  Token buffers are
// sized for the patch encoder (35 sequences per image), the largest of the
// three encoders; maps are NHWC f16.
struct DPBuf {
  h16* P;                          // patch-embed rows [35B*G*G][3*16*16]
  float *Xp, *Xi, *Xf;             // residual streams: patch / image / fov encoder
  h16 *Hn, *Q, *K, *Vt, *O, *Mh;   // block scratch
  h16* hook[2];                    // raw hook maps [B][4G][4G][D]
  h16* lev[3];                     // final-LN level maps: [B][G][G], [2G], [4G] x D
  h16 *im, *fm, *fovf;             // image / fov encoder maps [B][G][G][D], fov neck [..][F/2]
  h16 *tmp, *tmp2;                 // projection temporaries
  h16 *gcat, *glob;                // [B][2G][2G][2 sd0], fused global [.. sd0]
  h16 *f1, *f2, *i0, *i1;          // upsampled scale / intermediate features
  h16* pr[5];                      // 3x3 projections (pr[4] aliases i1 when Identity)
  h16 *h0, *h1, *tb, *sb, *ub;     // fusion stage
  h16 *c1, *ct;                    // head
  h16 *fv1, *fv2, *fv3;            // fov head
  float* sws;                      // E_STORE split-K partials (kSplitWsFloats)
};

// VGGT activations (vggt.hip plan_arena_vggt) over n = B*S frames.
struct VGBuf {
  h16* P;                  // patch-embed rows [n*np][672]
  float *X, *Xf;           // residual stream [n][T][D]; frame-block output snapshot at the taps
  h16 *Hn, *O, *Mh;        // block scratch
  h16 *Q, *K, *Vt;         // frame attention operands [n*H][Tpad][64]
  h16 *Qg, *Kg, *Vg;       // global attention operands [B*H][Tgpad][64] (alias Q/K/Vt when S == 1)
  h16* tap;                // LN(cat(frame, global)) patch tokens [n*np][2D]
  h16 *pj[4], *l1, *l2, *l4, *rn[4];
  h16 *tb, *sb, *ub, *vb, *p4, *p3, *p2, *c1;
  float* ws;               // fc2 split-K partials [4][ws_rows][D] (small-batch contexts only, else null)
  size_t ws_rows;
  float* sws;              // E_STORE split-K partials (kSplitWsFloats)
};

enum Family : int { FAMILY_DAV2 = 0, FAMILY_DEPTH_PRO = 1, FAMILY_VGGT = 2 };

}  // namespace mde

struct mde_engine {
  int device = 0;
  int family = mde::FAMILY_DAV2;
  mde::PackConfig cfg{};
  void* wmem = nullptr;
  size_t wbytes = 0;
  std::unordered_map<std::string, mde::DevTensor> t;
  // DA-V2 geometry
  int ph = 0, pw = 0, np = 0, T = 0, Tpad = 0, D = 0, H = 0, F = 0;
  int h4 = 0, w4 = 0;
  int c1p = 0;          // reassemble-0 channels padded to a multiple of 32 (direct-conv input)
  bool head_f32 = false;  // DA-V2 exact-fp32 DPT head (fp32 head weights packed, precision "fp32")
  float head_b2 = 0.f;  // final 1x1 conv bias (scalar kernel argument; both families)
  // Depth Pro geometry: G tokens per side of a 384^2 patch, pyramid levels
  int G = 0, nseq = 0;  // nseq = patches per image (35)
  int lev_n[3] = {0, 0, 0}, lev_pad[3] = {0, 0, 0}, lev_base[3] = {0, 0, 0}, lev_stride[3] = {0, 0, 0};
  int lev_f[3] = {0, 0, 0};  // downsample factor of the level (4, 2, 1)
  float fov_b = 0.f;
  // VGGT geometry: npre special tokens per frame, S frames per batch item,
  // Tg = S * T tokens per global-attention sequence (padded to Tgpad)
  int npre = 0, S = 1, Tg = 0, Tgpad = 0;

  const mde::DevTensor* get(const std::string& n) const {
    auto it = t.find(n);
    return it == t.end() ? nullptr : &it->second;
  }
};

namespace mde {

struct GraphKey {
  int batch;
  void* in;
  void* out;
  void* out2;
  bool operator<(const GraphKey& o) const {
    return std::tie(batch, in, out, out2) < std::tie(o.batch, o.in, o.out, o.out2);
  }
};

}  // namespace mde

struct mde_context {
  mde_engine* e = nullptr;
  int device = 0;
  int max_batch = 1;
  int batch = 1;
  void* in = nullptr;
  void* out = nullptr;
  void* out2 = nullptr;  // Depth Pro "fov_deg"
  void* arena = nullptr;
  size_t arena_bytes = 0;
  mde::DAV2Buf b{};
  mde::DPBuf d{};
  mde::VGBuf v{};
  bool graph_mode = true;
  hipStream_t cap_stream = nullptr;
  // captured forwards per (batch, io addresses), at most kMaxGraphs of them:
  // the least recently launched one is destroyed to make room (a caller that
  // rebinds fresh buffers every call pays a capture, not unbounded growth)
  static constexpr int kMaxGraphs = 8;
  std::map<mde::GraphKey, std::pair<hipGraph_t, hipGraphExec_t>> graphs;
  std::map<mde::GraphKey, unsigned long long> graph_used;
  // per cached graph: an event recorded behind its latest replay, so an
  // eviction waits for that replay only (not the whole device)
  std::map<mde::GraphKey, hipEvent_t> graph_done;
  unsigned long long graph_tick = 0;
  mde_layer_cb prof_cb = nullptr;
  void* prof_user = nullptr;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> prof_events;
  size_t prof_used = 0;
};

namespace mde {

// Bump allocator over the arena (base == nullptr: size only).
struct ArenaPlan {
  uint8_t* base;
  size_t off = 0;
  explicit ArenaPlan(uint8_t* b) : base(b) {}
  void* take(size_t bytes) {
    void* p = base ? (void*)(base + off) : nullptr;
    off += align_up(bytes, 256);
    return p;
  }
  h16* h(size_t elems) { return (h16*)take(elems * 2); }
  float* f(size_t elems) { return (float*)take(elems * 4); }
};

size_t plan_arena_dav2(const mde_engine& e, int B, DAV2Buf* b, uint8_t* base);
size_t plan_arena_dp(const mde_engine& e, int B, DPBuf* b, uint8_t* base);
size_t plan_arena_vggt(const mde_engine& e, int B, VGBuf* b, uint8_t* base);
// Load-time checks (tensor presence, supported geometry); fill the derived
// geometry.  Return an error message or "".
std::string setup_depth_pro(mde_engine* e);
std::string setup_vggt(mde_engine* e);

// The forward schedule: one method per model family, common helpers here.
struct Runner {
  mde_context& c;
  hipStream_t st;
  bool prof;
  hipError_t err = hipSuccess;

  template <class Fn>
  void step(const char* name, Fn&& fn) {
    if (err != hipSuccess) return;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
      if (c.prof_used >= c.prof_events.size()) {
        hipEvent_t a, b;
        if ((err = hipEventCreate(&a)) != hipSuccess) return;
        if ((err = hipEventCreate(&b)) != hipSuccess) return;
        c.prof_events.push_back({std::string(), {a, b}});
      }
      auto& slot = c.prof_events[c.prof_used++];
      slot.first = name;
      e0 = slot.second.first;
      e1 = slot.second.second;
      if ((err = hipEventRecord(e0, st)) != hipSuccess) return;
    }
    err = fn();
    if (err == hipSuccess && prof) err = hipEventRecord(e1, st);
  }

  const DevTensor& W(const std::string& n) { return *c.e->get(n); }
  const h16* w16(const std::string& n) { return (const h16*)W(n).ptr; }
  const float* w32(const std::string& n) { return (const float*)W(n).ptr; }
  const float* w32_opt(const std::string& n) {
    const DevTensor* t = c.e->get(n);
    return t ? (const float*)t->ptr : nullptr;
  }
  int ldw(const std::string& n) { return W(n).dims[W(n).ndim - 1]; }

  GemmParams dense(const h16* A, int lda, const std::string& w, int M, int N, int K) {
    GemmParams g;
    g.amode = A_DENSE;
    g.A = A;
    g.lda = lda;
    g.W = w16(w);
    g.ldw = ldw(w);
    g.M = M;
    g.N = N;
    g.K = K;
    return g;
  }

  // 3x3 pad-1 conv over NHWC map [B][h][w][cin] -> [B][ho][wo][cout]
  GemmParams conv(const h16* in, int B, int h, int w, int cin, const std::string& wn, int cout, int stride) {
    GemmParams g;
    g.amode = A_CONV3;
    g.A = in;
    g.cb = B;
    g.ch = h;
    g.cw = w;
    g.cc = cin;
    g.stride = stride;
    g.oh = (h - 1) / stride + 1;
    g.ow = (w - 1) / stride + 1;
    g.W = w16(wn);
    g.ldw = ldw(wn);
    g.M = B * g.oh * g.ow;
    g.N = cout;
    g.K = 9 * cin;
    g.out16 = nullptr;
    g.ldo = cout;
    return g;
  }

  // ConvTranspose(k = s = 2) of an NHWC map as a GEMM with a pixel-shuffle
  // epilogue; ldo = channel stride of the output map (concat slots)
  GemmParams convt2(const h16* in, int B, int h, int w, int cin, const std::string& wn, int cout, h16* out,
                    int ldo) {
    GemmParams g = dense(in, cin, wn, B * h * w, 4 * cout, cin);
    g.emode = E_CONVT;
    g.out16 = out;
    g.s = 2;
    g.cout = cout;
    g.ldo = ldo;
    g.ih = h;
    g.iw = w;
    return g;
  }

  // E_STORE split-K workspace for launch_gemm's small-grid policy (null: never split)
  float* split_ws = nullptr;

  // exact-fp32 dense GEMM (fp32.hip) over fp32 weights [Npad][ldw]
  Gemm32Params dense32(const float* A, int lda, const std::string& w, int M, int N, int K) {
    Gemm32Params g;
    g.A = A;
    g.lda = lda;
    g.W = w32(w);
    g.ldw = ldw(w);
    g.M = M;
    g.N = N;
    g.K = K;
    return g;
  }
  void gemm32(const char* name, const Gemm32Params& g) {
    step(name, [&] { return launch_gemm32(g, st); });
  }
  // exact-fp32 3x3 pad-1 conv over an fp32 NHWC map [B][h][w][cin] (implicit im2col)
  Gemm32Params conv32(const float* in, int B, int h, int w, int cin, const std::string& wn, int cout, int stride) {
    Gemm32Params g;
    g.amode = A_CONV3;
    g.emode = E_STORE;
    g.A = in;
    g.cb = B;
    g.ch = h;
    g.cw = w;
    g.cc = cin;
    g.stride = stride;
    g.oh = (h - 1) / stride + 1;
    g.ow = (w - 1) / stride + 1;
    g.W = w32(wn);
    g.ldw = ldw(wn);
    g.M = B * g.oh * g.ow;
    g.N = cout;
    g.K = 9 * cin;
    g.ldo = cout;
    return g;
  }
  // the fp32 pre-activation residual conv unit (rcu below, on fp32 maps)
  void rcu32(const std::string& pfx, const float* x, const float* extra, float* out, float* tmp, int B, int h, int w,
             int F) {
    Gemm32Params g1 = conv32(x, B, h, w, F, pfx + ".c1.w32", F, 1);
    g1.relu_in = 1;
    g1.bias = w32_opt(pfx + ".c1.b");
    g1.act = ACT_RELU;
    g1.out32 = tmp;
    gemm32((pfx + ".c1").c_str(), g1);
    Gemm32Params g2 = conv32(tmp, B, h, w, F, pfx + ".c2.w32", F, 1);
    g2.bias = w32_opt(pfx + ".c2.b");
    g2.res0 = x;
    g2.res1 = extra;
    g2.out32 = out;
    gemm32((pfx + ".c2").c_str(), g2);
  }
  void dav2_head32(int B, float* out);

  void gemm(const char* name, const GemmParams& g) {
    GemmParams q = g;
    if (split_ws && g.emode == E_STORE && !g.partial) {
      q.partial = split_ws;
      q.partial_cap = kSplitWsFloats;
      q.slot_cap = kSplitSlotFloats;
      q.tile_cnt = split_counters(split_ws);
      q.tile_cnt_cap = kTileCnt;
    }
    step(name, [&] { return launch_gemm(q, st); });
  }

  // pre-activation residual conv unit:
  // out = conv2(relu(conv1(relu(x)) + b1)) + b2 + x (+ extra)
  // relu_res: the skip adds relu(x) instead of x (an nn.ReLU(inplace=True)
  // activation overwrites the unit's input, as in VGGT's DPT head)
  // extra_up (GemmParams::res1_up): extra is the bilinear upsample of extra_up
  // [B][uh][uw][F], read on the fly where the conv route allows (else written
  // into extra first)
  void rcu(const std::string& pfx, const h16* x, const h16* extra, h16* out, h16* tmp, int B, int h, int w, int F,
           bool relu_res = false, const h16* extra_up = nullptr, int uh = 0, int uw = 0) {
    GemmParams g1 = conv(x, B, h, w, F, pfx + ".c1.w", F, 1);
    g1.relu_in = 1;
    g1.bias = w32_opt(pfx + ".c1.b");
    g1.act = ACT_RELU;
    g1.out16 = tmp;
    gemm((pfx + ".c1").c_str(), g1);
    GemmParams g2 = conv(tmp, B, h, w, F, pfx + ".c2.w", F, 1);
    g2.bias = w32_opt(pfx + ".c2.b");
    g2.res0 = x;
    g2.res0_relu = relu_res ? 1 : 0;
    g2.res1 = extra;
    g2.res1_up = extra_up;
    g2.res1_uh = uh;
    g2.res1_uw = uw;
    g2.out16 = out;
    gemm((pfx + ".c2").c_str(), g2);
  }

  hipError_t forward_dav2(int B, const void* img, float* out);
  bool dav2_fusion(int r, const h16* x0, const h16* x1, int B, int h, int w, h16* dst, int oh, int ow,
                   const h16* x0_up = nullptr, int uh = 0, int uw = 0);
  hipError_t forward_dp(int B, const float* img, float* out, float* fov);
  void dp_encoder(const std::string& pfx, float* X, const h16* P, int nseq, int hook_seqs);
  hipError_t forward_vggt(int B, const float* img, float* out);
  void vggt_block(const std::string& p, float eps, bool qk, int seqs, int T, int Tpad, h16* Q, h16* K, h16* Vt);
  void vggt_fusion(int r, const h16* x0, const h16* x1, int n, int h, int w, h16* dst, int oh, int ow);
};

}  // namespace mde
