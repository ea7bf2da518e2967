// Host-side launch interface of the hot-path kernels (internal to libmde_hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mde {

typedef _Float16 h16;

// How the A operand (rows = output pixels / tokens, K contiguous) is formed.
enum AMode : int {
  A_DENSE = 0,    // A[m*lda + k], row-major f16
  A_CONV3 = 1,    // implicit im2col of a 3x3 pad-1 conv over an NHWC f16 map
  A_CONV3_UP = 2  // same, over bilinear(align_corners=True)-upsampled NHWC map
};

// What the epilogue does with acc[m][n] (fp32).
enum EMode : int {
  E_STORE = 0,   // out16[m*ldo+n] = act(acc + bias[n]) (+ res0 + res1)
  E_QKV = 1,     // scatter to head-major q (pre-scaled), k and transposed v
  E_RESID = 2,   // x32[m*ldo+n] += ls[n] * (acc + bias[n])
  E_PATCH = 3,   // x32[(b*T+tok0+p)*ldo+n] = acc + bias[n] + pos[p*ldo+n]
  E_CONVT = 4,   // ConvTranspose(k=s) pixel-shuffle store into NHWC f16
  E_HEAD = 5,    // relu(acc+bias(+pe)) . w2 + b2 -> sigmoid*max | relu | exp -> fp32 map
  E_PARTIAL = 6  // split-K slice s (blockIdx.y, XCD-remapped): x32[s*M*ldo + m*ldo + n] = acc (split paths only)
};

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

struct GemmParams {
  int amode = A_DENSE, emode = E_STORE;
  int M = 0, N = 0, K = 0;
  const h16* A = nullptr; int lda = 0;
  const h16* W = nullptr; int ldw = 0;  // weights [Npad][ldw], ldw % 64 == 0
  // conv geometry: source NHWC map [cb][ch][cw][cc]; output map [cb][oh][ow]
  int cb = 0, ch = 0, cw = 0, cc = 0;
  int uh = 0, uw = 0;  // virtual (upsampled) input size, A_CONV3_UP
  int oh = 0, ow = 0, stride = 1;
  int relu_in = 0;
  // epilogue
  const float* bias = nullptr; int act = ACT_NONE;
  h16* out16 = nullptr; int ldo = 0;
  const h16* res0 = nullptr; const h16* res1 = nullptr;
  // E_STORE residual options: res0_relu -> add relu(res0) (VGGT's in-place
  // ReLU residual units); res0_rows > 0 -> res0 is a table of res0_rows rows
  // repeated over m (row m % res0_rows: a per-image positional embedding)
  int res0_relu = 0; int res0_rows = 0;
  // res1_up (switch "resize_fold"): res1 is the bilinear (align_corners)
  // upsample of res1_up [cb][res1_uh][res1_uw][N] to the output map [cb][oh][ow]
  // (3x3 conv problems, ldo == N).  The direct conv reads it through that
  // upsample in its epilogue; every other path first writes the upsample into
  // res1 (launch_gemm), so res1 must be a buffer of the output's shape either way
  const h16* res1_up = nullptr; int res1_uh = 0, res1_uw = 0;
  float* x32 = nullptr; const float* ls = nullptr;
  // f16 residual stream: when set, E_RESID / E_PATCH update / write xh
  // [m][ldo] f16 instead of x32 (DA-V2 engines with an f16 residual)
  h16* xh = nullptr;
  // E_QKV
  h16 *q = nullptr, *k = nullptr, *vt = nullptr;
  int T = 0, Tpad = 0, heads = 0; float qscale = 1.0f;
  // E_PATCH: patch rows start at token tok0 of each sequence (1 = after cls)
  const float* pos = nullptr; int npatch = 0; int tok0 = 1;
  // E_CONVT
  int s = 0, cout = 0, ih = 0, iw = 0;
  // E_HEAD: head_metric 0 ReLU, 1 max_depth * sigmoid, 2 exp; hpe (optional)
  // = f16 [hpe_pix][32] added to the hidden layer before its ReLU at pixel
  // m % hpe_pix (VGGT: the folded conv of the UV positional embedding)
  const float* w2 = nullptr; float b2 = 0.f; int head_metric = 1; float max_depth = 1.f;
  float* out32 = nullptr;
  const h16* hpe = nullptr; int hpe_pix = 0;
  // E_RESID split-K (small M, long K): splitk > 1 and partial = fp32
  // workspace [splitk][M][N]; the K range is cut into splitk slices whose
  // partial sums are added in slice order by a second kernel (deterministic)
  int splitk = 1; float* partial = nullptr;
  // E_STORE split-K (dense and 3x3-conv problems whose tile grid leaves most
  // of the chip idle: small batches, the DPT's 19^2 / 37^2 maps): when
  // partial_cap > 0 the launcher picks the slice count itself, bounded by
  // partial_cap fp32 elements of `partial`
  size_t partial_cap = 0;
  // Fused split-K (switch "splitk_fused"): with tile_cnt set (tile_cnt_cap
  // zero-initialised arrival counters, left zero by every launch) both split
  // paths above run as ONE launch whose last-arriving slice per tile adds the
  // slices' slots -- S x tiles x BM x BN fp32 in `partial`, at most slot_cap
  // elements -- in slice order and runs the epilogue; otherwise, or when the
  // slots do not fit, the slices + reduce-kernel form
  int* tile_cnt = nullptr; int tile_cnt_cap = 0; size_t slot_cap = 0;
  // LayerNorm folded across a GEMM boundary (DA-V2 f16-residual engines):
  //  * producer (E_RESID / E_PATCH over xh, and the split-K reduce): lnst_out
  //    = fp32 [lnst_ns][lnst_rows][2] -- per 32-column slice and token row
  //    (slice-major: a load of 16 consecutive rows is one 128-B line), the
  //    sum of the f16 values written and their squared deviations from the
  //    slice mean (M2; merged with Chan et al.'s formula, no E[x^2] - mean^2);
  //  * consumer (the next qkv / fc1, A = the raw f16 residual rows, W = W * gamma,
  //    bias = b + W beta): lnst_in = those partials, lnc1[n] = sum_k W[n][k]
  //    -> acc := rstd_m * (acc - mean_m * lnc1[n]) before the epilogue.
  float* lnst_out = nullptr;
  const float* lnst_in = nullptr; const float* lnc1 = nullptr;
  int lnst_ns = 0, lnst_rows = 0; float ln_eps = 1e-6f;
  // A_DENSE row skip (the DPT projects reading the residual stream through
  // the tap LayerNorm fold): a_tok > 1 -> GEMM row m reads A row (and LN
  // partial row) (m / (a_tok - 1)) * a_tok + 1 + m % (a_tok - 1), i.e. every
  // sequence's first (cls) row is skipped
  int a_tok = 0;
};

// Exact-fp32 encoder GEMM (fp32.hip; precision "fp32" engines): C = A W^T
// with fp32 A [M][lda] (lda % 4 == 0, 16-B aligned) and fp32 W [Npad][ldw]
// (ldw % 32 == 0, zero-padded), v_mfma_f32_16x16x4_f32.  emode:
//   E_STORE  out32 (fp32) or out16 (f16) [m*ldo + n] = act(acc + bias)
//   E_QKV    q (scaled by qscale) / k / v fp32 [B*heads][Tpad][64] rows
//   E_RESID  x32[m*ldo + n] += ls[n] * (acc + bias[n])
//   E_PATCH  x32[(b*T + 1 + p)*ldo + n] = acc + bias[n] + pos[p*ldo + n]
struct Gemm32Params {
  int emode = E_STORE;
  int amode = A_DENSE;  // A_DENSE or A_CONV3 (implicit im2col of a 3x3 pad-1 conv over an fp32 NHWC map)
  int M = 0, N = 0, K = 0;
  const float* A = nullptr; int lda = 0;
  const float* W = nullptr; int ldw = 0;
  const float* bias = nullptr; int act = ACT_NONE;
  float* out32 = nullptr; h16* out16 = nullptr; int ldo = 0;
  float* x32 = nullptr; const float* ls = nullptr;
  float *q = nullptr, *k = nullptr, *v = nullptr; int T = 0, Tpad = 0, heads = 0; float qscale = 1.f;
  const float* pos = nullptr; int npatch = 0;
  // A_CONV3: input map [cb][ch][cw][cc] (cc % 4 == 0), output [cb][oh][ow],
  // K = 9 cc in (ky, kx, c) order; relu_in: ReLU applied to the A operand
  int cb = 0, ch = 0, cw = 0, cc = 0, stride = 1, oh = 0, ow = 0, relu_in = 0;
  // E_STORE: out = act(acc + bias) + res0 + res1 (fp32 maps laid out like out32)
  const float* res0 = nullptr; const float* res1 = nullptr;
  // E_CONVT (ConvTranspose k = s): rows = input pixels [cb][ih][iw], column
  // n = (dy s + dx) cout + co -> out32 pixel (s iy + dy, s ix + dx), channel co
  // (stride ldo), + bias[co]
  int s = 0, cout = 0, ih = 0, iw = 0;
};
hipError_t launch_gemm32(const Gemm32Params& p, hipStream_t st);
// fp32 NHWC bilinear resize, align_corners=True ([B][ih][iw][C] -> [B][oh][ow][C], C % 4 == 0)
hipError_t launch_resize32(const float* in, float* out, int B, int ih, int iw, int C, int oh, int ow, hipStream_t st);
// DPT head tail over an fp32 hidden map hid [M][32] (already ReLU'd): out[m] =
// act(sum_c w2[c] hid[m][c] + b2), act = ReLU (relative), sigmoid * max_depth
// (metric, 1), exp (2) -- output_conv2's last 1x1 conv and activation
hipError_t launch_head32(const float* hid, const float* w2, float b2, int M, int metric, float max_depth, float* out,
                         hipStream_t st);
// fp32 attention over q (pre-scaled by dh^-0.5 * log2 e) / k / v fp32
// [B*H][Tpad][64] rows -> o fp32 [B*T][ldo], head h in columns 64h .. 64h+63
hipError_t launch_attention32(const float* q, const float* k, const float* v, float* o, int B, int H, int T,
                              int Tpad, int ldo, hipStream_t st);


// x32[m*ldo+n] += ls[n] * (sum_{s<S} P[s][m][n] + bias[n]), slices summed in
// order (elementwise.hip): the second half of the E_RESID split-K path
hipError_t launch_splitk_resid(const float* P, int S, int M, int N, const float* bias, const float* ls, float* x32,
                               h16* xh, int ldo, hipStream_t st, float* lnst_out = nullptr);  // lnst_out rows = M

// out16 = E_STORE epilogue of (sum_{s<S} P[s][m][n]) (elementwise.hip): the
// second half of the E_STORE split-K path
hipError_t launch_splitk_store(const float* P, int S, const GemmParams& p, hipStream_t st);

hipError_t launch_gemm(const GemmParams& p, hipStream_t st);
// slices launch_gemm's E_STORE split-K policy picks for p (1 = no split)
int gemm_store_split_slices(const GemmParams& p);

// Direct 3x3 conv with an LDS halo patch (conv.hip); launch_gemm routes
// A_CONV3 / A_CONV3_UP problems here when conv_direct_supported().
bool conv_direct_supported(const GemmParams& p);
// the direct conv takes p's res1 through GemmParams::res1_up (conv.hip)
bool conv3_takes_res1_up(const GemmParams& p);
hipError_t launch_conv3(const GemmParams& p, hipStream_t st);

// A-stationary panel GEMM (gemm_panel.hip) for K = 384 token-major E_STORE /
// E_QKV problems at large batch (the ViT-S fc1 and qkv); launch_gemm routes there when
// panel_gemm_eligible() (switch "panel").
bool panel_gemm_eligible(const GemmParams& p);
// compute units of the current device (cached)
int cu_count();
hipError_t launch_panel_gemm(const GemmParams& p, hipStream_t st);

// 256x256 phase-pipelined dense GEMM (gemm256.hip) for large token-major
// problems; launch_gemm routes there when gemm256_eligible() (switch "gemm256").
bool gemm256_eligible(const GemmParams& p);
hipError_t launch_gemm256(const GemmParams& p, hipStream_t st);

// ws (optional, attention_split_ws_bytes): fp32 workspace for the split-KV
// path the launcher takes on grids too small to fill the chip (batch 1)
// cfg (optional) = "<waves>[s<split>][g<groups>][r<ring>][q2]" ("8", "4s2",
// "4g2", ...): forces a workgroup shape / split for tests and tuning; nullptr
// or "" = the launch policy.
hipError_t launch_attention(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T,
                            int Tpad, int ldo, hipStream_t st, float* ws = nullptr, size_t ws_bytes = 0,
                            const char* cfg = nullptr);
size_t attention_split_ws_bytes(int B, int H, int T);

// x (fp32) or xh (f16) residual rows -> LayerNorm -> f16 y
hipError_t launch_layernorm(const float* x, h16* y, const float* g, const float* b, int rows, int D,
                            float eps, int T, int skip_cls, hipStream_t st, const h16* xh = nullptr);

// P32 (exact-fp32 engines): the patch rows as fp32 into P32 instead of f16 into P
hipError_t launch_patch_prep_u8(const unsigned char* img, h16* P, float* X, const float* cls_pos, int B, int H, int W,
                                int ph, int pw, int T, int D, float scale, const float* mean3, const float* std3,
                                hipStream_t st, h16* Xh = nullptr, float* lnst = nullptr,
                                const float* cls_st = nullptr, float* P32 = nullptr);
hipError_t launch_depth_postprocess(const float* in, int B, int ih, int iw, float* out, int oh, int ow, float lo,
                                    float hi, hipStream_t st);
hipError_t launch_patch_prep(const float* img, h16* P, float* X, const float* cls_pos, int B, int H,
                             int W, int ph, int pw, int T, int D, hipStream_t st, h16* Xh = nullptr,
                             float* lnst = nullptr, const float* cls_st = nullptr, float* P32 = nullptr);
// fp32 rows -> LayerNorm -> fp32 rows (exact-fp32 engines)
// (T, skip_cls = 1: the cls row of every T-row sequence dropped, the patch
// rows written as the [B*(T-1)][D] NHWC token map -- the taps' final norm)
hipError_t launch_layernorm32(const float* x, float* y, const float* g, const float* b, int rows, int D, float eps,
                              hipStream_t st, int T = 1, int skip_cls = 0);

hipError_t launch_resize(const h16* in, h16* out, int B, int ih, int iw, int C, int oh, int ow,
                         hipStream_t st);

// ---- Depth Pro (depth_pro_ops.hip) ----
// Pyramid levels of the patch encoder input, high-res first: sequences
// l in [first[i], first[i+1]) are the n[i] x n[i] patches of level i
// (row-major), taken with `stride` from the image downsampled by f[i].
struct DpPyramid {
  int nlev = 0, nseq = 0;  // nseq = patches per image
  int first[3] = {0, 0, 0}, n[3] = {0, 0, 0}, stride[3] = {0, 0, 0}, f[3] = {1, 1, 1};
};
// One merged level map: patches (base + r*n + c) of every image, G x G
// tokens each (row 0 of each sequence = cls, dropped), interior edges
// trimmed by pad -> [B][n G - 2 (n-1) pad]^2 NHWC.
struct DpMerge {
  int B = 0, n = 1, G = 0, pad = 0, base = 0, T = 0;
};
hipError_t launch_dp_patch_prep(const float* img, h16* P, int B, int S, int G, const DpPyramid& pyr,
                                hipStream_t st);
hipError_t launch_cls_rows(float* X, const float* cls, int nseq, int T, int D, hipStream_t st);
// g == nullptr: plain fp32 -> f16 copy (raw hook features); else LayerNorm(g, b)
hipError_t launch_merge_tokens(const float* x, h16* y, const float* g, const float* b, int D, const DpMerge& m,
                               float eps, hipStream_t st);
hipError_t launch_fov_final(const h16* in, const float* w, float bias, int K, int B, float* out, hipStream_t st);

// ---- VGGT (vggt_ops.hip) ----
// Token geometry of the q/k rows one qk_norm_rope launch covers: T tokens per
// sequence (rows padded to Tpad), P tokens per frame (T = S * P for global
// attention), the first npre of each frame special (RoPE position (0, 0)),
// the rest a grid gw wide at positions (row + 1, col + 1).
struct RopeGeom {
  int T = 0, Tpad = 0, P = 1, npre = 0, gw = 1;
  float qscale = 1.f, eps = 1e-5f;
};
// special-token rows [0, npre) of every sequence from pre[sets][npre][D]
// (sets 2: set 0 for the first frame of each batch item, 1 for the others)
hipError_t launch_prefix_rows(float* X, const float* pre, int nseq, int T, int npre, int D, int frames, int sets,
                              hipStream_t st);
hipError_t launch_rows_layernorm(float* X, const float* g, const float* b, int nseq, int T, int row0, int D, float eps,
                                 hipStream_t st);
hipError_t launch_qk_norm_rope(h16* q, h16* k, const float* qg, const float* qb, const float* kg, const float* kb,
                               const float* rope_cos, const float* rope_sin, int BH, const RopeGeom& geo,
                               hipStream_t st);
hipError_t launch_tap_concat_ln(const float* xa, const float* xb, h16* y, const float* g, const float* b, int nseq,
                                int T, int npre, int D, float eps, hipStream_t st);

}  // namespace mde
