/*
 * mde.h -- C ABI of libmde_hip.so, the MI355X (gfx950) monocular depth
 * inference engine (Depth Anything V2 family; Depth Pro).  Plain pointers, sizes and ints only: no torch, no HIP
 * C++ types (streams/events are opaque `void*` = hipStream_t / hipEvent_t).
 *
 * Every function returns 0 (MDE_OK) on success or an mde_status code;
 * mde_last_error() returns a thread-local description of the last failure.
 *
 * Which reference interface each group replaces (reference paths are
 * relative to the upstream repo yester31/Monocular_Depth_Estimation_TRT):
 *
 *   engine        core/common.py:141-312 get_engine() -> trt.ICudaEngine
 *                 (deserialize_cuda_engine, :298-299) and its introspection
 *                 used by core/common_runtime.py:131-175 (num_io_tensors,
 *                 get_tensor_name/shape/dtype/mode, get_tensor_profile_shape)
 *                 Depth Pro: models/depth_pro/onnx2trt.py:94-111 (same engine API,
 *                 outputs "canonical_inverse_depth" + "fov_deg", onnx_export.py:56)
 *                 VGGT: models/vggt/onnx2trt.py:95-107 (input "images" [1,S,3,518,518],
 *                 output "depth", onnx_export.py:125-127)
 *   context       engine.create_execution_context()
 *                 (models/depth_anything_v2/onnx2trt.py:93-94),
 *                 context.set_tensor_address (core/common_runtime.py:272-274),
 *                 context.set_input_shape (onnx2trt.py:99-100),
 *                 context.execute_async_v3 (core/common_runtime.py:269-270),
 *                 context.profiler = IProfiler (tools/profile_model.py:126,
 *                 core/profile.py:30-57)
 *   rt            the cuda-python cudart calls of core/common_runtime.py
 *                 (cudaMallocHost/cudaMalloc :64-73, cudaFree/cudaFreeHost
 *                 :106-108, cudaMemcpyAsync :245-255, cudaStreamCreate/
 *                 Synchronize/Destroy :135,:259,:182, cudaEvent* :220-237)
 *   op            no reference counterpart: the individual TensorRT layers of
 *                 the DA-V2 engine, exposed for per-kernel
 *                 parity tests and for integrators who run parts of the graph.
 */
#ifndef MDE_H_
#define MDE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDE_ABI_VERSION 8

typedef enum {
  MDE_OK = 0,
  MDE_ERR_ARG = 1,     /* bad argument (null pointer, bad size)          */
  MDE_ERR_FILE = 2,    /* packed file missing or unreadable              */
  MDE_ERR_FORMAT = 3,  /* packed file malformed / unsupported version    */
  MDE_ERR_HIP = 4,     /* HIP runtime error                              */
  MDE_ERR_NAME = 5,    /* unknown tensor name                            */
  MDE_ERR_SHAPE = 6,   /* shape outside the engine's profile             */
  MDE_ERR_STATE = 7    /* address not set, context busy, ...             */
} mde_status;

/* Same numbering as tensorrt.DataType for the types used here. */
typedef enum { MDE_FLOAT32 = 0, MDE_FLOAT16 = 1, MDE_UINT8 = 5 } mde_dtype; /* tensorrt.DataType values */

typedef struct mde_engine mde_engine;
typedef struct mde_context mde_context;

typedef struct {
  char name[64];
  int32_t dtype;    /* mde_dtype */
  int32_t is_input; /* 1 = INPUT, 0 = OUTPUT (trt.TensorIOMode) */
  int32_t rank;
  int64_t dims[8];  /* dims[0] = -1: batch is dynamic (see profile shape) */
} mde_io_desc;

typedef struct {
  char encoder[16];
  int32_t embed_dim, depth, num_heads, mlp_hidden, patch;
  int32_t img_h, img_w, features, head_hidden, metric;
  int32_t out_channels[4], taps[4];
  float max_depth, ln_eps;
  int32_t max_batch_hint;
  int64_t weight_bytes;
  int32_t input_format; /* 0: "input" float32 NCHW [B,3,H,W]; 1: "image_u8" uint8 NHWC [B,H,W,3] */
  int32_t family;       /* 0: Depth Anything V2 (io "input" -> "output" [B,H,W]);
                           1: Depth Pro (io "input" [B,3,1536,1536] -> "canonical_inverse_depth"
                              [B,1,1536,1536] and, with the FOV head, "fov_deg" [B]);
                           2: VGGT depth path (io "images" float32 [B,S,3,H,W] in [0,1] ->
                              "depth" [B,S,H,W,1]; S fixed at pack time) */
} mde_engine_info;

/* IProfiler.report_layer_time analogue: one call per launched layer. */
typedef void (*mde_layer_cb)(const char* layer_name, float ms, void* user);

/* ---- library ---------------------------------------------------------- */
int mde_version(void);
const char* mde_last_error(void);
/* Dispatch switches (no reference counterpart: TensorRT picks tactics at build
 * time).  Each starts at its default, is overridden once per process from the
 * environment variable MDE_<NAME>, and can be changed here afterwards; a
 * captured hipGraph keeps the choice it was captured with.  Names (range,
 * default): "splitk" (0-1, 1) split-K of small-grid GEMMs / DPT convs;
 * "lnfold" (0-1, 1) LayerNorm folded into the consumer GEMMs, read at context
 * creation; "conv_narrow" (0-1, 1) narrow conv channel tiles on small grids;
 * "upconv" (0-1, 1) separable upsampling head conv; "gemm256" (0-2, 1) 256^2
 * GEMM tiles (0 never, 1 auto, 2 always); "deep64" (0-1, 1) 4-deep ring for
 * small-grid 64^2 tiles; "w8small" (0-1, 1) 8-wave small-grid 128^2 tiles;
 * "conv_persist" (0-2, 1) persistent 64-channel RCU conv (1: 16 x 16 tiles,
 * 2: 8 x 16); "panel" (0-2, 1) A-stationary panel GEMM for the K = 384
 * qkv / fc1 at large batch (2: also the f16-residual proj); "panel32" (0-1,
 * 0) that GEMM on 32x32x16 MFMAs with the LN fold's mean term in the
 * accumulator's initial value (within 1 f16 ulp of the default); "narrow_resid"
 * (0-1, 1) 32 x 64 whole-K tiles for small-grid residual updates instead of
 * split-K + reduce; "attn16" (0-1, 1) the large-grid attention on 16x16x32
 * MFMAs (same softmax, other summation grouping); "splitk_fused" (0-1, 0) the
 * engines' split-K slices and their in-order reduce as one launch (the last
 * slice of a tile to arrive adds the slots; measured slower); "attn_tail" (0-2, 2)
 * the large-grid attention's partial query blocks dispatched after the full
 * ones (1: work order only, bit-identical; 2: those blocks also split their
 * keys over two wave groups); "resize_fold" (0-1, 1) the DPT fusion blocks' x2
 * resize read on the fly by the next block's residual conv (bit-identical).  The environment variable of a switch is exactly
 * MDE_ + its name upper-cased (MDE_DEEP64, MDE_W8SMALL, ...); a value that is
 * not an integer in range is reported on stderr and ignored.
 * Every setting computes the same depth map within the stated tolerance; the
 * tile switches are bit-identical.  MDE_ERR_NAME: unknown name; MDE_ERR_ARG:
 * value out of range. */
int mde_tuning_set(const char* name, int value);
int mde_tuning_get(const char* name, int* value);

/* ---- engine (replaces get_engine / ICudaEngine) ----------------------- */
int mde_engine_load(const char* packed_path, int device, mde_engine** out);
int mde_engine_load_memory(const void* data, size_t nbytes, int device, mde_engine** out);
int mde_engine_destroy(mde_engine* eng);
int mde_engine_get_info(const mde_engine* eng, mde_engine_info* out);
int mde_engine_num_io(const mde_engine* eng, int* n);
int mde_engine_io_desc(const mde_engine* eng, int index, mde_io_desc* out);
/* which: 0 = min, 1 = opt, 2 = max shape of the dynamic-batch profile */
int mde_engine_profile_shape(const mde_engine* eng, const char* name, int which, int64_t* dims, int* rank);

/* ---- execution context (replaces IExecutionContext) ------------------- */
int mde_context_create(mde_engine* eng, int max_batch, mde_context** out);
int mde_context_destroy(mde_context* ctx);
int mde_context_set_tensor_address(mde_context* ctx, const char* name, void* device_ptr);
int mde_context_set_input_shape(mde_context* ctx, const char* name, const int64_t* dims, int rank);
int mde_context_get_tensor_shape(const mde_context* ctx, const char* name, int64_t* dims, int* rank);
/* Asynchronous: enqueues the whole forward on `stream` (hipStream_t). */
int mde_context_enqueue(mde_context* ctx, void* stream);
/* 1 (default): capture the forward into a hipGraph per (batch, addresses)
 * and replay it; 0: launch every kernel eagerly. */
int mde_context_set_graph_mode(mde_context* ctx, int enable);
/* Non-null cb: enqueue runs eagerly with a hipEvent pair per layer,
 * synchronizes `stream` at the end and reports each layer's time. */
int mde_context_set_profiler(mde_context* ctx, mde_layer_cb cb, void* user);
int mde_context_workspace_bytes(const mde_context* ctx, size_t* bytes);

/* ---- HIP runtime helpers (replaces cuda-python cudart) ---------------- */
int mde_rt_device_count(int* n);
int mde_rt_set_device(int device);
int mde_rt_device_name(int device, char* buf, int buflen);
int mde_rt_malloc(void** ptr, size_t bytes);
int mde_rt_free(void* ptr);
int mde_rt_malloc_host(void** ptr, size_t bytes);
int mde_rt_free_host(void* ptr);
int mde_rt_memcpy_htod_async(void* dst, const void* src, size_t bytes, void* stream);
int mde_rt_memcpy_dtoh_async(void* dst, const void* src, size_t bytes, void* stream);
int mde_rt_memcpy_dtod_async(void* dst, const void* src, size_t bytes, void* stream);
int mde_rt_memset_async(void* dst, int value, size_t bytes, void* stream);
int mde_rt_stream_create(void** stream);
int mde_rt_stream_destroy(void* stream);
int mde_rt_stream_synchronize(void* stream);
int mde_rt_device_synchronize(void);
int mde_rt_event_create(void** event);
int mde_rt_event_destroy(void* event);
int mde_rt_event_record(void* event, void* stream);
int mde_rt_event_elapsed_ms(float* ms, void* start, void* end);

/* ---- kernel-level entry points ---------------------------------------- */
/* All tensors are device pointers.  f16 = IEEE half.  Weights W are
 * [Npad][ldw] f16 row-major (K contiguous), rows >= N zero, ldw % 64 == 0,
 * ldw >= K rounded up to 64, Npad a multiple of 128; N % 8 == 0.  Activation maps are
 * NHWC f16.  act: 0 none, 1 ReLU, 2 GELU(erf). */
/* The same over an f16 residual stream (precision "fp16" engines): x_f16 [rows][dim]. */
int mde_op_layernorm_f16(const void* x_f16, void* y_f16, const float* gamma, const float* beta, int rows, int dim,
                         float eps, int tokens, int skip_cls, void* stream);
int mde_op_layernorm(const float* x, void* y_f16, const float* gamma, const float* beta, int rows, int dim,
                     float eps, int tokens, int skip_cls, void* stream);
int mde_op_linear(const void* a_f16, int lda, const void* w_f16, int ldw, int m, int n, int k,
                  const float* bias, int act, void* out_f16, int ldo, void* stream);
int mde_op_linear_residual(const void* a_f16, int lda, const void* w_f16, int ldw, int m, int n, int k,
                           const float* bias, const float* layer_scale, float* x32, int ldx, void* stream);
int mde_op_qkv(const void* a_f16, const void* w_f16, int ldw, const float* bias, int batch, int tokens,
               int heads, int tokens_pad, float q_scale, void* q_f16, void* k_f16, void* vt_f16, void* stream);
/* mde_op_linear_residual over an f16 residual stream xh [m][ldx] (precision "fp16" engines):
 * xh += layer_scale * (a W^T + bias), one rounding to f16.  ln_partials (optional, n % 32 == 0):
 * fp32 [n/32][m][2] (slice-major) = per 32-column slice and row, the sum of the f16 values written
 * and their squared deviations from the slice mean -- the producer half of the folded LayerNorm (reference: the norm1 / norm2 after every
 * residual add of the DINOv2 blocks, upstream Block.forward). */
int mde_op_linear_residual_f16(const void* a_f16, int lda, const void* w_f16, int ldw, int m, int n, int k,
                               const float* bias, const float* layer_scale, void* xh_f16, int ldx, float* ln_partials,
                               void* stream);
/* The consumer half: out = act(LayerNorm(x) W^T + b) computed as act(rstd * (x Wg^T - mean * c1) + c2)
 * over the raw f16 rows x [m][k] (k % 32 == 0), with Wg = W * gamma (column k scaled by gamma[k]),
 * c1[n] = sum_k Wg[n][k], c2 = b + W beta, and mean / rstd (fp32, eps) from ln_partials [k/32][m][2] (k <= 1024). */
int mde_op_linear_lnfold(const void* x_f16, const float* ln_partials, float eps, const void* wg_f16, int ldw,
                         const float* c1, const float* c2, int m, int n, int k, int act, void* out_f16, int ldo,
                         void* stream);
/* mde_op_qkv with the LayerNorm folded in the same way (the DA-V2 engines' block qkv: norm1 ->
 * qkv, reference depth_anything_v2/dinov2_layers/block.py attn(norm1(x))): x [batch*tokens][64 heads]
 * raw f16 rows, ln_partials [heads*2][batch*tokens][2], wg = W * gamma, c1 / c2 as above. */
int mde_op_qkv_lnfold(const void* x_f16, const float* ln_partials, float eps, const void* wg_f16, int ldw,
                      const float* c1, const float* c2, int batch, int tokens, int heads, int tokens_pad,
                      float q_scale, void* q_f16, void* k_f16, void* vt_f16, void* stream);
/* q pre-multiplied by dh^-0.5 * log2(e) (scores in log2 units, as mde_op_qkv writes with
 * q_scale = 0.125 * log2(e)); k/q [B*H][tokens_pad][64], vt [B*H][64][tokens_pad] with key t
 * stored at column vt_pos(t) = t with bits 2 and 3 swapped, (t & ~12) | (t & 4) << 1 | (t & 8) >> 1
 * (the layout mde_op_qkv writes); ldo % 8 == 0 and o 16-B aligned. */
int mde_op_attention(const void* q_f16, const void* k_f16, const void* vt_f16, void* o_f16, int batch, int heads,
                     int tokens, int tokens_pad, int ldo, void* stream);
/* The same with an fp32 workspace for the split-KV path the launcher takes when the (head, query
 * block) grid is too small to fill the chip (batch 1); mde_op_attention_ws_bytes gives its size. */
int mde_op_attention_ws(const void* q_f16, const void* k_f16, const void* vt_f16, void* o_f16, int batch, int heads,
                        int tokens, int tokens_pad, int ldo, void* ws, size_t ws_bytes, void* stream);
size_t mde_op_attention_ws_bytes(int batch, int heads, int tokens);
/* mde_op_attention_ws with an explicit launch configuration (tests / tuning; no reference
 * counterpart): cfg = "<waves>[s<split>][g<groups>][r<ring>][q2][m]", e.g. "8" (256-query
 * workgroups), "8m" (the same on 16x16x32 MFMAs, unsplit 4 / 8 waves only), "4s2" (split-KV over two workgroups + merge kernel, needs ws), "4g2" (two key
 * groups of 64 queries inside one workgroup, merged through LDS); NULL or "" = the launcher's
 * policy. */
int mde_op_attention_cfg(const void* q_f16, const void* k_f16, const void* vt_f16, void* o_f16, int batch, int heads,
                         int tokens, int tokens_pad, int ldo, const char* cfg, void* ws, size_t ws_bytes,
                         void* stream);
/* Exact-fp32 kernels of precision "fp32" engines (fp32.hip; v_mfma_f32_16x16x4_f32 /
 * v_mfma_f32_32x32x2_f32, fp32 operands and accumulation): weights fp32 [Npad][ldw] (ldw % 32 == 0,
 * zero padded, Npad a multiple of 128), activations fp32 with lda % 4 == 0.  linear32: out = act(a w^T
 * + bias); linear_residual32: x32 += layer_scale * (a w^T + bias); qkv32: q (times q_scale) / k / v
 * fp32 [batch*heads][tokens_pad][64]; attention32: softmax over those (q pre-scaled by dh^-0.5 *
 * log2 e) -> o fp32 [batch*tokens][ldo]. */
int mde_op_linear32(const float* a, int lda, const float* w, int ldw, int m, int n, int k, const float* bias, int act,
                    float* out, int ldo, void* stream);
int mde_op_linear_residual32(const float* a, int lda, const float* w, int ldw, int m, int n, int k,
                             const float* bias, const float* layer_scale, float* x32, int ldx, void* stream);
int mde_op_qkv32(const float* a, const float* w, int ldw, const float* bias, int batch, int tokens, int heads,
                 int tokens_pad, float q_scale, float* q, float* k, float* v, void* stream);
int mde_op_attention32(const float* q, const float* k, const float* v, float* o, int batch, int heads, int tokens,
                       int tokens_pad, int ldo, void* stream);
/* The exact-fp32 DPT head's kernels (fp32.hip; precision "fp32" engines since ABI 7).  conv3x3_32: out
 * = act(conv3x3(relu_in ? ReLU(in) : in) + bias) + res0 + res1 over fp32 NHWC maps [batch][h][w][cin]
 * (cin % 4 == 0), pad 1, stride 1 or 2, weights fp32 [cout_pad][ldw] in (ky, kx, ci) order (ldw % 32
 * == 0, >= 9 cin rounded up to 32; cout % 4 == 0), res0 / res1 optional maps shaped like out --
 * reference: DPTHead's resConfUnit / layerN_rn / output_conv convs (upstream dpt.py), the reference's
 * fp32 TensorRT build (core/common.py:141-144).  conv_transpose32: ConvTranspose2d(k = s = stride)
 * as a GEMM with a pixel-shuffle epilogue, weights [(dy s + dx) cout + co][ldw] -- DPTHead
 * resize_layers 0/1.  resize32: bilinear, align_corners=True, fp32 NHWC (c % 4 == 0) --
 * F.interpolate in FeatureFusionBlock / the head. */
int mde_op_conv3x3_32(const float* in, int batch, int h, int w, int cin, const float* wt, int ldw, int cout,
                      int stride, int relu_in, const float* bias, int act, const float* res0, const float* res1,
                      float* out, void* stream);
int mde_op_conv_transpose32(const float* in, int batch, int h, int w, int cin, const float* wt, int ldw, int cout,
                            int stride, const float* bias, float* out, void* stream);
int mde_op_resize32(const float* in, int batch, int h, int w, int c, int oh, int ow, float* out, void* stream);
int mde_op_patch_embed(const float* img, int batch, int h, int w, const void* w_f16, int ldw, const float* bias,
                       const float* pos_patch, const float* cls_pos, int dim, void* patch_scratch_f16,
                       float* x32, void* stream);
int mde_op_conv3x3(const void* in_f16, int batch, int h, int w, int cin, const void* w_f16, int ldw, int cout,
                   int stride, int relu_in, const float* bias, int act, const void* res0_f16,
                   const void* res1_f16, void* out_f16, void* stream);
/* mde_op_conv3x3 / mde_op_linear (E_STORE) with an fp32 split-K workspace of
 * ws_floats elements: grids too small to fill the chip cut the K loop into
 * slices (partials summed in slice order, then the epilogue); *slices (may be
 * null) receives the slice count taken, 1 = no split.  The engine gives its
 * DPT convs such a workspace (small batches). */
int mde_op_conv3x3_ws(const void* in_f16, int batch, int h, int w, int cin, const void* w_f16, int ldw, int cout,
                      int stride, int relu_in, const float* bias, int act, const void* res0_f16,
                      const void* res1_f16, void* out_f16, float* ws, size_t ws_floats, int* slices, void* stream);
int mde_op_linear_ws(const void* a_f16, int lda, const void* w_f16, int ldw, int m, int n, int k, const float* bias,
                     int act, void* out_f16, int ldo, float* ws, size_t ws_floats, int* slices, void* stream);
int mde_op_conv3x3_up(const void* in_f16, int batch, int sh, int sw, int cin, int uh, int uw, const void* w_f16,
                      int ldw, int cout, const float* bias, int act, void* out_f16, void* stream);
int mde_op_conv_transpose(const void* in_f16, int batch, int h, int w, int cin, const void* w_f16, int ldw,
                          int cout, int stride, const float* bias, void* out_f16, void* stream);
int mde_op_resize_bilinear(const void* in_f16, int batch, int ih, int iw, int c, int oh, int ow, void* out_f16,
                           void* stream);
int mde_op_depth_head(const void* in_f16, int batch, int sh, int sw, int cin, int uh, int uw, const void* w_f16,
                      int ldw, const float* bias, const float* w2, float b2, int metric, float max_depth,
                      float* out_f32, void* stream);
/* uint8 NHWC image [batch][h][w][3] -> the patch-embed operand [batch*(h/14)*(w/14)][672] f16
 * (patch-major, channel, row, 16-wide padded column), computing ((float)u / scale - mean[c]) / std[c]
 * in fp32 (the ONNX preamble of reference core/onnx_tools.py:175-199: Cast, Div, Sub, Div). */
int mde_op_patch_prep_u8(const unsigned char* img_u8, int batch, int h, int w, float scale, const float* mean3,
                         const float* std3, void* patches_f16, void* stream);
/* Post-process (reference models/depth_anything_v2/onnx2trt.py:111-117): bilinear
 * align_corners=True resize of fp32 depth [batch][ih][iw] to [batch][oh][ow], then clamp to [lo, hi]. */
int mde_op_depth_postprocess(const float* depth, int batch, int ih, int iw, float* out, int oh, int ow, float lo,
                             float hi, void* stream);
/* Depth Pro pyramid patches (upstream DepthProEncoder._create_pyramid + _split, reference engine input
 * "input"): fp32 NCHW image [batch][3][size][size] (size = 4 * 384) -> f16 patch-embed rows
 * [nseq * batch * 576][768] ((c, py, px) order), sequence s = patch * batch + image with the 25
 * x1 patches (stride 288) first, then the 9 x0.5 patches (stride 192), then the x0.25 image;
 * downsampling = bilinear, align_corners=False, computed on the fly. */
int mde_op_dp_pyramid_patches(const float* img, int batch, int size, void* patches_f16, void* stream);
/* Merge encoder rows x32 [.. sequences][tokens][dim] (row 0 of each sequence = cls, dropped) of
 * the n x n patches (base + r*n + c) * batch + b into an NHWC f16 map [batch][side][side][dim],
 * side = n*g - 2(n-1)*pad, trimming `pad` rows/cols on interior patch edges (upstream _merge);
 * gamma/beta non-null: LayerNorm(eps) fused into the gather, else a plain fp32 -> f16 copy. */
int mde_op_merge_tokens(const float* x32, int batch, int tokens, int dim, int n, int g, int pad, int base,
                        const float* gamma, const float* beta, float eps, void* out_f16, void* stream);
/* VGGT attention prologue (upstream vggt layers/attention.py q_norm / k_norm + layers/rope.py
 * RotaryPositionEmbedding2D, base 100), in place on the head-major rows q/k [bh][tokens_pad][64]
 * f16 (the layout mde_op_qkv writes): LayerNorm(64, eps) with q_gamma/q_beta resp. k_gamma/k_beta,
 * then 2D RoPE -- token t sits at frame position p = t % frame_tokens; p < npre is at RoPE
 * position (0, 0), patch p - npre at (row + 1, col + 1) of a grid grid_w wide; features [0, 32)
 * rotate with the row, [32, 64) with the column (rotate_half inside each half); rope_cos /
 * rope_sin are fp32 [>= max position + 1][16] tables of angle(pos, j) = pos * 100^(-j/16) --
 * and finally q *= q_scale.  Rows >= tokens are not touched. */
int mde_op_qk_norm_rope(void* q_f16, void* k_f16, const float* q_gamma, const float* q_beta, const float* k_gamma,
                        const float* k_beta, int bh, int tokens, int tokens_pad, int frame_tokens, int npre,
                        int grid_w, const float* rope_cos, const float* rope_sin, float q_scale, float eps,
                        void* stream);
/* VGGT depth-head tap (upstream heads/dpt_head.py: self.norm over aggregated_tokens_list[i]
 * [:, :, patch_start_idx:], the list entries being cat(frame_out, global_out)): LayerNorm(2*dim,
 * eps) over cat(xa[row], xb[row]) for the patch rows npre .. tokens-1 of each of nseq sequences
 * (xa, xb fp32 [nseq][tokens][dim]) -> f16 [nseq * (tokens - npre)][2*dim]. */
int mde_op_tap_concat_ln(const float* xa, const float* xb, int nseq, int tokens, int npre, int dim,
                         const float* gamma, const float* beta, float eps, void* out_f16, void* stream);
#ifdef __cplusplus
}
#endif

#endif /* MDE_H_ */
