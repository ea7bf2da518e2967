// On-disk layout of a packed engine (DA-V2 or Depth Pro) (written by pack.py, read by
// engine.hip).  Little-endian, fixed-size records.
//
//   [0]            PackHeader   (32 B)
//   [32]           PackConfig   (256 B)
//   [288]          PackTensor x n_tensors (128 B each)
//   [data_offset]  tensor bytes, each at data_offset + PackTensor.offset
//                  (offsets 256-byte aligned)
#pragma once
#include <stdint.h>

namespace mde {

#pragma pack(push, 1)
struct PackHeader {
  char magic[8];  // "MDEPACK1"
  uint32_t version;
  uint32_t n_tensors;
  uint64_t data_offset;
  uint64_t data_bytes;
};
static_assert(sizeof(PackHeader) == 32, "PackHeader");

struct PackConfig {
  int32_t embed_dim, depth, num_heads, mlp_hidden, patch;
  int32_t img_h, img_w, features;
  int32_t out_channels[4];
  int32_t taps[4];
  int32_t head_hidden, metric;
  float max_depth, ln_eps;
  char encoder[16];
  // input preamble (reference core/onnx_tools.py:87-219 add_uint8_input):
  // input_u8 = 1 -> the binding is "image_u8" uint8 NHWC [B,H,W,3] and the
  // engine computes ((float)u / in_scale - in_mean[c]) / in_std[c] in fp32
  int32_t input_u8;
  float in_scale, in_mean[3], in_std[3];
  // model family (0 = Depth Anything V2, 1 = Depth Pro, 2 = VGGT) and the
  // Depth Pro decoder geometry (HF DepthProConfig fields; zero otherwise).  For Depth
  // Pro, img_h/img_w = the fixed 1536 input, patch = 16, vit_size = 384,
  // features = fusion_hidden_size, metric = 0 (ReLU head).
  int32_t family;
  int32_t vit_size, merge_pad, use_fov, fov_layers, fov_k;
  int32_t hooks[2], inter_dims[2], scaled_dims[3];
  // VGGT (family 2): embed_dim / depth / ln_eps above describe the DINOv2
  // patch embedding, taps index the aggregator blocks, metric = 2 (exp head);
  // frames = S (the packed frame count), npre = special tokens per frame (5),
  // aa_depth = frame/global block pairs, agg_eps = aggregator / head LN eps
  int32_t frames, npre, aa_depth;
  float agg_eps;
  // DA-V2: residual stream precision (get_engine precision): 1 = "fp16", the
  // stream kept in f16 as an fp16 TensorRT engine computes it; 0 = "fp32",
  // fp32 stream (Depth Pro / VGGT: always 0)
  int32_t resid_f16;
  // DA-V2: 1 = exact-fp32 encoder (precision "fp32"): fp32 weights *.w32 for
  // the patch embed and the block linears, fp32 activations, fp32 MFMA
  // (fp32.hip); 0 = f16 MFMA operands
  int32_t enc_f32;
  char reserved[52];
};
static_assert(sizeof(PackConfig) == 256, "PackConfig");

struct PackTensor {
  char name[80];
  int32_t dtype;  // 0 f32, 1 f16
  int32_t ndim;
  int32_t dims[4];
  uint64_t offset;
  uint64_t nbytes;
  char reserved[8];
};
static_assert(sizeof(PackTensor) == 128, "PackTensor");
#pragma pack(pop)

constexpr uint32_t kPackVersion = 1;

}  // namespace mde
