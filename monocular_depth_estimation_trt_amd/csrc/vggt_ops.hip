// Bandwidth-bound kernels of the VGGT depth path (gfx950):
//   * prefix rows: the special tokens of every sequence of the fp32 residual
//     stream -- DINOv2's cls + pos[0] and 4 registers, or the aggregator's
//     camera + 4 register tokens (set 0 for the first frame of a batch item,
//     set 1 for the others: upstream aggregator.slice_expand_and_flatten)
//   * in-place fp32 LayerNorm of a row range (DINOv2's final norm over the
//     patch tokens, which become the aggregator's frame tokens)
//   * per-head q/k LayerNorm(64) + 2D RoPE on the head-major q / k operands
//     the QKV epilogue wrote, with the attention's q scale applied last
//     (upstream layers/attention.py + layers/rope.py)
//   * the depth head's tap: LayerNorm(2D) over cat(frame_out, global_out) of
//     the patch tokens -> the f16 token map of the 1x1 projections
//     (upstream heads/dpt_head.py _forward_impl: self.norm on
//     aggregated_tokens_list[i][:, :, patch_start_idx:])
#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

// One thread per float4 of a prefix row.  sets == 2: sequence seq uses set
// (seq % frames == 0 ? 0 : 1); sets == 1: every sequence uses set 0.
__global__ void __launch_bounds__(256) prefix_rows_kernel(float* __restrict__ X, const float* __restrict__ pre, int nseq,
                                                          int T, int npre, int D, int frames, int sets) {
  const int q = D >> 2;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)nseq * npre * q) return;
  const int c = (int)(id % q);
  const long long r = id / q;
  const int row = (int)(r % npre);
  const int seq = (int)(r / npre);
  const int set = (sets == 2 && seq % frames != 0) ? 1 : 0;
  const float4 v = reinterpret_cast<const float4*>(pre + ((size_t)set * npre + row) * D)[c];
  reinterpret_cast<float4*>(X + ((size_t)seq * T + row) * D)[c] = v;
}

// One wave per row (seq, t), t in [row0, T); in place.
template <int PER>
__global__ void __launch_bounds__(256) rows_layernorm_kernel(float* __restrict__ X, const float* __restrict__ g,
                                                             const float* __restrict__ bt, int nseq, int T, int row0,
                                                             float eps) {
  constexpr int D = PER * 64;
  const int lane = threadIdx.x & 63;
  const int per_seq = T - row0;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long long)nseq * per_seq) return;
  const int seq = (int)(r / per_seq), t = row0 + (int)(r - (long long)seq * per_seq);
  float* xr = X + ((size_t)seq * T + t) * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = xr[i * 64 + lane];
    s += v[i];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float qv = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float d = v[i] - mean;
    qv += d * d;
  }
  const float rstd = rsqrtf(wave_sum(qv) * (1.0f / D) + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = i * 64 + lane;
    xr[c] = (v[i] - mean) * rstd * g[c] + bt[c];
  }
}

// q / k rows [BH][Tpad][64] f16; 8 lanes per row, lane c of the group owns
// features 8c .. 8c+7 (one 16-byte load/store).  LayerNorm over the 64
// features (shuffles inside the aligned 8-lane group), then RoPE: features
// [0, 32) rotate with the y position, [32, 64) with x; inside each half,
// feature j pairs with j +- 16 -- the lane c ^ 2 of the group, same slot --
// with frequency index j & 15 (upstream rotate_half over duplicated angles).
// Token t of a sequence sits at frame position p = t % P; p < npre are the
// special tokens at (0, 0) (the identity rotation), patch p - npre at
// (row + 1, col + 1) of a grid gw wide.  q is then scaled by qscale (the
// attention's dh^-0.5 log2 e).  All 8 lanes of a group take the same path.
__global__ void __launch_bounds__(256) qk_norm_rope_kernel(f16* __restrict__ q, f16* __restrict__ k,
                                                           const float* __restrict__ qg, const float* __restrict__ qb,
                                                           const float* __restrict__ kg, const float* __restrict__ kb,
                                                           const float* __restrict__ rcos, const float* __restrict__ rsin,
                                                           int BH, RopeGeom geo) {
  const long long gid = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int c = threadIdx.x & 7;
  const long long per = (long long)BH * geo.T;
  if (gid >= 2 * per) return;
  const bool isq = gid < per;
  const long long r = isq ? gid : gid - per;
  const int bh = (int)(r / geo.T), t = (int)(r - (long long)bh * geo.T);
  f16* row = (isq ? q : k) + ((size_t)bh * geo.Tpad + t) * 64 + c * 8;
  const float* gm = (isq ? qg : kg) + c * 8;
  const float* bm = (isq ? qb : kb) + c * 8;
  const f16x8 raw = *reinterpret_cast<const f16x8*>(row);
  float v[8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = (float)raw[j];
    s += v[j];
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  const float mean = s * (1.0f / 64);
  float qv = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] -= mean;
    qv += v[j] * v[j];
  }
  qv += __shfl_xor(qv, 1, 64);
  qv += __shfl_xor(qv, 2, 64);
  qv += __shfl_xor(qv, 4, 64);
  const float rstd = rsqrtf(qv * (1.0f / 64) + geo.eps);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * gm[j] + bm[j];
  const int p = t % geo.P;
  int pos = 0;
  if (p >= geo.npre) {
    const int pp = p - geo.npre;
    pos = (c < 4 ? pp / geo.gw : pp % geo.gw) + 1;
  }
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float partner = __shfl_xor(v[j], 2, 64);
    const int f = ((c & 3) * 8 + j) & 15;
    const float cs = rcos[pos * 16 + f], sn = rsin[pos * 16 + f];
    const float rot = (c & 2) ? partner : -partner;  // first 16 of a half: -x[j+16]; last 16: +x[j-16]
    o[j] = v[j] * cs + rot * sn;
  }
  const float sc = isq ? geo.qscale : 1.f;
  f16x8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (f16)(o[j] * sc);
  *reinterpret_cast<f16x8*>(row) = h;
}

// One wave per output row (seq, patch): LayerNorm over the 2D features of
// cat(xa[row], xb[row]) -> y[seq * np + patch][2D] f16.
template <int PER>
__global__ void __launch_bounds__(256) tap_concat_ln_kernel(const float* __restrict__ xa, const float* __restrict__ xb,
                                                            f16* __restrict__ y, const float* __restrict__ g,
                                                            const float* __restrict__ bt, int nseq, int T, int npre,
                                                            float eps) {
  constexpr int D = PER * 64;
  const int lane = threadIdx.x & 63;
  const int np = T - npre;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long long)nseq * np) return;
  const int seq = (int)(r / np), pi = (int)(r - (long long)seq * np);
  const size_t src = ((size_t)seq * T + npre + pi) * D;
  float va[PER], vb[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    va[i] = xa[src + i * 64 + lane];
    vb[i] = xb[src + i * 64 + lane];
    s += va[i] + vb[i];
  }
  const float mean = wave_sum(s) * (1.0f / (2 * D));
  float qv = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float da = va[i] - mean, db = vb[i] - mean;
    qv += da * da + db * db;
  }
  const float rstd = rsqrtf(wave_sum(qv) * (1.0f / (2 * D)) + eps);
  f16* yr = y + (size_t)r * (2 * D);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = i * 64 + lane;
    yr[c] = (f16)((va[i] - mean) * rstd * g[c] + bt[c]);
    yr[D + c] = (f16)((vb[i] - mean) * rstd * g[D + c] + bt[D + c]);
  }
}

}  // namespace

hipError_t launch_prefix_rows(float* X, const float* pre, int nseq, int T, int npre, int D, int frames, int sets,
                              hipStream_t st) {
  if (nseq <= 0) return hipSuccess;
  if (D % 4 || npre < 1 || npre > T || (sets != 1 && sets != 2) || frames < 1) return hipErrorInvalidValue;
  const long long n = (long long)nseq * npre * (D / 4);
  hipLaunchKernelGGL(prefix_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, pre, nseq, T, npre,
                     D, frames, sets);
  return hipGetLastError();
}

hipError_t launch_rows_layernorm(float* X, const float* g, const float* b, int nseq, int T, int row0, int D, float eps,
                                 hipStream_t st) {
  if (row0 < 0 || row0 >= T) return hipErrorInvalidValue;
  const long long rows = (long long)nseq * (T - row0);
  if (rows <= 0) return hipSuccess;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (D) {
    case 128: hipLaunchKernelGGL(rows_layernorm_kernel<2>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    case 256: hipLaunchKernelGGL(rows_layernorm_kernel<4>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    case 384: hipLaunchKernelGGL(rows_layernorm_kernel<6>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    case 512: hipLaunchKernelGGL(rows_layernorm_kernel<8>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    case 768: hipLaunchKernelGGL(rows_layernorm_kernel<12>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    case 1024: hipLaunchKernelGGL(rows_layernorm_kernel<16>, grid, block, 0, st, X, g, b, nseq, T, row0, eps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_qk_norm_rope(h16* q, h16* k, const float* qg, const float* qb, const float* kg, const float* kb,
                               const float* rope_cos, const float* rope_sin, int BH, const RopeGeom& geo,
                               hipStream_t st) {
  if (BH <= 0 || geo.T <= 0) return hipSuccess;
  if (geo.Tpad < geo.T || geo.P < 1 || geo.T % geo.P || geo.npre < 0 || geo.npre > geo.P || geo.gw < 1 ||
      (geo.P - geo.npre) % geo.gw)
    return hipErrorInvalidValue;
  const long long threads = 2LL * BH * geo.T * 8;
  hipLaunchKernelGGL(qk_norm_rope_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<f16*>(q), reinterpret_cast<f16*>(k), qg, qb, kg, kb, rope_cos, rope_sin, BH, geo);
  return hipGetLastError();
}

hipError_t launch_tap_concat_ln(const float* xa, const float* xb, h16* y, const float* g, const float* b, int nseq,
                                int T, int npre, int D, float eps, hipStream_t st) {
  if (npre < 0 || npre >= T) return hipErrorInvalidValue;
  const long long rows = (long long)nseq * (T - npre);
  if (rows <= 0) return hipSuccess;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  f16* yo = reinterpret_cast<f16*>(y);
#define MDE_TAPLN(PER)                                                                                          \
  case PER * 64:                                                                                                \
    hipLaunchKernelGGL((tap_concat_ln_kernel<PER>), grid, block, 0, st, xa, xb, yo, g, b, nseq, T, npre, eps); \
    break;
  switch (D) {
    MDE_TAPLN(2)
    MDE_TAPLN(4)
    MDE_TAPLN(6)
    MDE_TAPLN(8)
    MDE_TAPLN(12)
    MDE_TAPLN(16)
    default: return hipErrorInvalidValue;
  }
#undef MDE_TAPLN
  return hipGetLastError();
}

}  // namespace mde
