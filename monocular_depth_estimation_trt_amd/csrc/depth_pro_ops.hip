// Bandwidth-bound kernels of the Depth Pro forward (gfx950):
//   * pyramid patch im2col: the fp32 NCHW 1536^2 image -> f16 patch-embed
//     rows of all 35 384^2 patches of the x1 / x0.5 / x0.25 pyramid, the
//     bilinear(align_corners=False) downsample computed on the fly
//     (reference: upstream DepthProEncoder._create_pyramid + _split, restated
//     by HF:models/depth_pro/modeling_depth_pro.py:238-272, 74-88)
//   * cls rows of a residual stream (cls + pos[0])
//   * token merge: encoder rows -> NHWC feature map, dropping the cls token
//     and the `pad` rows/cols on interior patch edges, optionally with the
//     encoder's final LayerNorm fused in (HF:91-217 reshape_features +
//     merge_patches; the bilinear resize after it is the identity at the
//     1536 geometry, which the engine checks at load)
//   * the FOV head's last valid conv (a k x k x C dot product per image)
#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

constexpr int PS = 16;             // ViT patch size
constexpr int PROW = 3 * PS * PS;  // patch-embed K (768), (c, py, px) order

// One thread per (sequence, token, channel, patch row, 8-pixel half): eight
// output pixels, one 16-byte store.  Sequence s = l * B + b (HF's unfold
// order: patch-major, batch-minor; l runs over the high-res level first).
__global__ void __launch_bounds__(256) dp_patch_prep_kernel(const float* __restrict__ img, f16* __restrict__ P,
                                                            int B, int S, int G, DpPyramid pyr) {
  const int per_tok = 3 * PS * 2;
  const long long ntok = (long long)pyr.nseq * B * G * G;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= ntok * per_tok) return;
  const long long tokid = id / per_tok;
  const int r = (int)(id - tokid * per_tok);
  const int c = r / (2 * PS), py = (r >> 1) % PS, half = r & 1;
  const int GG = G * G;
  const long long seq = tokid / GG;
  const int tok = (int)(tokid - seq * GG);
  const int ty = tok / G, tx = tok - (tok / G) * G;
  const int l = (int)(seq / B), b = (int)(seq - (long long)l * B);
  int lev = 0;
  while (lev + 1 < pyr.nlev && l >= pyr.first[lev + 1]) ++lev;
  const int idx = l - pyr.first[lev], n = pyr.n[lev], f = pyr.f[lev];
  const int pr = idx / n, pc = idx - (idx / n) * n;
  const int Y = pr * pyr.stride[lev] + ty * PS + py;
  const int X0 = pc * pyr.stride[lev] + tx * PS + half * 8;
  const float* plane = img + ((size_t)b * 3 + c) * S * S;
  f16x8 v;
  if (f == 1) {
    const float* src = plane + (size_t)Y * S + X0;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (f16)src[j];
  } else {
    // bilinear, align_corners=False, scale f: src = f (dst + 0.5) - 0.5 =
    // f dst + (f - 1) / 2 -> taps (f dst + (f-2)/2, +1), lambda 0.5 each way
#pragma clang fp contract(off)
    const int y0 = f * Y + (f - 2) / 2;
    const float* r0 = plane + (size_t)y0 * S;
    const float* r1 = r0 + S;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int x0 = f * (X0 + j) + (f - 2) / 2;
      const float a = 0.5f * (0.5f * r0[x0] + 0.5f * r0[x0 + 1]);
      const float d = 0.5f * (0.5f * r1[x0] + 0.5f * r1[x0 + 1]);
      v[j] = (f16)(a + d);
    }
  }
  *reinterpret_cast<f16x8*>(P + tokid * PROW + c * PS * PS + py * PS + half * 8) = v;
}

__global__ void __launch_bounds__(256) cls_rows_kernel(float* __restrict__ X, const float* __restrict__ cls, int nseq,
                                                       int T, int D) {
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)nseq * D) return;
  const int s = (int)(id / D), d = (int)(id - (long long)s * D);
  X[(size_t)s * T * D + d] = cls[d];
}

// One wave per output map pixel (b, Y, X) of a merged level map; source row =
// token (ty, tx) of patch (r, c) of the level, sequence (base + r n + c) B + b.
template <int PER, bool LN>
__global__ void __launch_bounds__(256) merge_tokens_kernel(const float* __restrict__ x, f16* __restrict__ y,
                                                           const float* __restrict__ g, const float* __restrict__ bt,
                                                           DpMerge m, float eps) {
  constexpr int D = PER * 64;
  const int lane = threadIdx.x & 63;
  const long long pix = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int HW = m.n * m.G - 2 * (m.n - 1) * m.pad;
  if (pix >= (long long)m.B * HW * HW) return;
  const int X = (int)(pix % HW);
  const long long q = pix / HW;
  const int Y = (int)(q % HW), b = (int)(q / HW);
  auto split = [&](int v, int& pidx, int& t) {
    const int first = m.G - m.pad, mid = m.G - 2 * m.pad;
    if (m.n == 1 || v < first) {
      pidx = 0;
      t = v;
      return;
    }
    const int k = v - first;
    pidx = 1 + k / mid;
    if (pidx > m.n - 1) pidx = m.n - 1;
    t = m.pad + k - (pidx - 1) * mid;
  };
  int pr, ty, pc, tx;
  split(Y, pr, ty);
  split(X, pc, tx);
  const long long seq = (long long)(m.base + pr * m.n + pc) * m.B + b;
  const float* xr = x + ((size_t)seq * m.T + 1 + ty * m.G + tx) * D;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = xr[i * 64 + lane];
  f16* yr = y + (size_t)pix * D;
  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) s += v[i];
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
      yr[c] = (f16)((v[i] - mean) * rstd * g[c] + bt[c]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) yr[i * 64 + lane] = (f16)v[i];
  }
}

__global__ void __launch_bounds__(256) fov_final_kernel(const f16* __restrict__ in, const float* __restrict__ w,
                                                        float bias, int K, float* __restrict__ out) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const f16* src = in + (size_t)b * K;
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += (float)src[i] * w[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[b] = bias + ((red[0] + red[1]) + (red[2] + red[3]));
}

}  // namespace

hipError_t launch_dp_patch_prep(const float* img, h16* P, int B, int S, int G, const DpPyramid& pyr,
                                hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (pyr.nlev < 1 || pyr.nlev > 3 || G * PS > S) return hipErrorInvalidValue;
  for (int i = 0; i < pyr.nlev; ++i) {
    const int f = pyr.f[i];
    if (f != 1 && f != 2 && f != 4) return hipErrorInvalidValue;
    // the last sample of the level must stay inside the (downsampled) image
    const int last = (pyr.n[i] - 1) * pyr.stride[i] + G * PS;
    if (last * f > S) return hipErrorInvalidValue;
  }
  const long long n = (long long)pyr.nseq * B * G * G * 3 * PS * 2;
  hipLaunchKernelGGL(dp_patch_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, img,
                     reinterpret_cast<f16*>(P), B, S, G, pyr);
  return hipGetLastError();
}

hipError_t launch_cls_rows(float* X, const float* cls, int nseq, int T, int D, hipStream_t st) {
  const long long n = (long long)nseq * D;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cls_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, cls, nseq, T, D);
  return hipGetLastError();
}

hipError_t launch_merge_tokens(const float* x, h16* y, const float* g, const float* b, int D, const DpMerge& m,
                               float eps, hipStream_t st) {
  if (m.n < 1 || m.G < 1 || m.pad < 0 || 2 * m.pad >= m.G || (m.n == 1 && m.pad != 0) || m.T < m.G * m.G + 1)
    return hipErrorInvalidValue;
  const bool ln = g != nullptr;
  if (ln && !b) return hipErrorInvalidValue;
  const int HW = m.n * m.G - 2 * (m.n - 1) * m.pad;
  const long long pix = (long long)m.B * HW * HW;
  if (pix <= 0) return hipSuccess;
  dim3 grid((unsigned)((pix + 3) / 4)), block(256);
  f16* yo = reinterpret_cast<f16*>(y);
#define MDE_MERGE(PER)                                                                                   \
  case PER * 64:                                                                                         \
    if (ln) hipLaunchKernelGGL((merge_tokens_kernel<PER, true>), grid, block, 0, st, x, yo, g, b, m, eps);  \
    else hipLaunchKernelGGL((merge_tokens_kernel<PER, false>), grid, block, 0, st, x, yo, g, b, m, eps);  \
    break;
  switch (D) {
    MDE_MERGE(2)
    MDE_MERGE(4)
    MDE_MERGE(6)
    MDE_MERGE(12)
    MDE_MERGE(16)
    default: return hipErrorInvalidValue;
  }
#undef MDE_MERGE
  return hipGetLastError();
}

hipError_t launch_fov_final(const h16* in, const float* w, float bias, int K, int B, float* out, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (K <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fov_final_kernel, dim3(B), dim3(256), 0, st, reinterpret_cast<const f16*>(in), w, bias, K, out);
  return hipGetLastError();
}

}  // namespace mde
