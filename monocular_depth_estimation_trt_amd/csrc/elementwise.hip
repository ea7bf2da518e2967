// Bandwidth-bound kernels of the DA-V2 forward (gfx950):
//   * LayerNorm over D of the fp32 residual stream -> f16 (block norm1/norm2,
//     SURVEY.md 8a a8; the final `norm` of the 4 taps with the cls row dropped
//     and the token map written as NHWC, a13)
//   * patch im2col: fp32 NCHW image -> f16 patch rows [B*np][3*14*16] (kx
//     padded 14->16 so every 8-element K chunk is 16-byte aligned), plus the
//     cls row of the residual stream (cls + pos[0]) (a6, a7)
//   * bilinear resize, align_corners=True, NHWC f16 (a17 fusion upsample)
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

// One wave per row; PER = D/64 elements per lane, lane-strided (coalesced).
// XT = float (fp32 residual stream) or f16 (f16 stream); statistics in fp32.
template <int PER, class XT, class YT = f16>
__global__ void __launch_bounds__(256) layernorm_kernel(const XT* __restrict__ x, YT* __restrict__ y,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ bt, int rows, float eps,
                                                        int T, int skip_cls) {
  constexpr int D = PER * 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  int orow = row;
  if (skip_cls) {
    const int b = row / T, t = row - (row / T) * T;
    if (t == 0) return;
    orow = b * (T - 1) + t - 1;
  }
  const XT* xr = x + (size_t)row * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = (float)xr[i * 64 + lane];
    s += v[i];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  YT* yr = y + (size_t)orow * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = i * 64 + lane;
    yr[c] = (YT)((v[i] - mean) * rstd * g[c] + bt[c]);
  }
}

// f16 residual rows: 16 lanes per row, 4 rows per wave, 16 rows per
// workgroup; a lane owns C8/16 chunks of 8 consecutive columns (16-B loads
// and stores, all issued before the reduction); statistics in fp32 over
// xor-shuffles inside the 16-lane group.  D = 8 * C8, C8 % 16 == 0.
MDE_DEV float sum16(float v) {
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

template <int C8>
__global__ void __launch_bounds__(256) layernorm_h8_kernel(const f16* __restrict__ x, f16* __restrict__ y,
                                                           const float* __restrict__ g, const float* __restrict__ bt,
                                                           int rows, float eps, int T, int skip_cls) {
  constexpr int D = C8 * 8, PER = C8 / 16;
  static_assert(C8 % 16 == 0, "row width");
  const int l16 = threadIdx.x & 15;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= rows) return;  // whole 16-lane groups leave together
  int orow = row;
  if (skip_cls) {
    const int b = row / T, t = row - (row / T) * T;
    if (t == 0) return;
    orow = b * (T - 1) + t - 1;
  }
  const f16* xr = x + (size_t)row * D;
  f16x8 h[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) h[i] = *reinterpret_cast<const f16x8*>(xr + (i * 16 + l16) * 8);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (float)h[i][j];
  const float mean = sum16(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (float)h[i][j] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(sum16(q) * (1.0f / D) + eps);
  f16* yr = y + (size_t)orow * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = (i * 16 + l16) * 8;
    const float4 g0 = *reinterpret_cast<const float4*>(g + c), g1 = *reinterpret_cast<const float4*>(g + c + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(bt + c), b1 = *reinterpret_cast<const float4*>(bt + c + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f16)(((float)h[i][j] - mean) * rstd * gg[j] + bb[j]);
    *reinterpret_cast<f16x8*>(yr + c) = o;
  }
}

#ifndef MDE_RESIZE_F16
#define MDE_RESIZE_F16 1  // NHWC f16 resize blend in packed f16 (0: fp32 blend, A/B)
#endif

constexpr int PK = 3 * 14 * 16;  // patch row length (K of the patch-embed GEMM)

// 8 patch-row values (kx half) -> P: f16x8, or two float4 (exact-fp32 engines)
template <class PT>
MDE_DEV void store8(PT* dst, const float (&v)[8]) {
  if constexpr (std::is_same<PT, float>::value) {
    reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    f16x8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (f16)v[j];
    *reinterpret_cast<f16x8*>(dst) = h;
  }
}

template <class PT>
__global__ void __launch_bounds__(256) patch_prep_kernel(const float* __restrict__ img, PT* __restrict__ P,
                                                         float* __restrict__ X, const float* __restrict__ cls_pos,
                                                         int B, int H, int W, int ph, int pw, int T, int D,
                                                         f16* __restrict__ Xh, float* __restrict__ lnst,
                                                         const float* __restrict__ cls_st) {
  const long long np = (long long)ph * pw;
  // one thread per (image, channel, image row, patch column): the row's 14
  // pixels of that patch (56 B; consecutive threads read consecutive pixel
  // runs, so a wave reads whole image rows) -> the patch's 16-wide kernel row
  // (14 values + 2 zeros).  Round 6: the input is read once (155 MB at B =
  // 48); the previous (patch, row, half) order fetched 269 MB.
  const int rows = ph * 14;
  const long long nchunk = (long long)B * 3 * rows * pw;
  long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id < nchunk) {
    int px, y, c, b;
    if (nchunk < (1LL << 31)) {  // 32-bit index split (a 64-bit divide is emulated)
      const unsigned u = (unsigned)id, q = u / (unsigned)pw;
      px = (int)(u - q * (unsigned)pw);
      const unsigned q2 = q / (unsigned)rows;
      y = (int)(q - q2 * (unsigned)rows);
      b = (int)(q2 / 3u);
      c = (int)(q2 - (unsigned)b * 3u);
    } else {
      const long long q = id / pw;
      px = (int)(id - q * pw);
      const long long q2 = q / rows;
      y = (int)(q - q2 * rows);
      b = (int)(q2 / 3);
      c = (int)(q2 - (long long)b * 3);
    }
    const int py = y / 14, ky = y - py * 14;
    const float* src = img + (((size_t)b * 3 + c) * H + y) * W + px * 14;
    float v[16];
    if ((W & 1) == 0) {  // 8-B aligned pixel runs
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const float2 t = *reinterpret_cast<const float2*>(src + 2 * j);
        v[2 * j] = t.x;
        v[2 * j + 1] = t.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 14; ++j) v[j] = src[j];
    }
    v[14] = v[15] = 0.0f;
    PT* dst = P + ((long long)b * np + (long long)py * pw + px) * PK + c * 224 + ky * 16;
    const float* lo = v;
    const float* hi = v + 8;
    store8(dst, *reinterpret_cast<const float(*)[8]>(lo));
    store8(dst + 8, *reinterpret_cast<const float(*)[8]>(hi));
    return;
  }
  id -= nchunk;
  if (id < (long long)B * D) {
    const int b = (int)(id / D), d = (int)(id - (long long)(id / D) * D);
    if (Xh) Xh[(size_t)b * T * D + d] = (f16)cls_pos[d];
    else X[(size_t)b * T * D + d] = cls_pos[d];
    return;
  }
  id -= (long long)B * D;
  // the cls rows' LayerNorm partials (folded LN, GemmParams::lnst_out): the
  // row is the same f16 vector in every image, its partials come packed
  if (lnst && id < (long long)B * (D / 16)) {
    const int per = D / 16, b = (int)(id / per), k = (int)(id - (long long)b * per);
    lnst[((size_t)(k >> 1) * B * T + (size_t)b * T) * 2 + (k & 1)] = cls_st[k];
  }
}

// uint8 NHWC variant of patch_prep_kernel: the reference's uint8 preamble
// (core/onnx_tools.py:175-199: Cast -> Div(scale) -> Sub(mean) -> Div(std),
// all fp32) fused into the patch gather.  One thread per (patch, kernel row,
// 8-column half): 8 pixels x 3 channels, three 16-byte chunk stores.  The
// IEEE ops are spelled out (__fdiv_rn / __fsub_rn) so no FMA contraction
// changes the bits against the host preprocessing.
struct InNorm {
  float scale, mean[3], stdv[3];
};

template <class PT>
__global__ void __launch_bounds__(256) patch_prep_u8_kernel(const unsigned char* __restrict__ img, PT* __restrict__ P,
                                                            float* __restrict__ X, const float* __restrict__ cls_pos,
                                                            int B, int H, int W, int ph, int pw, int T, int D,
                                                            InNorm nrm, f16* __restrict__ Xh, float* __restrict__ lnst,
                                                            const float* __restrict__ cls_st) {
  const long long np = (long long)ph * pw;
  const long long nchunk = (long long)B * np * 28;  // 14 rows x 2 halves
  long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id < nchunk) {
    const long long patch = id / 28;
    const int r = (int)(id - patch * 28);
    const int ky = r >> 1, half = r & 1;
    const int b = (int)(patch / np);
    const int pi = (int)(patch - (long long)b * np);
    const int py = pi / pw, px = pi - (pi / pw) * pw;
    const unsigned char* src = img + (((size_t)b * H + py * 14 + ky) * W + px * 14 + half * 8) * 3;
    const int nvalid = half ? 6 : 8;
    float v[3][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float f = 0.f;
        if (j < nvalid) {
          f = __fdiv_rn((float)src[j * 3 + c], nrm.scale);
          f = __fdiv_rn(__fsub_rn(f, nrm.mean[c]), nrm.stdv[c]);
        }
        v[c][j] = f;
      }
#pragma unroll
    for (int c = 0; c < 3; ++c) store8(P + patch * PK + c * 224 + ky * 16 + half * 8, v[c]);
    return;
  }
  id -= nchunk;
  if ((X || Xh) && id < (long long)B * D) {
    const int b = (int)(id / D), d = (int)(id - (long long)(id / D) * D);
    if (Xh) Xh[(size_t)b * T * D + d] = (f16)cls_pos[d];
    else X[(size_t)b * T * D + d] = cls_pos[d];
    return;
  }
  if (X || Xh) id -= (long long)B * D;
  if (lnst && id < (long long)B * (D / 16)) {
    const int per = D / 16, b = (int)(id / per), k = (int)(id - (long long)b * per);
    lnst[((size_t)(k >> 1) * B * T + (size_t)b * T) * 2 + (k & 1)] = cls_st[k];
  }
}

// Depth post-process: PyTorch upsample_bilinear2d(align_corners=True) of one
// fp32 channel, then clamp (reference onnx2trt.py:111-117).  One thread per
// output pixel, fp32 index math exactly as resize_kernel below.
__global__ void __launch_bounds__(256) depth_post_kernel(const float* __restrict__ in, float* __restrict__ out, int B,
                                                         int ih, int iw, int oh, int ow, float lo, float hi) {
  const long long n = (long long)B * oh * ow;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  int ox, oy, b;
  if (n < (1LL << 31)) {  // 32-bit index split (see resize_kernel)
    unsigned u = (unsigned)id;
    ox = (int)(u % (unsigned)ow);
    u /= (unsigned)ow;
    oy = (int)(u % (unsigned)oh);
    b = (int)(u / (unsigned)oh);
  } else {
    ox = (int)(id % ow);
    const long long q = id / ow;
    oy = (int)(q % oh);
    b = (int)(q / oh);
  }
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  ac_index(ac_scale(ih, oh), oy, ih, y0, y1, ly0, ly1);
  ac_index(ac_scale(iw, ow), ox, iw, x0, x1, lx0, lx1);
  const float* s = in + (size_t)b * ih * iw;
  const float v = ly0 * (lx0 * s[(size_t)y0 * iw + x0] + lx1 * s[(size_t)y0 * iw + x1]) +
                  ly1 * (lx0 * s[(size_t)y1 * iw + x0] + lx1 * s[(size_t)y1 * iw + x1]);
  out[id] = fminf(fmaxf(v, lo), hi);
}

// PyTorch upsample_bilinear2d(align_corners=True): src = dst*(in-1)/(out-1),
// h1 = floor(src), h1p = (h1 < in-1), lambda = src - h1; fp32 arithmetic.
__global__ void __launch_bounds__(256) resize_kernel(const f16* __restrict__ in, f16* __restrict__ out, int B,
                                                     int ih, int iw, int C, int oh, int ow) {
  const int C8 = C >> 3;
  const long long n = (long long)B * oh * ow * C8;
  // Block order stays round-robin over the XCDs: an XCD-contiguous order
  // (mde_device.h xcd_remap) fetches each source row into one L2 only (rf2
  // at B=48: 150 -> 34 MB fetched, = the source map) but runs SLOWER, 44.9
  // -> 54-56 us (profiles/r03_v2_remap_ab.txt); the duplicate fetches are
  // Infinity-Cache hits, and one address-ordered stream over the whole map
  // beats eight disjoint ones
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  int c8, ox, oy, b;
  if (n < (1LL << 31)) {  // 32-bit index split: a 64-bit divide is a long emulated sequence
    unsigned u = (unsigned)id;
    c8 = (int)(u % (unsigned)C8);
    u /= (unsigned)C8;
    ox = (int)(u % (unsigned)ow);
    u /= (unsigned)ow;
    oy = (int)(u % (unsigned)oh);
    b = (int)(u / (unsigned)oh);
  } else {
    c8 = (int)(id % C8);
    long long pix = id / C8;
    ox = (int)(pix % ow);
    pix /= ow;
    oy = (int)(pix % oh);
    b = (int)(pix / oh);
  }
#if MDE_RESIZE_F16
  // packed f16 blend in lerp form (mde_device.h upsample8, shared with the
  // E_STORE epilogue's resize-on-read): each axis' two weights sum to exactly
  // 1, so the out_conv bias folded in front of this resize (engine.hip
  // dav2_fusion) passes unchanged and a constant map stays constant
  // (tests/test_gpu_ops.py::test_resize_constant)
  const f16x8 v = upsample8(in, b, ih, iw, C, oh, ow, oy, ox, c8 * 8);
#else
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  ac_index(ac_scale(ih, oh), oy, ih, y0, y1, ly0, ly1);
  ac_index(ac_scale(iw, ow), ox, iw, x0, x1, lx0, lx1);
  const f16* base = in + (size_t)b * ih * iw * C + c8 * 8;
  const f16x8 a = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * iw + x0) * C);
  const f16x8 bb = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * iw + x1) * C);
  const f16x8 c = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * iw + x0) * C);
  const f16x8 d = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * iw + x1) * C);
  f16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = (f16)(ly0 * (lx0 * (float)a[j] + lx1 * (float)bb[j]) + ly1 * (lx0 * (float)c[j] + lx1 * (float)d[j]));
#endif
  *reinterpret_cast<f16x8*>(out + (size_t)id * 8) = v;
}

}  // namespace

hipError_t launch_layernorm(const float* x, h16* y, const float* g, const float* b, int rows, int D, float eps,
                            int T, int skip_cls, hipStream_t st, const h16* xh) {
  if (rows <= 0) return hipSuccess;
  dim3 grid((rows + 3) / 4), block(256);
  f16* yo = reinterpret_cast<f16*>(y);
  const f16* xf = reinterpret_cast<const f16*>(xh);
#define MDE_LN(PER)                                                                                                 \
  if (xh) hipLaunchKernelGGL((layernorm_h8_kernel<PER * 8>), dim3((rows + 15) / 16), block, 0, st, xf, yo, g, b, rows, \
                             eps, T, skip_cls);                                                                      \
  else hipLaunchKernelGGL((layernorm_kernel<PER, float>), grid, block, 0, st, x, yo, g, b, rows, eps, T, skip_cls);
  switch (D) {
    case 128: MDE_LN(2) break;
    case 256: MDE_LN(4) break;
    case 384: MDE_LN(6) break;
    case 768: MDE_LN(12) break;
    case 1024: MDE_LN(16) break;
    default: return hipErrorInvalidValue;
  }
#undef MDE_LN
  return hipGetLastError();
}

hipError_t launch_layernorm32(const float* x, float* y, const float* g, const float* b, int rows, int D, float eps,
                              hipStream_t st, int T, int skip_cls) {
  if (T <= 0 || (skip_cls && T < 2)) return hipErrorInvalidValue;
  if (rows <= 0) return hipSuccess;
  const dim3 grid((rows + 3) / 4), block(256);
  switch (D) {
    case 128: hipLaunchKernelGGL((layernorm_kernel<2, float, float>), grid, block, 0, st, x, y, g, b, rows, eps, T, skip_cls); break;
    case 256: hipLaunchKernelGGL((layernorm_kernel<4, float, float>), grid, block, 0, st, x, y, g, b, rows, eps, T, skip_cls); break;
    case 384: hipLaunchKernelGGL((layernorm_kernel<6, float, float>), grid, block, 0, st, x, y, g, b, rows, eps, T, skip_cls); break;
    case 768: hipLaunchKernelGGL((layernorm_kernel<12, float, float>), grid, block, 0, st, x, y, g, b, rows, eps, T, skip_cls); break;
    case 1024: hipLaunchKernelGGL((layernorm_kernel<16, float, float>), grid, block, 0, st, x, y, g, b, rows, eps, T, skip_cls); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_patch_prep(const float* img, h16* P, float* X, const float* cls_pos, int B, int H, int W, int ph,
                             int pw, int T, int D, hipStream_t st, h16* Xh, float* lnst, const float* cls_st, float* P32) {
  if (lnst && (!cls_st || (D & 31))) return hipErrorInvalidValue;
  if (H < ph * 14 || W < pw * 14) return hipErrorInvalidValue;
  const long long n = (long long)B * 3 * ph * 14 * pw + (long long)B * D + (lnst ? (long long)B * (D / 16) : 0);
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (P32)
    hipLaunchKernelGGL(patch_prep_kernel<float>, grid, block, 0, st, img, P32, X, cls_pos, B, H, W, ph, pw, T, D,
                       reinterpret_cast<f16*>(Xh), lnst, cls_st);
  else
    hipLaunchKernelGGL(patch_prep_kernel<f16>, grid, block, 0, st, img, reinterpret_cast<f16*>(P), X, cls_pos, B, H,
                       W, ph, pw, T, D, reinterpret_cast<f16*>(Xh), lnst, cls_st);
  return hipGetLastError();
}

hipError_t launch_patch_prep_u8(const unsigned char* img, h16* P, float* X, const float* cls_pos, int B, int H, int W,
                                int ph, int pw, int T, int D, float scale, const float* mean3, const float* std3,
                                hipStream_t st, h16* Xh, float* lnst, const float* cls_st, float* P32) {
  if (ph < 1 || pw < 1 || H < ph * 14 || W < pw * 14 || scale == 0.f) return hipErrorInvalidValue;
  if (lnst && (!cls_st || (D & 31) || !(X || Xh))) return hipErrorInvalidValue;
  const long long n = (long long)B * ph * pw * 28 + ((X || Xh) ? (long long)B * D : 0) +
                      (lnst ? (long long)B * (D / 16) : 0);
  if (n <= 0) return hipSuccess;
  InNorm nrm;
  nrm.scale = scale;
  for (int c = 0; c < 3; ++c) {
    nrm.mean[c] = mean3[c];
    nrm.stdv[c] = std3[c];
  }
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (P32)
    hipLaunchKernelGGL(patch_prep_u8_kernel<float>, grid, block, 0, st, img, P32, X, cls_pos, B, H, W, ph, pw, T, D,
                       nrm, reinterpret_cast<f16*>(Xh), lnst, cls_st);
  else
    hipLaunchKernelGGL(patch_prep_u8_kernel<f16>, grid, block, 0, st, img, reinterpret_cast<f16*>(P), X, cls_pos, B,
                       H, W, ph, pw, T, D, nrm, reinterpret_cast<f16*>(Xh), lnst, cls_st);
  return hipGetLastError();
}

hipError_t launch_depth_postprocess(const float* in, int B, int ih, int iw, float* out, int oh, int ow, float lo,
                                    float hi, hipStream_t st) {
  if (ih < 1 || iw < 1 || oh < 1 || ow < 1 || B < 1) return hipErrorInvalidValue;
  const long long n = (long long)B * oh * ow;
  hipLaunchKernelGGL(depth_post_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, out, B, ih, iw, oh,
                     ow, lo, hi);
  return hipGetLastError();
}

namespace {
// second half of the E_RESID split-K path (gemm.hip): one thread per 4
// columns, slices added in order 0..S-1, then the E_RESID update
__global__ void splitk_resid_kernel(const float* __restrict__ P, int S, int M, int N, const float* __restrict__ bias,
                                    const float* __restrict__ ls, float* __restrict__ x32, f16* __restrict__ xh,
                                    int ldo, float* __restrict__ lnst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n4 = N >> 2;
  if (i >= (long long)M * n4) return;  // M * n4 is a multiple of 8 (N % 32 == 0): 8-lane groups stay whole
  const int m = (int)(i / n4), n = (int)(i - (long long)m * n4) * 4;
  const size_t plane = (size_t)M * N;
  // every operand loaded up front and the slices four at a time (a runtime
  // loop of load -> add paid one round trip per slice), summed in order
  // 0..S-1 as before
  const float4 bn = bias ? *reinterpret_cast<const float4*>(bias + n) : float4{0.f, 0.f, 0.f, 0.f};
  const float4 l = *reinterpret_cast<const float4*>(ls + n);
  f16x4 xh0{};
  float4 x320{};
  if (xh) xh0 = *reinterpret_cast<const f16x4*>(xh + (size_t)m * ldo + n);
  else x320 = *reinterpret_cast<const float4*>(x32 + (size_t)m * ldo + n);
  float4 a = *reinterpret_cast<const float4*>(P + (size_t)m * N + n);
  for (int s0 = 1; s0 < S; s0 += 4) {
    float4 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + j < S) b[j] = *reinterpret_cast<const float4*>(P + (s0 + j) * plane + (size_t)m * N + n);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + j < S) {
        a.x += b[j].x; a.y += b[j].y; a.z += b[j].z; a.w += b[j].w;
      }
  }
  if (xh) {
    f16x4* x = reinterpret_cast<f16x4*>(xh + (size_t)m * ldo + n);
    f16x4 xv = xh0;
    xv[0] = (f16)((float)xv[0] + l.x * (a.x + bn.x));
    xv[1] = (f16)((float)xv[1] + l.y * (a.y + bn.y));
    xv[2] = (f16)((float)xv[2] + l.z * (a.z + bn.z));
    xv[3] = (f16)((float)xv[3] + l.w * (a.w + bn.w));
    *x = xv;
    if (lnst) {  // folded LN: (sum, M2 about the slice mean) of the row's 32-column slices, 8 lanes each
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) s1 += (float)xv[r];
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) s1 += __shfl_xor(s1, o);
      const float ms = s1 * (1.f / 32.f);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = (float)xv[r] - ms;
        s2 += d * d;
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) s2 += __shfl_xor(s2, o);
      if ((n & 31) == 0) *reinterpret_cast<float2*>(lnst + ((size_t)(n >> 5) * M + m) * 2) = make_float2(s1, s2);
    }
    return;
  }
  float4* x = reinterpret_cast<float4*>(x32 + (size_t)m * ldo + n);
  float4 xv = x320;
  xv.x += l.x * (a.x + bn.x);
  xv.y += l.y * (a.y + bn.y);
  xv.z += l.z * (a.z + bn.z);
  xv.w += l.w * (a.w + bn.w);
  *x = xv;
}
}  // namespace

hipError_t launch_splitk_resid(const float* P, int S, int M, int N, const float* bias, const float* ls, float* x32,
                               h16* xh, int ldo, hipStream_t st, float* lnst) {
  if (S < 1 || (N & 3) || (ldo & 3) || !ls || (lnst && (!xh || (N & 31)))) return hipErrorInvalidValue;
  const long long n = (long long)M * (N >> 2);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(splitk_resid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, S, M, N, bias, ls,
                     x32, reinterpret_cast<f16*>(xh), ldo, lnst);
  return hipGetLastError();
}

namespace {
// second half of the E_STORE split-K path (gemm.hip launch_split_store): one
// thread per 8 columns of a row, slices added in order 0..S-1, then the
// E_STORE epilogue of tile_epilogue.h (bias, activation, then the residual
// adds, one rounding to f16)
__global__ void splitk_store_kernel(const float* __restrict__ P, int S, int M, int N, GemmParams p) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n8 = N >> 3;
  if (i >= (long long)M * n8) return;
  const int m = (int)(i / n8), n = (int)(i - (long long)m * n8) * 8;
  const size_t plane = (size_t)M * N;
  const float* src = P + (size_t)m * N + n;
  float4 a0 = *reinterpret_cast<const float4*>(src), a1 = *reinterpret_cast<const float4*>(src + 4);
  for (int s0 = 1; s0 < S; s0 += 4) {  // four slices per batch of loads, summed in order
    float4 b0[4], b1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + j < S) {
        b0[j] = *reinterpret_cast<const float4*>(src + (s0 + j) * plane);
        b1[j] = *reinterpret_cast<const float4*>(src + (s0 + j) * plane + 4);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + j < S) {
        a0.x += b0[j].x; a0.y += b0[j].y; a0.z += b0[j].z; a0.w += b0[j].w;
        a1.x += b1[j].x; a1.y += b1[j].y; a1.z += b1[j].z; a1.w += b1[j].w;
      }
  }
  float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  if (p.bias) {
    const float4 c0 = *reinterpret_cast<const float4*>(p.bias + n), c1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
    v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
    v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
  }
  if (p.act == ACT_RELU) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
  } else if (p.act == ACT_GELU) {
#pragma unroll
    for (int r = 0; r < 8; r += 2) {
      const f32x2 g = gelu_erf2(f32x2{v[r], v[r + 1]});
      v[r] = g[0], v[r + 1] = g[1];
    }
  }
  const size_t o = (size_t)m * p.ldo + n;
  if (p.res0) {
    const size_t ro = p.res0_rows > 0 ? (size_t)(m % p.res0_rows) * p.ldo + n : o;
    const f16x8 r0 = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res0) + ro);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += p.res0_relu ? fmaxf((float)r0[r], 0.f) : (float)r0[r];
  }
  if (p.res1) {
    const f16x8 r1 = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res1) + o);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += (float)r1[r];
  }
  f16x8 h;
#pragma unroll
  for (int r = 0; r < 8; ++r) h[r] = (f16)v[r];
  *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.out16) + o) = h;
}
}  // namespace

hipError_t launch_splitk_store(const float* P, int S, const GemmParams& p, hipStream_t st) {
  if (S < 1 || (p.N & 7) || (p.ldo & 7) || !p.out16 || p.ldo < p.N) return hipErrorInvalidValue;
  const long long n = (long long)p.M * (p.N >> 3);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(splitk_store_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, S, p.M, p.N, p);
  return hipGetLastError();
}

hipError_t launch_resize(const h16* in, h16* out, int B, int ih, int iw, int C, int oh, int ow, hipStream_t st) {
  if (C & 7) return hipErrorInvalidValue;
  const long long n = (long long)B * oh * ow * (C >> 3);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(resize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const f16*>(in), reinterpret_cast<f16*>(out), B, ih, iw, C, oh, ow);
  return hipGetLastError();
}

}  // namespace mde
