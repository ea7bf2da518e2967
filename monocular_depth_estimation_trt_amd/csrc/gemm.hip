// MFMA (v_mfma_f32_16x16x32_f16) GEMM / implicit-GEMM convolution for gfx950.
//
// One kernel template serves every dense contraction of the DA-V2 forward:
//   C[M,N] = A[M,K] * W[N,K]^T   (fp16 operands, fp32 accumulation)
// where A is either a row-major activation (linear layers, 1x1 convs,
// ConvTranspose k==s) or the implicit im2col of a 3x3/pad-1 convolution over an
// NHWC map (optionally bilinear-upsampled on the fly), and the epilogue fuses
// what follows the contraction in the reference graph (bias, GELU/ReLU,
// LayerScale + residual, q/k/v head split, pos-embed add, ConvT pixel
// shuffle, RCU residual adds, the 1x1 depth head + sigmoid).
//
// Reference ops covered: a6 patch embed, a9 qkv/proj, a11
// LayerScale+residual, a12 fc1+GELU/fc2, a14 projects, a15 resize_layers,
// a16 layerN_rn, a17 RCU convs + out_conv, a18/a19 head convs.
//
// Tiling: BM x BN x 32 block tile, WM x WN waves, each wave owns
// (BM/WM) x (BN/WN) as 16x16 MFMA tiles.  Operands are register-staged into
// a double-buffered LDS image (one barrier per K-step) with 64-byte rows and
// the chunk swizzle c ^ ((row>>1)&3), which makes every ds_read_b128 lane
// group of the fragment reads conflict-free.
#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

constexpr int BK = 32;

MDE_DEV int swz(int row, int chunk) { return (chunk ^ ((row >> 1) & 3)) * 8; }

template <int BM, int BN, int WM, int WN, int AM, int EM>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(const GemmParams p) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / (WM * 16);
  constexpr int TN = BN / (WN * 16);
  static_assert(TM * WM * 16 == BM && TN * WN * 16 == BN, "tile");
  constexpr int RSTEP = NT / 4;               // rows covered by one pass of the block
  constexpr int AL = (BM + RSTEP - 1) / RSTEP;  // A chunks per thread
  constexpr int BL = (BN + RSTEP - 1) / RSTEP;  // B chunks per thread
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) f16 lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int ntn = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kc = tid & 3;      // 16-byte chunk column this thread stages
  const int rbase = tid >> 2;  // first row this thread stages

  // ---- A-row state (fixed over the K loop) ----
  const f16* arow[AL];
  int iy0[AL], ix0[AL];
  bool rv[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int r = rbase + i * RSTEP;
    const int gm = m0 + r;
    rv[i] = (r < BM) && (gm < p.M);
    const int gmc = rv[i] ? gm : 0;
    if constexpr (AM == A_DENSE) {
      arow[i] = reinterpret_cast<const f16*>(p.A) + (size_t)gmc * p.lda;
      iy0[i] = ix0[i] = 0;
    } else {
      const int hw = p.oh * p.ow;
      const int b = gmc / hw;
      const int rem = gmc - b * hw;
      const int oy = rem / p.ow, ox = rem - (rem / p.ow) * p.ow;
      iy0[i] = oy * p.stride - 1;
      ix0[i] = ox * p.stride - 1;
      arow[i] = reinterpret_cast<const f16*>(p.A) + (size_t)b * p.ch * p.cw * p.cc;
    }
  }
  // conv: (tap, c0) of k = k0 + kc*8, advanced by BK per step
  int tap = 0, c0 = kc * 8;
  if constexpr (AM != A_DENSE) {
    while (c0 >= p.cc) { c0 -= p.cc; ++tap; }
  }
  float usy = 0.f, usx = 0.f;
  if constexpr (AM == A_CONV3_UP) {
    usy = p.uh > 1 ? (float)(p.ch - 1) / (float)(p.uh - 1) : 0.f;
    usx = p.uw > 1 ? (float)(p.cw - 1) / (float)(p.uw - 1) : 0.f;
  }

  const f16* wrow[BL];
  bool bv[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int r = rbase + i * RSTEP;
    bv[i] = r < BN;
    wrow[i] = reinterpret_cast<const f16*>(p.W) + (size_t)(n0 + (bv[i] ? r : 0)) * p.ldw;
  }

  f16x8 ra[AL], rb[BL];

  auto fetch = [&](int k0) {
    const int k = k0 + kc * 8;
    const bool kv = k < p.K;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      f16x8 v = zero8();
      if constexpr (AM == A_DENSE) {
        if (rv[i] && kv) v = *reinterpret_cast<const f16x8*>(arow[i] + k);
      } else {
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
        const int iy = iy0[i] + ky, ix = ix0[i] + kx;
        if constexpr (AM == A_CONV3) {
          if (rv[i] && kv && iy >= 0 && iy < p.ch && ix >= 0 && ix < p.cw)
            v = *reinterpret_cast<const f16x8*>(arow[i] + ((size_t)iy * p.cw + ix) * p.cc + c0);
        } else {  // A_CONV3_UP: virtual map = bilinear(align_corners) upsample to uh x uw
          if (rv[i] && kv && iy >= 0 && iy < p.uh && ix >= 0 && ix < p.uw) {
            const float fy = usy * (float)iy, fx = usx * (float)ix;
            const int y0 = (int)fy, x0 = (int)fx;
            const int y1 = y0 + (y0 < p.ch - 1 ? 1 : 0), x1 = x0 + (x0 < p.cw - 1 ? 1 : 0);
            const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
            const float lx1 = fx - (float)x0, lx0 = 1.f - lx1;
            const f16* base = arow[i] + c0;
            const f16x8 a = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * p.cw + x0) * p.cc);
            const f16x8 b = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * p.cw + x1) * p.cc);
            const f16x8 c = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * p.cw + x0) * p.cc);
            const f16x8 d = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * p.cw + x1) * p.cc);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float t = ly0 * (lx0 * (float)a[j] + lx1 * (float)b[j]) +
                              ly1 * (lx0 * (float)c[j] + lx1 * (float)d[j]);
              v[j] = (f16)t;
            }
          }
        }
        if (p.relu_in) v = relu8(v);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      if (bv[i]) rb[i] = *reinterpret_cast<const f16x8*>(wrow[i] + k);
    }
    if constexpr (AM != A_DENSE) {
      c0 += BK;
      while (c0 >= p.cc) { c0 -= p.cc; ++tap; }
    }
  };

  auto stash = [&](int buf) {
    f16* sA = lds + buf * STAGE;
    f16* sB = sA + BM * BK;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int r = rbase + i * RSTEP;
      if (r < BM) *reinterpret_cast<f16x8*>(sA + r * BK + swz(r, kc)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int r = rbase + i * RSTEP;
      if (bv[i]) *reinterpret_cast<f16x8*>(sB + r * BK + swz(r, kc)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  fetch(0);
  stash(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) fetch((kt + 1) * BK);
    const f16* sA = lds + cur * STAGE;
    const f16* sB = sA + BM * BK;
    f16x8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * TM * 16 + i * 16 + (lane & 15);
      fa[i] = *reinterpret_cast<const f16x8*>(sA + r * BK + swz(r, lane >> 4));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wn * TN * 16 + j * 16 + (lane & 15);
      fb[j] = *reinterpret_cast<const f16x8*>(sB + r * BK + swz(r, lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
    if (kt + 1 < nk) stash(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const int mrow0 = m0 + wm * TM * 16 + (lane >> 4) * 4;
  const int ncol0 = n0 + wn * TN * 16 + (lane & 15);

  if constexpr (EM == E_HEAD) {
    static_assert(BN == 32 && WN == 1 && TN == 2, "head epilogue needs the full 32-channel row");
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float part = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = j * 16 + (lane & 15);
          const float v = acc[i][j][r] + p.bias[n];
          part += (v > 0.f ? v : 0.f) * p.w2[n];
        }
        part += __shfl_xor(part, 1, 64);
        part += __shfl_xor(part, 2, 64);
        part += __shfl_xor(part, 4, 64);
        part += __shfl_xor(part, 8, 64);
        const int m = mrow0 + i * 16 + r;
        if ((lane & 15) == 0 && m < p.M) {
          const float z = part + p.b2;
          p.out32[m] = p.head_metric ? p.max_depth / (1.f + __expf(-z)) : (z > 0.f ? z : 0.f);
        }
      }
    }
    return;
  } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = ncol0 + j * 16;
      if (n >= p.N) continue;
      const float bn = p.bias ? p.bias[n] : 0.f;
      // per-column constants of the scatter epilogues
      int qwhich = 0, qh = 0, qd = 0;
      int cq = 0, cco = 0, cdy = 0, cdx = 0;
      float lsn = 0.f;
      if constexpr (EM == E_QKV) {
        const int D = p.heads * 64;
        qwhich = n / D;
        const int w = n - qwhich * D;
        qh = w >> 6;
        qd = w & 63;
      }
      if constexpr (EM == E_CONVT) {
        cq = n / p.cout;
        cco = n - cq * p.cout;
        cdy = cq / p.s;
        cdx = cq - cdy * p.s;
      }
      if constexpr (EM == E_RESID) lsn = p.ls[n];
      const float bconv = (EM == E_CONVT) ? p.bias[cco] : bn;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mrow0 + i * 16 + r;
          if (m >= p.M) continue;
          float v = acc[i][j][r];
          if constexpr (EM == E_STORE) {
            v += bn;
            if (p.act == ACT_RELU) v = v > 0.f ? v : 0.f;
            else if (p.act == ACT_GELU) v = gelu_erf(v);
            const size_t o = (size_t)m * p.ldo + n;
            if (p.res0) v += (float)reinterpret_cast<const f16*>(p.res0)[o];
            if (p.res1) v += (float)reinterpret_cast<const f16*>(p.res1)[o];
            reinterpret_cast<f16*>(p.out16)[o] = (f16)v;
          } else if constexpr (EM == E_QKV) {
            v += bn;
            const int b = m / p.T, t = m - (m / p.T) * p.T;
            const size_t bh = (size_t)b * p.heads + qh;
            if (qwhich == 0)
              reinterpret_cast<f16*>(p.q)[(bh * p.Tpad + t) * 64 + qd] = (f16)(v * p.qscale);
            else if (qwhich == 1)
              reinterpret_cast<f16*>(p.k)[(bh * p.Tpad + t) * 64 + qd] = (f16)v;
            else
              reinterpret_cast<f16*>(p.vt)[(bh * 64 + qd) * p.Tpad + t] = (f16)v;
          } else if constexpr (EM == E_RESID) {
            float* x = p.x32 + (size_t)m * p.ldo + n;
            *x = *x + lsn * (v + bn);
          } else if constexpr (EM == E_PATCH) {
            const int b = m / p.npatch, pi = m - (m / p.npatch) * p.npatch;
            p.x32[((size_t)b * p.T + 1 + pi) * p.ldo + n] = v + bn + p.pos[(size_t)pi * p.ldo + n];
          } else if constexpr (EM == E_CONVT) {
            const int hw = p.ih * p.iw;
            const int b = m / hw, rem = m - (m / hw) * hw;
            const int y = rem / p.iw, x = rem - (rem / p.iw) * p.iw;
            const int OH = p.ih * p.s, OW = p.iw * p.s;
            const size_t o = (((size_t)b * OH + y * p.s + cdy) * OW + x * p.s + cdx) * p.cout + cco;
            reinterpret_cast<f16*>(p.out16)[o] = (f16)(v + bconv);
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int AM, int EM>
hipError_t run(const GemmParams& p, hipStream_t st) {
  const int gm = (p.M + BM - 1) / BM, gn = (p.N + BN - 1) / BN;
  const long long blocks = (long long)gm * gn;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AM, EM>), dim3((unsigned)blocks),
                     dim3(WM * WN * 64), 0, st, p);
  return hipGetLastError();
}

template <int AM, int EM>
hipError_t dispatch(const GemmParams& p, hipStream_t st) {
  if constexpr (EM == E_HEAD) {
    return run<128, 32, 4, 1, AM, EM>(p, st);
  } else {
    if constexpr (EM == E_STORE) {
      if (p.N <= 32) return run<128, 32, 4, 1, AM, EM>(p, st);
      if (p.N <= 64) {
        if (p.M >= 128 * 256) return run<128, 64, 4, 1, AM, EM>(p, st);
        return run<64, 64, 2, 2, AM, EM>(p, st);
      }
    }
    const long long big = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128);
    if (big >= 240) return run<128, 128, 2, 2, AM, EM>(p, st);
    return run<64, 64, 2, 2, AM, EM>(p, st);
  }
}

}  // namespace

hipError_t launch_gemm(const GemmParams& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.K <= 0 || (p.K & 7) || (p.ldw & 31) || p.ldw < ((p.K + 31) / 32) * 32) return hipErrorInvalidValue;
  if (p.amode != A_DENSE && (p.cc & 7)) return hipErrorInvalidValue;
  if (p.emode == E_HEAD && (p.N != 32 || p.amode == A_DENSE)) return hipErrorInvalidValue;
  switch (p.amode) {
    case A_DENSE:
      switch (p.emode) {
        case E_STORE: return dispatch<A_DENSE, E_STORE>(p, st);
        case E_QKV: return dispatch<A_DENSE, E_QKV>(p, st);
        case E_RESID: return dispatch<A_DENSE, E_RESID>(p, st);
        case E_PATCH: return dispatch<A_DENSE, E_PATCH>(p, st);
        case E_CONVT: return dispatch<A_DENSE, E_CONVT>(p, st);
        default: return hipErrorInvalidValue;
      }
    case A_CONV3:
      if (p.emode == E_STORE) return dispatch<A_CONV3, E_STORE>(p, st);
      return hipErrorInvalidValue;
    case A_CONV3_UP:
      if (p.emode == E_STORE) return dispatch<A_CONV3_UP, E_STORE>(p, st);
      if (p.emode == E_HEAD) return dispatch<A_CONV3_UP, E_HEAD>(p, st);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mde
