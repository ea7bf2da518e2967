// Exact-fp32 encoder kernels for precision "fp32" engines (gfx950).
//
// The reference's default engine (core/common.py:141-144, get_engine(...,
// precision="fp32")) is a TensorRT fp32 build: TF32 tensor-core math (10-bit
// mantissa) with fp32 storage and an 8-bit exponent everywhere.  Its
// "fp16" build is the one the benchmarks use.  These kernels give the
// DINOv2 encoder of a precision "fp32" engine fp32 operands end to end --
// activations, weights, q / k / v, attention probabilities and the MLP
// hidden layer all fp32 (23-bit mantissa, fp32 range) -- on gfx950's exact
// fp32 matrix instructions (v_mfma_f32_16x16x4_f32 / v_mfma_f32_32x32x2_f32,
// MI355X_MICROARCH.md: 157 TF/s, the fp32 vector rate, bit-equal to an fmaf
// chain).  Since round 5 the DPT head of such an engine is fp32 too (packs
// with the fp32 head weights, `head.c1.w32`): projects, resize layers,
// layerN_rn, the fusion blocks and the depth head on fp32 maps, as the
// reference's fp32 TensorRT engine runs every layer in fp32
// (reports/tune/fp32_depth_anything_v2.json: 'Float': 188 layers).
//
//   gemm32_kernel     C = A W^T, W fp32 [Npad][ldw]; A fp32 [M][lda] (A_DENSE)
//                     or the implicit im2col of a 3x3 pad-1 conv over an fp32
//                     NHWC map (A_CONV3, optional ReLU on the operand);
//                     epilogues E_STORE (fp32 or f16 out, bias, ReLU / GELU,
//                     two residual maps), E_QKV (fp32 q / k / v
//                     [B*H][Tpad][64], q scaled), E_RESID (x32 += ls * (acc +
//                     bias)), E_PATCH (x32 rows = acc + bias + pos), E_CONVT
//                     (ConvTranspose k = s pixel shuffle)
//   attn32_kernel     softmax(q k^T) v over those fp32 rows, online softmax in
//                     log2 units (q carries dh^-0.5 * log2 e), fp32 out
//   resize32_kernel   bilinear align_corners=True over fp32 NHWC maps
//   head32_kernel     output_conv2's last 1x1 conv + activation over the
//                     fp32 hidden map
//
// The GEMM keeps the f16 kernel's LDS geometry (gemm.hip): 128-B rows (here 32
// floats, one K-step), chunk swizzle c ^ (row & 7) applied on the global_load_lds
// source address, conflict-free ds_read_b128 fragment reads.  One 16-B read
// (4 consecutive k) of a lane feeds four 16x16x4 MFMAs, lane group g of MFMA
// t taking k = 16 s + 4 g + t -- the K order of a sum is permuted, identically
// for A and W.  At 32 cycles per 16x16x4 MFMA and 128 of them per K-step per
// wave, the loads of a K-step (32 KB per 128^2 workgroup) hide behind a
// two-stage ring.
#include <cstdint>

#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

MDE_DEV void glds16f(const void* src, void* lds) { __builtin_amdgcn_global_load_lds(src, lds, 16, 0, 0); }
MDE_DEV void wait_vm32() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

MDE_DEV int pch32(int r, int lc) { return lc ^ (r & 7); }

// padding taps of the implicit-im2col A read this (a glds lane cannot be
// masked, it can be redirected)
__device__ __attribute__((aligned(16))) float g_zero32[4];

template <int BM, int BN, int EM, int AM>
__global__ void __launch_bounds__(256) gemm32_kernel(const Gemm32Params p) {
  constexpr int WM = 2, WN = 2, NW = 4;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  constexpr int ROWB = 128, CH = 8, RW = 8;  // 32 floats per row; 8 rows per glds wave-instruction
  constexpr int AINS = BM / RW, BINS = BN / RW;
  static_assert(AINS % NW == 0 && BINS % NW == 0, "glds rows per wave");
  constexpr int APASS = AINS / NW, BPASS = BINS / NW;
  constexpr int STAGE = (BM + BN) * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / ntn, tn = bid - (bid / ntn) * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lrow = lane / CH;
  const int lch = pch32(lrow, lane % CH);
  const float* arow[APASS];
  int iy0[APASS], ix0[APASS];
  bool rv[APASS];
#pragma unroll
  for (int i = 0; i < APASS; ++i) {
    const int gm = m0 + (wave + i * NW) * RW + lrow;
    rv[i] = gm < p.M;
    const int gmc = rv[i] ? gm : p.M - 1;
    if constexpr (AM == A_DENSE) {
      arow[i] = p.A + (size_t)gmc * p.lda + lch * 4;
      iy0[i] = ix0[i] = 0;
    } else {  // output pixel (b, oy, ox) of row gm
      const int hw = p.oh * p.ow;
      const int b = gmc / hw, rem = gmc - (gmc / hw) * hw;
      const int oy = rem / p.ow, ox = rem - (rem / p.ow) * p.ow;
      iy0[i] = oy * p.stride - 1;
      ix0[i] = ox * p.stride - 1;
      arow[i] = p.A + (size_t)b * p.ch * p.cw * p.cc;
    }
  }
  const float* wrow = p.W + (size_t)(n0 + wave * RW + lrow) * p.ldw + lch * 4;
  const int nk = (p.K + 31) / 32;
  // A_CONV3: this lane's chunk at K-step kt is k = 32 kt + 4 lch = tap * cc + c
  // (cc % 4 == 0: a chunk never straddles taps), advanced by 32 per step
  int tap = 0, cch = lch * 4;
  if constexpr (AM == A_CONV3) {
    tap = cch / p.cc;
    cch -= tap * p.cc;
  }

  auto issue = [&](int kt, int buf) {
    char* sb = smem + buf * STAGE;
    const int k0 = kt * 32;
    if constexpr (AM == A_DENSE) {
      // K tail: W is zero-padded to ldw; a lane whose chunk lies past K reads
      // column 0 of its row instead (finite, and inside the row even when K < 32)
      const int ka = k0 + lch * 4 < p.K ? k0 : -lch * 4;
#pragma unroll
      for (int i = 0; i < APASS; ++i) glds16f(arow[i] + ka, sb + (wave + i * NW) * RW * ROWB);
    } else {
      const bool kv = k0 + lch * 4 < p.K;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
      for (int i = 0; i < APASS; ++i) {
        const int iy = iy0[i] + ky, ix = ix0[i] + kx;
        const bool ok = rv[i] && kv && iy >= 0 && iy < p.ch && ix >= 0 && ix < p.cw;
        const float* src = ok ? arow[i] + ((size_t)iy * p.cw + ix) * p.cc + cch : g_zero32;
        glds16f(src, sb + (wave + i * NW) * RW * ROWB);
      }
      cch += 32;
      while (cch >= p.cc) {
        cch -= p.cc;
        ++tap;
      }
    }
#pragma unroll
    for (int i = 0; i < BPASS; ++i)
      glds16f(wrow + (size_t)i * NW * RW * p.ldw + k0, sb + BM * ROWB + (wave + i * NW) * RW * ROWB);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](int buf) {
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + BM * ROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lc = 4 * s + (lane >> 4);
      f32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 16 + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const f32x4*>(sA + r * ROWB + pch32(r, lc) * 16);
        if constexpr (AM == A_CONV3) {
          if (p.relu_in) {
#pragma unroll
            for (int t = 0; t < 4; ++t) fa[i][t] = fa[i][t] > 0.f ? fa[i][t] : 0.f;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * TN * 16 + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const f32x4*>(sB + r * ROWB + pch32(r, lc) * 16);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j][t], fa[i][t], acc[i][j], 0, 0, 0);
    }
  };

  issue(0, 0);
  wait_vm32();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
    mma(kt & 1);
    wait_vm32();
    __syncthreads();
  }

  // epilogue: lane owns row m = .. + (lane & 15), columns n .. n + 3 of each block
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * TM * 16 + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 16 + j * 16 + (lane >> 4) * 4;
      if (n >= p.N) continue;
      f32x4 v = acc[i][j];
      if (EM != E_CONVT && p.bias) {
        const float4 b = *reinterpret_cast<const float4*>(p.bias + n);
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
      }
      if constexpr (EM == E_STORE) {
        if (p.act == ACT_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
        } else if (p.act == ACT_GELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = 0.5f * v[r] * (1.f + erff(v[r] * 0.70710678118654752f));
        }
        if (p.res0) {
          const float4 r = *reinterpret_cast<const float4*>(p.res0 + (size_t)m * p.ldo + n);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if (p.res1) {
          const float4 r = *reinterpret_cast<const float4*>(p.res1 + (size_t)m * p.ldo + n);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if (p.out32) {
          *reinterpret_cast<float4*>(p.out32 + (size_t)m * p.ldo + n) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          const f16x4 h = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
          *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.out16) + (size_t)m * p.ldo + n) = h;
        }
      } else if constexpr (EM == E_RESID) {
        float4* x = reinterpret_cast<float4*>(p.x32 + (size_t)m * p.ldo + n);
        const float4 ls = *reinterpret_cast<const float4*>(p.ls + n);
        float4 xv = *x;
        xv.x = fmaf(ls.x, v[0], xv.x);
        xv.y = fmaf(ls.y, v[1], xv.y);
        xv.z = fmaf(ls.z, v[2], xv.z);
        xv.w = fmaf(ls.w, v[3], xv.w);
        *x = xv;
      } else if constexpr (EM == E_PATCH) {
        const int b = m / p.npatch, pi = m - (m / p.npatch) * p.npatch;
        const float4 ps = *reinterpret_cast<const float4*>(p.pos + (size_t)pi * p.ldo + n);
        *reinterpret_cast<float4*>(p.x32 + ((size_t)b * p.T + 1 + pi) * p.ldo + n) =
            make_float4(v[0] + ps.x, v[1] + ps.y, v[2] + ps.z, v[3] + ps.w);
      } else if constexpr (EM == E_CONVT) {
        // cout % 4 == 0: the lane's four columns are four channels of one (dy, dx)
        const int hw = p.ih * p.iw;
        const int b = m / hw, rem = m - (m / hw) * hw;
        const int iy = rem / p.iw, ix = rem - (rem / p.iw) * p.iw;
        const int q = n / p.cout, co = n - (n / p.cout) * p.cout;
        const int dy = q / p.s, dx = q - (q / p.s) * p.s;
        const float4 bb = p.bias ? *reinterpret_cast<const float4*>(p.bias + co) : make_float4(0.f, 0.f, 0.f, 0.f);
        const size_t px = ((size_t)b * p.ih * p.s + (size_t)iy * p.s + dy) * ((size_t)p.iw * p.s) + (size_t)ix * p.s + dx;
        *reinterpret_cast<float4*>(p.out32 + px * p.ldo + co) =
            make_float4(v[0] + bb.x, v[1] + bb.y, v[2] + bb.z, v[3] + bb.w);
      } else if constexpr (EM == E_QKV) {
        const int D = p.heads * 64;
        const int which = n / D, hn = n - which * D, h = hn >> 6, d = hn & 63;
        const int b = m / p.T, t = m - (m / p.T) * p.T;
        float* dst = which == 0 ? p.q : (which == 1 ? p.k : p.v);
        const float sc = which == 0 ? p.qscale : 1.f;
        *reinterpret_cast<float4*>(dst + (((size_t)b * p.heads + h) * p.Tpad + t) * 64 + d) =
            make_float4(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
      }
    }
  }
}

template <int BM, int BN>
hipError_t run32(const Gemm32Params& p, hipStream_t st) {
  const long long tiles = (long long)((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  if (tiles <= 0) return hipSuccess;
  const dim3 grid((unsigned)tiles), block(256);
  if (p.amode == A_CONV3) {
    if (p.emode != E_STORE) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_STORE, A_CONV3>), grid, block, 0, st, p);
    return hipGetLastError();
  }
  switch (p.emode) {
    case E_STORE: hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_STORE, A_DENSE>), grid, block, 0, st, p); break;
    case E_QKV: hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_QKV, A_DENSE>), grid, block, 0, st, p); break;
    case E_RESID: hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_RESID, A_DENSE>), grid, block, 0, st, p); break;
    case E_PATCH: hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_PATCH, A_DENSE>), grid, block, 0, st, p); break;
    case E_CONVT: hipLaunchKernelGGL((gemm32_kernel<BM, BN, E_CONVT, A_DENSE>), grid, block, 0, st, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fp32 attention.  A wave owns 32 queries and a range of 32-key blocks.
// S^T = K Q^T on v_mfma_f32_32x32x2_f32 (A = K: 32 keys x 2 dims, B = Q^T):
// lane (query l & 31, half h = l >> 5) holds Q[q][t + 32 h], t = 0..31, and
// MFMA t takes dims {t, t + 32} -- one float4 of a K row feeds four MFMAs.
// The accumulator layout is the 32x32x16 f16 kernel's (attention.hip): the
// query on the lane, 16 keys per lane half, so the online softmax is the same
// register reduction + one permlane32_swap.  O^T += V^T P^T (A = V^T: 32 dh x
// 2 keys, B = P^T): MFMA t pairs the lane's own probability p[t] (key
// rho(t, h) = (t & 3) + 8 (t >> 2) + 4 h) with V[rho(t, h)][dh] -- no lane
// exchange, one coalesced 4-B V read per lane per MFMA.  K / V fragments come
// straight from L2 (a head's K and V are 0.7 MB at T = 1370, re-read by every
// query block); two waves per SIMD hide the loads behind the other's MFMAs
// (128 MFMAs of 64 cycles per 32-key block).  NKG = 4: the workgroup's four
// waves take the same 32 queries and a quarter of the key blocks each, merged
// through LDS (small grids: batch 1); NKG = 1: four query blocks.
constexpr float RESCALE_T32 = 8.f;

MDE_DEV float swap_max32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MDE_DEV float swap_sum32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int NKG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
attn32_kernel(const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
              float* __restrict__ o, int H, int T, int Tpad, int ldo, int nqb) {
  constexpr int NQW = 4 / NKG;
  __shared__ __attribute__((aligned(16))) float mbuf[NKG > 1 ? (NKG - 1) * 64 * 34 : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = NKG > 1 ? wave : 0, qw = NKG > 1 ? 0 : wave;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = wg / nqb, qblk = wg - (wg / nqb) * nqb;
  const int b = bh / H, hd = bh - (bh / H) * H;
  const int q0 = (qblk * NQW + qw) * 32;
  const int l31 = lane & 31, hh = lane >> 5;
  const float* qb = q + (size_t)bh * Tpad * 64;
  const float* kb = k + (size_t)bh * Tpad * 64;
  const float* vb = v + (size_t)bh * Tpad * 64;

  // Q^T fragments: dims t + 32 hh of query q0 + l31 (rows >= T are the zero pad of Tpad, or clamped)
  float qf[32];
  {
    const int qi = q0 + l31 < Tpad ? q0 + l31 : Tpad - 1;
    const float4* src = reinterpret_cast<const float4*>(qb + (size_t)qi * 64 + 32 * hh);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 x = src[u];
      qf[4 * u] = x.x;
      qf[4 * u + 1] = x.y;
      qf[4 * u + 2] = x.z;
      qf[4 * u + 3] = x.w;
    }
  }
  const int nkb = (T + 31) / 32;
  const int per = (nkb + NKG - 1) / NKG;
  const int kb0 = kg * per, kb1 = min(nkb, kb0 + per);

  float m_run = 0.f, l_run = 0.f;
  f32x16 acc[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = 0.f;
  const bool active = q0 < T;

  for (int blk = kb0; active && blk < kb1; ++blk) {
    const int key0 = blk * 32;
    // S^T over 64 dims: 32 MFMAs, K row key0 + l31, dims 4u + 32 hh .. + 3
    f32x16 sc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = 0.f;
    {
      const int kr = key0 + l31 < Tpad ? key0 + l31 : Tpad - 1;
      const float4* ks = reinterpret_cast<const float4*>(kb + (size_t)kr * 64 + 32 * hh);
      float4 kf[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) kf[u] = ks[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u].x, qf[4 * u], sc, 0, 0, 0);
        sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u].y, qf[4 * u + 1], sc, 0, 0, 0);
        sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u].z, qf[4 * u + 2], sc, 0, 0, 0);
        sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u].w, qf[4 * u + 3], sc, 0, 0, 0);
      }
    }
    // keys >= T -> -inf (register r: key key0 + (r & 3) + 8 (r >> 2) + 4 hh)
    if (key0 + 32 > T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key0 + (r & 3) + 8 * (r >> 2) + 4 * hh >= T) sc[r] = -INFINITY;
    }
    float mx = sc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
    mx = swap_max32(mx);
    const bool first = blk == kb0;
    if (first || mx > m_run + RESCALE_T32) {
      const float mnew = first ? mx : fmaxf(mx, m_run);
      if (!first) {
        const float alpha = __builtin_amdgcn_exp2f(m_run - mnew);
        l_run *= alpha;
        acc[0] *= alpha;
        acc[1] *= alpha;
      }
      m_run = mnew;
    }
    float pr[16];
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      pr[r] = __builtin_amdgcn_exp2f(sc[r] - m_run);
      ls += pr[r];
    }
    l_run += ls;
    // O^T += V^T P^T: MFMA t pairs p[t] with V[key0 + rho(t, hh)][32 db + l31]
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      float vf[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int key = key0 + (t & 3) + 8 * (t >> 2) + 4 * hh;
        vf[t] = vb[(size_t)(key < Tpad ? key : Tpad - 1) * 64 + 32 * db + l31];
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[db] = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[t], pr[t], acc[db], 0, 0, 0);
    }
  }

  if constexpr (NKG > 1) {
    // merge the key groups: waves 1.. park (O^T, m, l), wave 0 rescales and sums
    if (wave > 0) {
      float* w = mbuf + (wave - 1) * 64 * 34;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const f32x16& a = acc[c >> 2];
        *reinterpret_cast<float4*>(w + (c * 64 + lane) * 4) =
            make_float4(a[4 * (c & 3)], a[4 * (c & 3) + 1], a[4 * (c & 3) + 2], a[4 * (c & 3) + 3]);
      }
      w[8 * 64 * 4 + lane * 2] = m_run;
      w[8 * 64 * 4 + lane * 2 + 1] = l_run;
    }
    __syncthreads();
    if (wave > 0 || !active) return;
    float mg[NKG];
    mg[0] = m_run;
    float mmax = m_run;
#pragma unroll
    for (int g = 1; g < NKG; ++g) {
      mg[g] = mbuf[(g - 1) * 64 * 34 + 8 * 64 * 4 + lane * 2];
      if (g * per < nkb) mmax = fmaxf(mmax, mg[g]);
    }
    const float a0 = __builtin_amdgcn_exp2f(m_run - mmax);
    l_run *= a0;
    acc[0] *= a0;
    acc[1] *= a0;
#pragma unroll
    for (int g = 1; g < NKG; ++g) {
      if (g * per >= nkb) continue;
      const float* w = mbuf + (g - 1) * 64 * 34;
      const float ag = __builtin_amdgcn_exp2f(mg[g] - mmax);
      l_run += ag * w[8 * 64 * 4 + lane * 2 + 1];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4 x = *reinterpret_cast<const float4*>(w + (c * 64 + lane) * 4);
        acc[c >> 2][4 * (c & 3)] += ag * x.x;
        acc[c >> 2][4 * (c & 3) + 1] += ag * x.y;
        acc[c >> 2][4 * (c & 3) + 2] += ag * x.z;
        acc[c >> 2][4 * (c & 3) + 3] += ag * x.w;
      }
    }
  }
  if (!active) return;
  const int qi = q0 + l31;
  if (qi >= T) return;
  const float inv = 1.f / swap_sum32(l_run);
  // lane holds O^T[dh = 32 db + (r & 3) + 8 (r >> 2) + 4 hh][qi]: 4 consecutive dh per group
  float* orow = o + ((size_t)b * T + qi) * ldo + hd * 64;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *reinterpret_cast<float4*>(orow + 32 * db + 8 * g4 + 4 * hh) =
          make_float4(acc[db][4 * g4] * inv, acc[db][4 * g4 + 1] * inv, acc[db][4 * g4 + 2] * inv,
                      acc[db][4 * g4 + 3] * inv);
}

// fp32 NHWC bilinear resize, align_corners=True (PyTorch's index math,
// mde_device.h ac_index); one thread per (pixel, 4 channels)
__global__ void __launch_bounds__(256) resize32_kernel(const float* __restrict__ in, float* __restrict__ out, int ih,
                                                       int iw, int C4, int oh, int ow, long long n) {
  const long long id = (long long)blockIdx.x * 256 + threadIdx.x;
  if (id >= n) return;
  const int c4 = (int)(id % C4);
  long long pix = id / C4;
  const int ox = (int)(pix % ow);
  pix /= ow;
  const int oy = (int)(pix % oh);
  const int b = (int)(pix / oh);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  ac_index(ac_scale(ih, oh), oy, ih, y0, y1, ly0, ly1);
  ac_index(ac_scale(iw, ow), ox, iw, x0, x1, lx0, lx1);
  const size_t C = (size_t)C4 * 4;
  const float* base = in + (size_t)b * ih * iw * C + c4 * 4;
  const float4 a = *reinterpret_cast<const float4*>(base + ((size_t)y0 * iw + x0) * C);
  const float4 bb = *reinterpret_cast<const float4*>(base + ((size_t)y0 * iw + x1) * C);
  const float4 c = *reinterpret_cast<const float4*>(base + ((size_t)y1 * iw + x0) * C);
  const float4 d = *reinterpret_cast<const float4*>(base + ((size_t)y1 * iw + x1) * C);
  float4 v;
  v.x = ly0 * (lx0 * a.x + lx1 * bb.x) + ly1 * (lx0 * c.x + lx1 * d.x);
  v.y = ly0 * (lx0 * a.y + lx1 * bb.y) + ly1 * (lx0 * c.y + lx1 * d.y);
  v.z = ly0 * (lx0 * a.z + lx1 * bb.z) + ly1 * (lx0 * c.z + lx1 * d.z);
  v.w = ly0 * (lx0 * a.w + lx1 * bb.w) + ly1 * (lx0 * c.w + lx1 * d.w);
  *reinterpret_cast<float4*>(out + (size_t)id * 4) = v;
}

// output_conv2's last 1x1 conv (32 -> 1) + activation over the ReLU'd fp32
// hidden map; one thread per pixel (the E_HEAD epilogue's arithmetic)
__global__ void __launch_bounds__(256) head32_kernel(const float* __restrict__ hid, const float* __restrict__ w2,
                                                     float b2, int M, int metric, float max_depth,
                                                     float* __restrict__ out) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float4* h = reinterpret_cast<const float4*>(hid + (size_t)m * 32);
  float z = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4 v = h[j];
    z += v.x * w2[4 * j] + v.y * w2[4 * j + 1] + v.z * w2[4 * j + 2] + v.w * w2[4 * j + 3];
  }
  z += b2;
  out[m] = metric == 2 ? __expf(z) : metric ? max_depth / (1.f + __expf(-z)) : (z > 0.f ? z : 0.f);
}

}  // namespace

hipError_t launch_resize32(const float* in, float* out, int B, int ih, int iw, int C, int oh, int ow, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (!in || !out || ih <= 0 || iw <= 0 || oh <= 0 || ow <= 0 || C <= 0 || (C & 3) || ((uintptr_t)in & 15) ||
      ((uintptr_t)out & 15))
    return hipErrorInvalidValue;
  const long long n = (long long)B * oh * ow * (C / 4);
  hipLaunchKernelGGL(resize32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, out, ih, iw, C / 4, oh,
                     ow, n);
  return hipGetLastError();
}

hipError_t launch_head32(const float* hid, const float* w2, float b2, int M, int metric, float max_depth, float* out,
                         hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!hid || !w2 || !out || ((uintptr_t)hid & 15)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head32_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, hid, w2, b2, M, metric,
                     max_depth, out);
  return hipGetLastError();
}

hipError_t launch_gemm32(const Gemm32Params& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.K <= 0 || (p.K & 3) || (p.N & 3) || (p.ldw & 31) || p.ldw < ((p.K + 31) / 32) * 32 || !p.A || !p.W)
    return hipErrorInvalidValue;
  if (p.amode == A_DENSE) {
    if ((p.lda & 3) || p.lda < p.K) return hipErrorInvalidValue;
  } else if (p.amode == A_CONV3) {
    // the grid assumes M = cb * oh * ow output pixels of a 3x3 pad-1 conv
    if (p.cc <= 0 || (p.cc & 3) || p.K != 9 * p.cc || p.cb <= 0 || p.ch <= 0 || p.cw <= 0 || p.stride < 1 ||
        p.oh != (p.ch - 1) / p.stride + 1 || p.ow != (p.cw - 1) / p.stride + 1 || p.M != p.cb * p.oh * p.ow ||
        p.emode != E_STORE)
      return hipErrorInvalidValue;
  } else {
    return hipErrorInvalidValue;
  }
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.W & 15)) return hipErrorInvalidValue;
  switch (p.emode) {
    case E_STORE:
      if ((p.out32 == nullptr) == (p.out16 == nullptr) || (p.ldo & 3) || p.ldo < p.N) return hipErrorInvalidValue;
      if ((p.res0 || p.res1) && !p.out32) return hipErrorInvalidValue;
      break;
    case E_CONVT:
      if (!p.out32 || p.s < 1 || p.cout <= 0 || (p.cout & 3) || p.N != p.s * p.s * p.cout || p.ih <= 0 ||
          p.iw <= 0 || p.cb <= 0 || p.M != p.cb * p.ih * p.iw || (p.ldo & 3) || p.ldo < p.cout)
        return hipErrorInvalidValue;
      break;
    case E_RESID:
      if (!p.x32 || !p.ls || (p.ldo & 3)) return hipErrorInvalidValue;
      break;
    case E_PATCH:
      if (!p.x32 || !p.pos || p.npatch <= 0 || (p.ldo & 3)) return hipErrorInvalidValue;
      break;
    case E_QKV:
      if (!p.q || !p.k || !p.v || p.heads <= 0 || p.N != 3 * p.heads * 64 || p.Tpad < p.T || p.T <= 0)
        return hipErrorInvalidValue;
      break;
    default: return hipErrorInvalidValue;
  }
  // 128^2 tiles once they fill the CUs twice over; else 64^2 (batch 1)
  const long long t128 = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128);
  if (t128 >= 512) return run32<128, 128>(p, st);
  return run32<64, 64>(p, st);
}

hipError_t launch_attention32(const float* q, const float* k, const float* v, float* o, int B, int H, int T,
                              int Tpad, int ldo, hipStream_t st) {
  if (B <= 0 || T <= 0) return hipSuccess;
  if (!q || !k || !v || !o || Tpad < T || (ldo & 3) || ldo < H * 64 || ((uintptr_t)o & 15)) return hipErrorInvalidValue;
  const long long bh = (long long)B * H;
  const long long wg128 = bh * ((T + 127) / 128);
  if (wg128 >= 512) {
    const int nqb = (T + 127) / 128;
    hipLaunchKernelGGL((attn32_kernel<1>), dim3((unsigned)(bh * nqb)), dim3(256), 0, st, q, k, v, o, H, T, Tpad, ldo,
                       nqb);
  } else {
    const int nqb = (T + 31) / 32;
    hipLaunchKernelGGL((attn32_kernel<4>), dim3((unsigned)(bh * nqb)), dim3(256), 0, st, q, k, v, o, H, T, Tpad, ldo,
                       nqb);
  }
  return hipGetLastError();
}

}  // namespace mde
