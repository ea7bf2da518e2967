// Direct 3x3 / pad-1 convolution over NHWC f16 maps with an LDS halo patch,
// MFMA 16x16x32 f16, for the DPT head (SURVEY.md 8a a15 conv s2, a16
// layerN_rn, a17 RCU convs, a18/a19 output_conv1/2).
//
// A block computes an 8 x 16 pixel output tile x BN channels.  Per channel
// chunk (CK = 32 or 64 channels) it stages the (8S+2) x (16S+2) input patch
// once in LDS -- by global_load_lds (padding pixels redirected to a zero
// line) or, for the upsampling variant, by blending each virtual pixel of the
// bilinear(align_corners=True) upsample once in registers -- and then runs
// the 9 taps as MFMA k-steps whose A fragments are read straight out of the
// patch (16 lanes = 16 consecutive pixels of a tile row).  Versus implicit
// im2col this loads every input pixel ~1.4x instead of 9x (36x for the
// upsampled head input).  Weights ([Cout][ky][kx][Cin], packer layout) stream
// through a double-buffered LDS stage per tap.  Patch rows are CK*2 bytes
// with the chunk swizzle of the GEMM (c ^ (pix & 7) for 128-B rows,
// c ^ ((pix >> 1) & 3) for 64-B rows): conflict-free fragment reads at S = 1.
#include "mde_device.h"
#include "mde_ops.h"
#include "tile_epilogue.h"

#ifndef MDE_EPI_LDS
#define MDE_EPI_LDS 1  // row-major epilogue staged through LDS (whole-line stores)
#endif
#ifndef MDE_UP_BLEND_F16
// bilinear blend of the upsampling convs in packed f16, as TensorRT's fp16
// Resize (0: fp32 blend, A/B).  B=30: output_conv2 0.439 -> 0.367 ms,
// output_conv1 0.259 -> 0.221 ms
#define MDE_UP_BLEND_F16 1
#endif
#ifndef MDE_CONV_BRES
#define MDE_CONV_BRES 1  // 32-wide convs with one channel chunk: all 9 weight taps LDS-resident (1: CK 32, 2: + CK 64)
#endif

namespace mde {

namespace {

__device__ __attribute__((aligned(64))) f16 g_zero_conv[64];

MDE_DEV void glds16c(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
MDE_DEV void wait_vmc() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

typedef f16 f16x2c __attribute__((ext_vector_type(2)));

// a + (b - a) * w on halves 2J, 2J+1: v_pk_add_f16 (neg) + v_pk_fma_f16.  The
// subtraction is spelled out -- hipcc splits an f16x8 fsub into scalar
// v_sub_f16 + SDWA + repack (3 VALU per pair instead of 1).  (Pairs are
// taken with shufflevector: a bit_cast of the f16x8 to a u32x4 followed by
// element reads miscompiles in ROCm 7.2's hipcc -- every element became
// element 0.)
template <int J>
MDE_DEV f16x2c lerp2(const f16x8& a, const f16x8& b, f16x2c w2) {
  const f16x2c a2 = __builtin_shufflevector(a, a, 2 * J, 2 * J + 1);
  const f16x2c b2 = __builtin_shufflevector(b, b, 2 * J, 2 * J + 1);
  unsigned dd;
  asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]"
      : "=v"(dd)
      : "v"(__builtin_bit_cast(unsigned, b2)), "v"(__builtin_bit_cast(unsigned, a2)));
  return a2 + __builtin_bit_cast(f16x2c, dd) * w2;
}

MDE_DEV f16x8 lerp8(const f16x8& a, const f16x8& b, f16 w) {
  const f16x2c w2 = {w, w};
  const f16x2c r0 = lerp2<0>(a, b, w2), r1 = lerp2<1>(a, b, w2), r2 = lerp2<2>(a, b, w2), r3 = lerp2<3>(a, b, w2);
  return __builtin_shufflevector(__builtin_shufflevector(r0, r1, 0, 1, 2, 3), __builtin_shufflevector(r2, r3, 0, 1, 2, 3),
                                 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int CK>
MDE_DEV int cpch(int pix, int lc) {
  if constexpr (CK == 64) return lc ^ (pix & 7);
  else return lc ^ ((pix >> 1) & 3);
}

constexpr int TH = 8, TW = 16;

//
// BRES (one channel chunk, p.cc == CK): the 9 weight taps (9 x BN x CK f16)
// are staged once with the patch, so the tap loop runs without a barrier --
// the head convs (32 output channels) otherwise pay 10 barriers for 36 MFMAs
// per wave.
template <int BN, int WM, int WN, int CK, int S, bool UP, int EM, bool BRES = false>
__global__ void __launch_bounds__(WM * WN * 64) conv3_kernel(const GemmParams p) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = TH * TW;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  static_assert(TM * WM * 16 == BM && TN * WN * 16 == BN, "tile");
  static_assert(EM != E_HEAD || (BN == 32 && WN == 1), "head epilogue");
  constexpr int ROWB = CK * 2, CH = CK / 8, RWP = 64 / CH;  // patch row bytes, chunks, pixels per wave-instr
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3, PHW = PH * PW;
  constexpr int PINS = (PHW + RWP - 1) / RWP;                // glds wave-instructions per patch
  constexpr int PPAD = PINS * RWP;
  constexpr int PATCH = PPAD * ROWB;
  constexpr int BSTAGE = BN * ROWB;
  constexpr int BINS = BN / RWP;                              // B rows per wave-instruction = RWP
  static_assert(BINS * RWP == BN, "B tile rows");
  // the LDS-staged epilogue reuses the patch/B space for the fp32 tile
  constexpr int MAIN = PATCH + (BRES ? 9 : 2) * BSTAGE, EPI = MDE_EPI_LDS ? BM * BN * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[MAIN > EPI ? MAIN : EPI];
  char* sP = smem;
  char* sB0 = smem + PATCH;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;

  const int Ho = p.oh, Wo = p.ow;
  const int tiles_x = (Wo + TW - 1) / TW, tiles_y = (Ho + TH - 1) / TH;
  const int ntn = (p.N + BN - 1) / BN;
  // XCD-aware order (as the GEMM): workgroups are dealt round-robin over the
  // 8 XCDs, so hand each XCD a contiguous run of tiles -- horizontally and
  // vertically adjacent tiles then share their halo / bilinear source rows in
  // one L2 instead of each XCD fetching them again (head.output_conv2 at
  // B=30 fetched ~2x its 168 MB source map without it).  Bijective.
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % ntn;
  bid /= ntn;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int n0 = tn * BN;
  // source map geometry: UP -> the (ch x cw) map is upsampled to (uh x uw) first
  const int IH = UP ? p.uh : p.ch, IW = UP ? p.uw : p.cw;
  const int iy0 = ty * TH * S - 1, ix0 = tx * TW * S - 1;
  const f16* img = reinterpret_cast<const f16*>(p.A) + (size_t)b * p.ch * p.cw * p.cc;

  const int lrow = lane / CH;
  const int lch = cpch<CK>(lrow, lane % CH);  // logical chunk this lane fetches (glds)
  const f16* wbase = reinterpret_cast<const f16*>(p.W) + (size_t)(n0 + lrow) * p.ldw + lch * 8;

  float usy = 0.f, usx = 0.f;
  if constexpr (UP) {
    usy = ac_scale(p.ch, p.uh);
    usx = ac_scale(p.cw, p.uw);
  }

  auto load_patch = [&](int chunk) {
    const int cbase = chunk * CK;
    if constexpr (!UP) {
      for (int q = wave; q < PINS; q += NW) {
        const int pp = q * RWP + lrow;
        const int py = pp / PW, px = pp - (pp / PW) * PW;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool ok = pp < PHW && iy >= 0 && iy < IH && ix >= 0 && ix < IW;
        const f16* src = ok ? img + ((size_t)iy * p.cw + ix) * p.cc + cbase + lch * 8 : g_zero_conv;
        glds16c(src, sP + q * RWP * ROWB);
      }
    } else {
      // one thread per (virtual pixel, 4 channel chunks): its source indices
      // and weights once for 32 channels (per chunk: 3.9x the VALU at CK 32,
      // and one item per pixel starves the 64-channel conv of lanes: output_conv1
      // 0.205 -> 0.220 ms at B=28); 32-bit element offsets inside the image
      // (a source map of one image is < 2^31 halves) so the four taps load
      // as saddr + voffset; the blend on whole f16x8 vectors (lerp8)
      const unsigned rowstride = (unsigned)p.cw * (unsigned)p.cc;
      constexpr int CG = CH < 4 ? CH : 4, NG = CH / CG;  // chunks per item, items per pixel
      for (int it = tid; it < PHW * NG; it += NT) {
        const int pp = it / NG, g0 = (it - (it / NG) * NG) * CG;
        const int py = pp / PW, px = pp - (pp / PW) * PW;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool inside = iy >= 0 && iy < IH && ix >= 0 && ix < IW;
        int y0 = 0, y1 = 0, x0 = 0, x1 = 0;
        float ly0 = 0.f, ly1 = 0.f, lx0 = 0.f, lx1 = 0.f;
        if (inside) {
          ac_index(usy, iy, p.ch, y0, y1, ly0, ly1);
          ac_index(usx, ix, p.cw, x0, x1, lx0, lx1);
        }
        const unsigned r0 = (unsigned)y0 * rowstride + (unsigned)cbase, r1 = (unsigned)y1 * rowstride + (unsigned)cbase;
        const unsigned o0 = (unsigned)x0 * (unsigned)p.cc, o1 = (unsigned)x1 * (unsigned)p.cc;
#pragma unroll
        for (int q = 0; q < CG; ++q) {
          const int lc = g0 + q;
          f16x8 v = zero8();
          if (inside) {
            const f16x8 a = *reinterpret_cast<const f16x8*>(img + (r0 + o0 + lc * 8));
            const f16x8 bq = *reinterpret_cast<const f16x8*>(img + (r0 + o1 + lc * 8));
            const f16x8 c = *reinterpret_cast<const f16x8*>(img + (r1 + o0 + lc * 8));
            const f16x8 d = *reinterpret_cast<const f16x8*>(img + (r1 + o1 + lc * 8));
#if MDE_UP_BLEND_F16
            // packed f16 blend in lerp form, a + (b - a) * w: the two weights of
            // each axis sum to exactly 1, so a constant map (or a folded bias)
            // is preserved
            v = lerp8(lerp8(a, bq, (f16)lx1), lerp8(c, d, (f16)lx1), (f16)ly1);
#else
#pragma unroll
            for (int j = 0; j < 8; ++j)
              v[j] = (f16)(ly0 * (lx0 * (float)a[j] + lx1 * (float)bq[j]) + ly1 * (lx0 * (float)c[j] + lx1 * (float)d[j]));
#endif
          }
          if (p.relu_in) v = relu8(v);
          *reinterpret_cast<f16x8*>(sP + pp * ROWB + cpch<CK>(pp, lc) * 16) = v;
        }
      }
    }
  };
  auto load_b = [&](int step, int buf) {
    const int chunk = step / 9, t = step - (step / 9) * 9;
    const int k0 = t * p.cc + chunk * CK;
    char* dst = sB0 + buf * BSTAGE;
    for (int q = wave; q < BINS; q += NW) glds16c(wbase + (size_t)q * RWP * p.ldw + k0, dst + q * RWP * ROWB);
  };

  // pre-activation ReLU of the staged (glds) patch, once per pixel in LDS
  // instead of on each of the 9 tap reads of it; callers barrier after
  auto relu_patch = [&] {
    if constexpr (!UP) {
      if (p.relu_in) {
        for (int c = tid; c < PATCH / 16; c += NT) {
          f16x8* q = reinterpret_cast<f16x8*>(sP + c * 16);
          *q = relu8(*q);
        }
      }
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunk = p.cc / CK;
  const int nsteps = 9 * nchunk;
  if constexpr (BRES) {
    load_patch(0);
#pragma unroll
    for (int t = 0; t < 9; ++t) load_b(t, t);
    wait_vmc();
    __syncthreads();
    if (!UP && p.relu_in) {
      relu_patch();
      __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const char* sB = sB0 + t * BSTAGE;
      const int ky = t / 3, kx = t - (t / 3) * 3;
#pragma unroll
      for (int s = 0; s < CK / 32; ++s) {
        const int lc = 4 * s + (lane >> 4);
        f16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int pp = ((wm * TM + i) * S + ky) * PW + (lane & 15) * S + kx;
          fa[i] = *reinterpret_cast<const f16x8*>(sP + pp * ROWB + cpch<CK>(pp, lc) * 16);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * TN * 16 + j * 16 + (lane & 15);
          fb[j] = *reinterpret_cast<const f16x8*>(sB + r * ROWB + cpch<CK>(r, lc) * 16);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
      }
    }
    __syncthreads();  // every wave done with the patch before the epilogue reuses the LDS
  }
  for (int chunk = 0; chunk < (BRES ? 0 : nchunk); ++chunk) {
    if (chunk > 0) __syncthreads();  // every wave done with the previous patch
    load_patch(chunk);
    const int step0 = chunk * 9;
    load_b(step0, step0 & 1);
    wait_vmc();
    __syncthreads();
    if (!UP && p.relu_in) {
      relu_patch();
      __syncthreads();
    }
    for (int t = 0; t < 9; ++t) {
      const int step = step0 + t;
      if (t + 1 < 9) load_b(step + 1, (step + 1) & 1);
      const char* sB = sB0 + (step & 1) * BSTAGE;
      const int ky = t / 3, kx = t - (t / 3) * 3;
#pragma unroll
      for (int s = 0; s < CK / 32; ++s) {
        const int lc = 4 * s + (lane >> 4);
        f16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int py = wm * TM + i;  // tile row (TW = 16 -> one 16-row MFMA block per tile row)
          const int pp = (py * S + ky) * PW + (lane & 15) * S + kx;
          fa[i] = *reinterpret_cast<const f16x8*>(sP + pp * ROWB + cpch<CK>(pp, lc) * 16);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * TN * 16 + j * 16 + (lane & 15);
          fb[j] = *reinterpret_cast<const f16x8*>(sB + r * ROWB + cpch<CK>(r, lc) * 16);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
      }
      wait_vmc();
      __syncthreads();
    }
  }
  (void)nsteps;

  int mrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int oy = ty * TH + wm * TM + i, ox = tx * TW + (lane & 15);
    mrow[i] = (oy < Ho && ox < Wo) ? ((b * Ho + oy) * Wo + ox) : -1;
  }
#if MDE_EPI_LDS
  // the main loop ended on a barrier: the LDS is free
  if (!store_tile_lds<EM, TM, TN>(
          p, acc,
          [&](int row) {
            const int oy = ty * TH + wm * TM + (row >> 4), ox = tx * TW + (row & 15);
            return (oy < Ho && ox < Wo) ? ((b * Ho + oy) * Wo + ox) : -1;
          },
          n0 + wn * TN * 16, lane, smem + wave * (TM * 16) * (TN * 16) * 4))
#endif
    store_tile<EM, TM, TN>(p, acc, mrow, n0 + wn * TN * 16 + (lane >> 4) * 4, lane);
}

template <int BN, int WM, int WN, int CK, int S, bool UP, int EM>
hipError_t run_conv(const GemmParams& p, hipStream_t st) {
  const long long blocks =
      (long long)p.cb * ((p.oh + TH - 1) / TH) * ((p.ow + TW - 1) / TW) * ((p.N + BN - 1) / BN);
  if (blocks <= 0) return hipSuccess;
  constexpr bool BRES_OK = BN == 32 && (CK == 32 ? MDE_CONV_BRES >= 1 : MDE_CONV_BRES >= 2);
  if (BRES_OK && p.cc == CK)
    hipLaunchKernelGGL((conv3_kernel<BN, WM, WN, CK, S, UP, EM, BRES_OK>), dim3((unsigned)blocks),
                       dim3(WM * WN * 64), 0, st, p);
  else
    hipLaunchKernelGGL((conv3_kernel<BN, WM, WN, CK, S, UP, EM>), dim3((unsigned)blocks), dim3(WM * WN * 64), 0,
                       st, p);
  return hipGetLastError();
}

template <int CK, int S, bool UP, int EM>
hipError_t conv_tiles(const GemmParams& p, hipStream_t st) {
  if constexpr (EM == E_HEAD) {
    return run_conv<32, 4, 1, CK, S, UP, EM>(p, st);
  } else {
    if (p.N <= 32) return run_conv<32, 4, 1, CK, S, UP, EM>(p, st);
    if (p.N <= 64) return run_conv<64, 4, 1, CK, S, UP, EM>(p, st);
    return run_conv<128, 2, 2, CK, S, UP, EM>(p, st);
  }
}

}  // namespace

bool conv_direct_supported(const GemmParams& p) {
  if (p.cc % 32) return false;
  if (p.amode == A_CONV3_UP) return p.stride == 1;
  return p.stride == 1 || p.stride == 2;
}

hipError_t launch_conv3(const GemmParams& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (!conv_direct_supported(p) || (p.N & 7) || (p.ldw & 63) || p.ldw < 9 * p.cc) return hipErrorInvalidValue;
  const bool up = p.amode == A_CONV3_UP;
  const bool ck64 = (p.cc % 64) == 0 && p.stride == 1;
  if (p.emode == E_HEAD) {
    if (p.N != 32 || p.stride != 1) return hipErrorInvalidValue;
    if (up) return ck64 ? conv_tiles<64, 1, true, E_HEAD>(p, st) : conv_tiles<32, 1, true, E_HEAD>(p, st);
    return ck64 ? conv_tiles<64, 1, false, E_HEAD>(p, st) : conv_tiles<32, 1, false, E_HEAD>(p, st);
  }
  if (p.emode != E_STORE) return hipErrorInvalidValue;
  if (up) return ck64 ? conv_tiles<64, 1, true, E_STORE>(p, st) : conv_tiles<32, 1, true, E_STORE>(p, st);
  if (p.stride == 2) return conv_tiles<32, 2, false, E_STORE>(p, st);
  return ck64 ? conv_tiles<64, 1, false, E_STORE>(p, st) : conv_tiles<32, 1, false, E_STORE>(p, st);
}

}  // namespace mde
