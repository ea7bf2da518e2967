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
#include <cstdlib>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"
#include "tile_epilogue.h"
#include "tuning.h"

#ifndef MDE_EPI_LDS
#define MDE_EPI_LDS 1  // row-major epilogue staged through LDS (whole-line stores)
#endif
#ifndef MDE_UP_BLEND_F16
// bilinear blend of the upsampling convs in packed f16, as TensorRT's fp16
// Resize (0: fp32 blend, A/B).  B=30: output_conv2 0.439 -> 0.367 ms,
// output_conv1 0.259 -> 0.221 ms
#define MDE_UP_BLEND_F16 1
#endif
#ifndef MDE_CONVP_RELU_PASS
#define MDE_CONVP_RELU_PASS 1  // persistent conv1: input ReLU as an LDS pass per patch (0: on each fragment read)
#endif
#ifndef MDE_CONV_BRES
// 32-wide convs with one channel chunk: all 9 weight taps LDS-resident (1: CK
// 32, 2: + CK 64 -- the batch-1 ViT-S RCUs on 32-channel tiles: 36 KB of taps,
// two workgroups per CU on a 380-workgroup grid; rcu.conv 0.144 -> 0.117 ms,
// forward 0.825 -> 0.798 ms, b1 1044-1049 -> 1077-1079 FPS, two same-box
// pairs, gpurun_out/r4s51)
#define MDE_CONV_BRES 2
#endif

namespace mde {

namespace {

__device__ __attribute__((aligned(64))) f16 g_zero_conv[64];

MDE_DEV void glds16c(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
MDE_DEV void wait_vmc() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The same LDS-DMA (64-bit vaddr form) issued from inline asm: hipcc does not
// see it, so its ds_read waits in the DMA's shadow stay counted (lgkmcnt(N))
// instead of lgkmcnt(0) -- it models a pending FLAT LDS-DMA as an
// out-of-order lgkm event.  The caller counts the DMA itself (vmcnt) and
// orders LDS accesses around it with "memory" asm.  M0 is written and
// restored inside the statement (compiler-reserved).
MDE_DEV void glds16_asm(const void* src, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_dst)
               : "memory");
}
// workgroup barrier without __syncthreads()'s fence (which drains vmcnt, i.e.
// also the epilogue's global stores): own LDS accesses retired, s_barrier
MDE_DEV void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

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
// 4-wave tiles of the plain (non-upsampling) conv held to 128 registers: the
// 64-channel RCU conv (CK 64) otherwise allocates 82 VGPRs + 48 AGPRs = three
// waves per SIMD; at four its 39 KB of LDS still lets four workgroups share a CU
template <int BN, int WM, int WN, int CK, int S, bool UP, int EM, bool BRES = false, int TY = TH>
__global__ void __launch_bounds__(WM * WN * 64)
    __attribute__((amdgpu_waves_per_eu((WM * WN == 4 || WM * WN == 8) && !UP ? 4 : 1))) conv3_kernel(const GemmParams p) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = TY * TW;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  static_assert(TM * WM * 16 == BM && TN * WN * 16 == BN, "tile");
  static_assert(EM != E_HEAD || (BN == 32 && WN == 1), "head epilogue");
  constexpr int ROWB = CK * 2, CH = CK / 8, RWP = 64 / CH;  // patch row bytes, chunks, pixels per wave-instr
  constexpr int PH = (TY - 1) * S + 3, PW = (TW - 1) * S + 3, PHW = PH * PW;
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
  const int tiles_x = (Wo + TW - 1) / TW, tiles_y = (Ho + TY - 1) / TY;
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
  const int iy0 = ty * TY * S - 1, ix0 = tx * TW * S - 1;
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
    const int oy = ty * TY + wm * TM + i, ox = tx * TW + (lane & 15);
    mrow[i] = (oy < Ho && ox < Wo) ? ((b * Ho + oy) * Wo + ox) : -1;
  }
#if MDE_EPI_LDS
  // the main loop ended on a barrier: the LDS is free
  if (!store_tile_lds<EM, TM, TN, 0, true>(
          p, acc,
          [&](int row) {
            const int oy = ty * TY + wm * TM + (row >> 4), ox = tx * TW + (row & 15);
            return (oy < Ho && ox < Wo) ? ((b * Ho + oy) * Wo + ox) : -1;
          },
          n0 + wn * TN * 16, lane, smem + wave * (TM * 16) * (TN * 16) * 4))
#endif
    store_tile<EM, TM, TN, true>(p, acc, mrow, n0 + wn * TN * 16 + (lane >> 4) * 4, lane);
}

template <int BN, int WM, int WN, int CK, int S, bool UP, int EM, int TY = TH>
hipError_t run_conv(const GemmParams& p, hipStream_t st) {
  const long long blocks =
      (long long)p.cb * ((p.oh + TY - 1) / TY) * ((p.ow + TW - 1) / TW) * ((p.N + BN - 1) / BN);
  if (blocks <= 0) return hipSuccess;
  constexpr bool BRES_OK = BN == 32 && (CK == 32 ? MDE_CONV_BRES >= 1 : MDE_CONV_BRES >= 2);
  if (BRES_OK && p.cc == CK)
    hipLaunchKernelGGL((conv3_kernel<BN, WM, WN, CK, S, UP, EM, BRES_OK, TY>), dim3((unsigned)blocks),
                       dim3(WM * WN * 64), 0, st, p);
  else
    hipLaunchKernelGGL((conv3_kernel<BN, WM, WN, CK, S, UP, EM, false, TY>), dim3((unsigned)blocks),
                       dim3(WM * WN * 64), 0, st, p);
  return hipGetLastError();
}

// Narrower channel tiles for small grids (switch "conv_narrow", tuning.h):
// wide convs (N > 64) whose 128-channel grid leaves CUs with
// one or two workgroups (under 512: batch 1, e.g. ViT-L's 148^2 256-channel
// RCUs at 380) take 64-channel tiles -- twice the workgroups at 40 KB LDS
// each, the busiest CU carrying ~3 half-width tiles instead of 2 full ones;
// 64-channel convs under one workgroup per CU take 32-channel tiles.
bool conv_narrow_tiles() { return knob(KNOB_CONV_NARROW) != 0; }

template <int CK, int S, bool UP, int EM>
hipError_t conv_tiles(const GemmParams& p, hipStream_t st) {
  if constexpr (EM == E_HEAD) {
    return run_conv<32, 4, 1, CK, S, UP, EM>(p, st);
  } else {
    if (p.N <= 32) return run_conv<32, 4, 1, CK, S, UP, EM>(p, st);
    if (p.N <= 64) {
      // 64-channel convs on a grid under one workgroup per CU (batch 1: the
      // ViT-S RCUs at 148^2 are 190 tiles) split the channels over two
      // 32-wide workgroups: ViT-S B=1 rcu.conv 0.165 -> 0.144 ms, forward
      // 0.854 -> 0.826 ms (same box, profiles/r03_v11_*)
      const long long wg64 = (long long)p.cb * ((p.oh + TH - 1) / TH) * ((p.ow + TW - 1) / TW);
      if (!UP && p.N == 64 && conv_narrow_tiles() && wg64 < 256) return run_conv<32, 4, 1, CK, S, UP, EM>(p, st);
      return run_conv<64, 4, 1, CK, S, UP, EM>(p, st);
    }
    const long long wg128 = (long long)p.cb * ((p.oh + TH - 1) / TH) * ((p.ow + TW - 1) / TW) * ((p.N + 127) / 128);
    if (!UP && conv_narrow_tiles() && wg128 < 512) return run_conv<64, 4, 1, CK, S, UP, EM>(p, st);
    return run_conv<128, 2, 2, CK, S, UP, EM>(p, st);
  }
}

// ---------------------------------------------------------------------------
// Persistent 64 -> 64 channel direct conv (the DPT RCU convs at 64 features,
// stride 1): conv3_kernel streams the 9 weight taps (72 KB) through LDS once
// per 128-pixel tile -- 576 B of L2 -> LDS traffic per output pixel beside
// ~180 B of patch, and a barrier per tap.  Here one workgroup per CU keeps
// the whole weight set LDS-resident, walks a run of tiles, and prefetches the
// next tile's patch into the second of two patch buffers while the MFMAs run
// on the first; the tap loop has no barrier.  Same fragments and MFMA order
// as conv3_kernel at CK 64 (one chunk, taps in order, two k-steps each):
// bit-identical.
// The tap loop is address-free: every fragment read is one of 16 per-lane
// patch addresses (the chunk swizzle of pixel pp depends on (pp & 7) only,
// and a tap moves pp by a compile-time amount) or 4 weight addresses, plus an
// immediate offset -- the tile loop is unrolled by two so the patch buffer
// is a constant too (computed addresses cost ~3 VALU per MFMA, which the
// 8 issue cycles an MFMA leaves cannot hold).  The input ReLU (conv1) is one
// LDS pass over each landed patch, not 4 VALU per fragment read.
// MODE (the two RCU convs): 0 = ReLU'd input, bias, ReLU, no residual
// (conv1); 1 = bias + res0; 2 = bias + res0 + res1 (conv2); 3 = plain (bias
// optional: layer1_rn, whose 48 input channels are padded to 64).  Its own
// epilogue: the residual rows are loaded before the MFMAs and consumed on
// every path (rows outside the map load row 0 and skip the store), so no load
// is left pending across the tile loop -- hipcc otherwise guards the next
// iteration with vmcnt(0), draining the patch prefetch before the first read.
// The tile parks in the patch buffer just consumed: f16 rows (MODE 0: the f16
// value is the output) or fp32 in two 16-row passes, then leaves as whole
// 128-B rows.
// TYP = 16 (the default, switch value 1): 16 x 16-pixel tiles on 8 waves,
// LDS 154 KB; 8 (value 2, A/B): 8 x 16 on 4 waves, 118 KB -- one wave per
// SIMD, measured slower.  Each wave: 2 tile rows x 64 channels.
template <int TYP, int MODE>
__global__ void __launch_bounds__(TYP * 32) __attribute__((amdgpu_waves_per_eu(1)))
conv64p_kernel(const GemmParams p) {
  constexpr int NW = TYP / 2, NT = NW * 64, TM = 2, TN = 4;
  constexpr int ROWB = 128, RWP = 8;  // patch / weight rows of 64 halves, rows per wave-instruction
  constexpr int PH = TYP + 2, PW = TW + 2, PHW = PH * PW;
  constexpr int PINS = (PHW + RWP - 1) / RWP;
  constexpr int PATCH = PINS * RWP * ROWB;
  constexpr int WOFF = 2 * PATCH;  // weights after the two patch buffers: row (tap, n) at WOFF + (tap * 64 + n) * 128
  constexpr int WB = 9 * 64 * ROWB;
  constexpr int EPIW = 16 * 64 * 4;  // staging slice per wave: 16 fp32 rows (or 32 f16 rows)
  constexpr int NRES = MODE == 3 ? 0 : MODE;
  constexpr bool F16STAGE = MODE == 0 || MODE == 3;  // no residual: the staged f16 value is the output
  static_assert(NW * EPIW <= PATCH, "epilogue staging fits the consumed patch buffer");
  static_assert(PATCH + ((TM + 1) * PW + 2) * ROWB < 65536 && 7 * 8192 + 3 * 2048 < 65536, "ds_read immediate offsets");
  static_assert(PW % 8 == 2, "pixel row stride = 2 mod 8 (the swizzle table below)");
  __shared__ __attribute__((aligned(16))) char smem[2 * PATCH + WB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ho = p.oh, Wo = p.ow;
  const int tiles_x = (Wo + TW - 1) / TW, tiles_y = (Ho + TYP - 1) / TYP;
  const int ntiles = p.cb * tiles_x * tiles_y;
  // XCD x (= blockIdx % 8, one L2) owns tiles [x nt / 8, (x+1) nt / 8); its
  // workgroups stride through the run, so the tiles in flight on an XCD are
  // neighbours sharing halo rows in its L2 (as upconv_kernel)
  const int x8 = blockIdx.x & 7, g8 = (int)gridDim.x >> 3;
  int t = (int)((long long)x8 * ntiles / 8) + (int)(blockIdx.x >> 3);
  const int tend = (int)((long long)(x8 + 1) * ntiles / 8);
  if (t >= tend) return;  // uniform, before any load

  const int lrow = lane >> 3;
  const int lch = cpch<64>(lrow, lane & 7);  // logical chunk this lane fetches (glds)
  const size_t imgsz = (size_t)p.ch * p.cw * 64;

  // ---- the weight set, once
  for (int q = wave; q < 9 * 64 / RWP; q += NW) {
    const int tap = q >> 3, n = (q & 7) * RWP + lrow;
    glds16c(reinterpret_cast<const f16*>(p.W) + (size_t)n * p.ldw + tap * 64 + lch * 8, smem + WOFF + q * RWP * ROWB);
  }
  // ASM: the in-loop prefetch (glds16_asm); the prologue's patch uses the
  // builtin, drained by __syncthreads()'s vmcnt(0) before the loop
  auto load_patch = [&](int tt, int buf, auto asm_tag) {
    const int tx = tt % tiles_x, r = tt / tiles_x;
    const int ty = r % tiles_y, b = r / tiles_y;
    const int iy0 = ty * TYP - 1, ix0 = tx * TW - 1;
    const f16* img = reinterpret_cast<const f16*>(p.A) + (size_t)b * imgsz;
    char* dst = smem + buf * PATCH;
    for (int q = wave; q < PINS; q += NW) {
      const int pp = q * RWP + lrow;
      const int py = pp / PW, px = pp - (pp / PW) * PW;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = pp < PHW && iy >= 0 && iy < p.ch && ix >= 0 && ix < p.cw;
      const f16* src = ok ? img + ((size_t)iy * p.cw + ix) * 64 + lch * 8 : g_zero_conv;
      if constexpr (decltype(asm_tag)::value)
        glds16_asm(src, __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(dst + q * RWP * ROWB)));
      else
        glds16c(src, dst + q * RWP * ROWB);
    }
  };
  // MODE 0: ReLU of a landed patch, in place (callers barrier before and after)
  auto relu_patch = [&](int buf) {
    for (int c = tid; c < PATCH / 16; c += NT) {
      f16x8* q = reinterpret_cast<f16x8*>(smem + buf * PATCH + c * 16);
      *q = relu8(*q);
    }
  };

  // fragment addresses.  Patch: pixel pp = (wave TM + i + ky) PW + (lane & 15)
  // + kx, logical chunk lc = 4 s + (lane >> 4) at physical chunk lc ^ (pp & 7);
  // with PW = 2 mod 8, pp & 7 = (u + e) & 7 for u = (2 wave TM + (lane & 15))
  // and e = 2 (i + ky) + kx, so the 16 (e & 7, s) addresses below plus the
  // immediate ((i + ky) PW + kx) * 128 + BUF * PATCH cover every read.
  // Weights: row j 16 + (lane & 15) of a tap, (row & 7) = (lane & 7).
  int pa[8][2], wa[2], wa8[2];
  {
    const int u = 2 * wave * TM + (lane & 15);
    const int rowbase = ((wave * TM) * PW + (lane & 15)) * ROWB;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) pa[e][s2] = rowbase + ((((4 * s2 + (lane >> 4)) ^ ((u + e) & 7))) << 4);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      wa[s2] = WOFF + (lane & 15) * ROWB + (((4 * s2 + (lane >> 4)) ^ (lane & 7)) << 4);
      wa8[s2] = wa[s2] + 8 * 64 * ROWB;
    }
  }

  // epilogue geometry: the MFMA layout parks column quad (lane >> 4) of
  // pixel row (lane & 15); the read-back lane owns row (lane >> 3) of each
  // 8-row group and channels 8 (lane & 7) .. + 7
  const int rr = lane >> 3, c8 = lane & 7;
  float4 bias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
    bias[j] = p.bias ? *reinterpret_cast<const float4*>(p.bias + j * 16 + (lane >> 4) * 4) : float4{0.f, 0.f, 0.f, 0.f};

  load_patch(t, 0, std::false_type{});
  wait_vmc();
  __syncthreads();
  if constexpr (MODE == 0) {
    if (MDE_CONVP_RELU_PASS) relu_patch(0);
    lds_sync();
  }

  // one tile: MFMAs on patch buffer BUF while the next tile's patch lands in
  // the other; returns true when the workgroup's run is done
  auto step = [&](auto buf_tag) -> bool {
    constexpr int BUF = decltype(buf_tag)::value;
    const int tn = t + g8;
    // (every wave's epilogue staging in BUF ^ 1 was read before the barrier
    // that ended the previous tile)
    if (tn < tend) load_patch(tn, BUF ^ 1, std::true_type{});

    const int tx = t % tiles_x, r = t / tiles_x;
    const int ty = r % tiles_y, b = r / tiles_y;
    // output row (pixel) of read-back row it * 8 + rr of this wave, or -1
    int mo[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = it * 8 + rr;
      const int oy = ty * TYP + wave * TM + (row >> 4), ox = tx * TW + (row & 15);
      mo[it] = (oy < Ho && ox < Wo) ? ((b * Ho + oy) * Wo + ox) : -1;
    }
    // residual rows, loaded now and consumed after the MFMAs on every path
    f16x8 res[NRES > 0 ? NRES : 1][4];
    if constexpr (NRES > 0) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const size_t o = (size_t)(mo[it] < 0 ? 0 : mo[it]) * p.ldo + c8 * 8;
        res[0][it] = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res0) + o);
        if constexpr (NRES > 1) res[1][it] = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res1) + o);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // issue the loads here, not sunk next to their use behind the MFMAs

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int e = 2 * (i + ky) + kx;
          fa[i] = *reinterpret_cast<const f16x8*>(smem + pa[e & 7][s2] + (BUF * PATCH + ((i + ky) * PW + kx) * ROWB));
          if constexpr (MODE == 0 && !MDE_CONVP_RELU_PASS) fa[i] = relu8(fa[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const f16x8*>(smem + (tap < 8 ? wa[s2] + tap * 64 * ROWB : wa8[s2]) + j * 16 * ROWB);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);  // (tap MFMAs)
      }
    }
    // (the epilogue's residual conversions stay below: hoisted among the
    // MFMAs they would wait for the loads -- and, in order, the prefetch)
    __builtin_amdgcn_sched_barrier(0);
    // the next patch landed (own DMAs; the previous tile's stores and this
    // tile's residual loads, all issued before the MFMAs, too) -- after the
    // barrier every wave's DMAs and patch reads are done: the epilogue may
    // stage in this buffer and the next tile read the other
    wait_vmc();
    lds_sync();
    if constexpr (MODE == 0) {
      if (MDE_CONVP_RELU_PASS && tn < tend) relu_patch(BUF ^ 1);
    }

    char* stage = smem + BUF * PATCH + wave * EPIW;
    f16* const out = reinterpret_cast<f16*>(p.out16);
    if constexpr (F16STAGE) {
      // f16 rows: row r at r * 128, 16-B chunk c swizzled by (r & 7)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float4 bn = bias[j];
          const float v0 = acc[i][j][0] + bn.x, v1 = acc[i][j][1] + bn.y;
          const float v2 = acc[i][j][2] + bn.z, v3 = acc[i][j][3] + bn.w;
          const f16x4 h = MODE == 0 ? f16x4{(f16)(v0 > 0.f ? v0 : 0.f), (f16)(v1 > 0.f ? v1 : 0.f),
                                            (f16)(v2 > 0.f ? v2 : 0.f), (f16)(v3 > 0.f ? v3 : 0.f)}
                                    : f16x4{(f16)v0, (f16)v1, (f16)v2, (f16)v3};
          const int row = i * 16 + (lane & 15), q = j * 4 + (lane >> 4);  // 8-B column quad
          *reinterpret_cast<f16x4*>(stage + row * 128 + ((((q >> 1) ^ (row & 7)) << 4) | ((q & 1) << 3))) = h;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int row = it * 8 + rr;
        const f16x8 h = *reinterpret_cast<const f16x8*>(stage + row * 128 + ((c8 ^ (row & 7)) << 4));
        if (mo[it] >= 0) *reinterpret_cast<f16x8*>(out + (size_t)mo[it] * p.ldo + c8 * 8) = h;
      }
    } else {
      // fp32 rows of 256 B, 16-B chunk c swizzled by (r & 7); two passes of
      // 16 rows (accumulator row block i)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (i > 0) __builtin_amdgcn_wave_barrier();  // pass 0's reads before pass 1 overwrites the slice
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float4 bn = bias[j];
          const f32x4 v = {acc[i][j][0] + bn.x, acc[i][j][1] + bn.y, acc[i][j][2] + bn.z, acc[i][j][3] + bn.w};
          const int row = lane & 15, q = j * 4 + (lane >> 4);  // 16-B chunk
          *reinterpret_cast<f32x4*>(stage + row * 256 + ((q ^ (row & 7)) << 4)) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int it = i * 2 + h2, row = h2 * 8 + rr;
          const f32x4 a = *reinterpret_cast<const f32x4*>(stage + row * 256 + (((2 * c8) ^ (row & 7)) << 4));
          const f32x4 bb = *reinterpret_cast<const f32x4*>(stage + row * 256 + (((2 * c8 + 1) ^ (row & 7)) << 4));
          float v[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
          const f16x8 r0 = res[0][it];
          if (p.res0_relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += fmaxf((float)r0[e], 0.f);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)r0[e];
          }
          if constexpr (NRES > 1) {
            const f16x8 r1 = res[NRES - 1][it];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)r1[e];
          }
          f16x8 h;
#pragma unroll
          for (int e = 0; e < 8; ++e) h[e] = (f16)v[e];
          if (mo[it] >= 0) *reinterpret_cast<f16x8*>(out + (size_t)mo[it] * p.ldo + c8 * 8) = h;
        }
      }
    }
    if (tn >= tend) return true;
    lds_sync();  // staging reads retired before the next prefetch overwrites them; the next patch is ReLU'd (stores stay in flight)
    t = tn;
    return false;
  };
  for (;;) {
    if (step(std::integral_constant<int, 0>{})) break;
    if (step(std::integral_constant<int, 1>{})) break;
  }
}

// Persistent conv for the RCU shapes (64 -> 64 channels, stride 1, E_STORE:
// conv1 = ReLU'd input + bias + ReLU, conv2 = bias + residual(s), and the
// plain conv of layer1_rn) on grids of >= 4 tiles per CU (switch "conv_persist"): ViT-S's
// 148^2 / 74^2 RCUs at batch >= 8
// conv64p mode of p (0-3, above), or -1 when the persistent conv does not take it
int conv64p_mode(const GemmParams& p) {
  const int mode = knob(KNOB_CONV_PERSIST);
  if (!mode || p.amode != A_CONV3 || p.emode != E_STORE || p.stride != 1 || p.N != 64 || p.cc != 64 ||
      p.ch != p.oh || p.cw != p.ow || p.ldo < 64 || (p.ldo & 7) || p.res0_rows > 0)
    return -1;
  const bool r1 = p.res1 || p.res1_up;
  int m;
  if (p.relu_in && p.act == ACT_RELU && !p.res0 && !r1) m = 0;
  else if (!p.relu_in && p.act == ACT_NONE && !p.res0 && !r1) m = 3;
  else if (!p.relu_in && p.act == ACT_NONE && p.res0) m = r1 ? 2 : 1;
  else return -1;
  const int typ = mode == 2 ? 8 : 16;
  const long long tiles = (long long)p.cb * ((p.oh + typ - 1) / typ) * ((p.ow + TW - 1) / TW);
  if (tiles < 4 * 256 || tiles >= (1ll << 31)) return -1;
  return m;
}

bool conv64p_launch(const GemmParams& p, hipStream_t st, hipError_t& err) {
  const int m = conv64p_mode(p);
  if (m < 0) return false;
  const int typ = knob(KNOB_CONV_PERSIST) == 2 ? 8 : 16;
  const dim3 grid(256), block(typ * 32);
  if (typ == 16) {
    if (m == 0) hipLaunchKernelGGL((conv64p_kernel<16, 0>), grid, block, 0, st, p);
    else if (m == 1) hipLaunchKernelGGL((conv64p_kernel<16, 1>), grid, block, 0, st, p);
    else if (m == 2) hipLaunchKernelGGL((conv64p_kernel<16, 2>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((conv64p_kernel<16, 3>), grid, block, 0, st, p);
  } else {
    if (m == 0) hipLaunchKernelGGL((conv64p_kernel<8, 0>), grid, block, 0, st, p);
    else if (m == 1) hipLaunchKernelGGL((conv64p_kernel<8, 1>), grid, block, 0, st, p);
    else if (m == 2) hipLaunchKernelGGL((conv64p_kernel<8, 2>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((conv64p_kernel<8, 3>), grid, block, 0, st, p);
  }
  err = hipGetLastError();
  return true;
}

// ---------------------------------------------------------------------------
// Separable upsampling conv (A_CONV3_UP, 32 output channels: the DPT head's
// output_conv1 at ViT-S and output_conv2 at every width).
//
// conv3_kernel's upsampling loader blends each virtual pixel of its 10 x 18
// patch from 4 source taps: 4 loads and 3 lerps per pixel, 1.4 virtual
// pixels per output, and every 128-pixel workgroup restages the 9 weight
// taps.  The bilinear upsample is separable, so this kernel builds the patch
// in two passes over a 16 x 16 output tile (18 x 18 virtual patch):
//   pass H: for each source row the tile touches (<= 12) and each patch
//           column, lerp the two source columns (2 loads, 1 lerp);
//   pass V: for each patch pixel, lerp the two H rows (2 LDS reads, 1 lerp).
// Per output pixel: ~1.7 loads and ~2.1 lerps instead of 5.6 and 4.2.  The
// weights: at cc = 32 all 9 taps resident (18 KB, staged once); wider, the
// item's 32-channel chunk restaged per item.  The blend is the same
// two-level lerp in the same order (horizontal, then vertical) as
// conv3_kernel, so the patch is bit-identical; at cc = 32 the MFMA order is
// too (cc > 32: 32-channel chunks, tap-major inside a chunk).  8 waves x (2
// tile rows x 32 channels); LDS 52 KB at every cc: three workgroups per CU
// (the patch and H buffers swizzled by column, uoff below).
constexpr int UTH = 16, UTW = 16;                        // output tile
constexpr int UPH = UTH + 2, UPW = UTW + 2;              // virtual patch
// source rows per tile (host-checked, exactly): 12 keeps the cc = 32 kernel
// at 52 KB of LDS -- three workgroups per CU also at the hardware's LDS
// allocation granule (13 rows, 53.1 KB, measured 3.1 resident waves per SIMD)
constexpr int USR = 12;
constexpr int UPATCH = UPH * UPW * 64, UHBUF = USR * UPW * 64;
// byte offset of (row, column, logical 16-B chunk) in the patch / H buffers:
// rows of UPW pixels x 64 B, the chunk swizzled by the COLUMN only (within a
// row the same bank spread as a pixel-index swizzle; across rows a pure
// offset, so the 3 x 3 taps' row steps fold into ds_read immediates and a
// lane needs one base address per column shift)
MDE_DEV int uoff(int row, int col, int lc) { return row * (UPW * 64) + col * 64 + ((lc ^ ((col >> 1) & 3)) << 4); }

template <int NCH, int EM, bool PERSIST>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NCH == 1 ? 6 : 4)))
upconv_kernel(const GemmParams p) {
  static_assert(EM == E_STORE || EM == E_HEAD, "upconv epilogues");
  constexpr int NT = 512, TM = 2, TN = 2;
  // cc > 32: the current item's chunk of the weights is restaged per item
  // (18 KB from L2) instead of all chunks resident, so every NCH keeps the
  // 52 KB that fit three workgroups per CU (output_conv1 at cc = 64: 72 KB,
  // two per CU, otherwise)
  constexpr bool SW = NCH > 1;
  constexpr int WROWS = 9 * (SW ? 1 : NCH) * 32;  // weight rows of 64 B: (tap, chunk, out channel)
  // E_STORE stages f16 rows (store_tile_lds HALF: 2 KB per wave) in the patch
  // space, which no wave writes again before the next item's first barrier
  // bias (and the head's 1x1 weights) live in LDS: a global load in the
  // epilogue would wait (vmcnt is in order) for the next item's prefetch
  __shared__ __attribute__((aligned(16))) char smem[UPATCH + UHBUF + WROWS * 64 + 256];
  char* const sP = smem;
  char* const sH = smem + UPATCH;
  char* const sW = sH + UHBUF;
  float* const sBias = reinterpret_cast<float*>(sW + WROWS * 64);  // [32] bias, [32] w2 (E_HEAD)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ho = p.oh, Wo = p.ow;
  const int tiles_x = (Wo + UTW - 1) / UTW, tiles_y = (Ho + UTH - 1) / UTH;
  const int ntiles = p.cb * tiles_x * tiles_y;
  // tiles of this workgroup: t, t + tstep, ... < tend.  Persistent: XCD x
  // (= blockIdx % 8, one L2) owns the contiguous range [x nt / 8, (x+1) nt / 8)
  // and its workgroups stride through it, so the tiles an XCD has in flight
  // are neighbours sharing their source rows in its L2.
  int t, tstep, tend;
  if constexpr (PERSIST) {
    const int x = blockIdx.x & 7, g8 = (int)gridDim.x >> 3;
    t = (int)((long long)x * ntiles / 8) + (int)(blockIdx.x >> 3);
    tend = (int)((long long)(x + 1) * ntiles / 8);
    tstep = g8;
  } else {
    t = xcd_remap(blockIdx.x, gridDim.x);
    tend = t + 1;
    tstep = 1;
  }
  if (t >= tend) return;  // uniform, before any load is issued
  const float usy = ac_scale(p.ch, p.uh), usx = ac_scale(p.cw, p.uw);
  const unsigned rowstride = (unsigned)p.cw * (unsigned)p.cc;

  // ---- weights, all taps and chunks, once (glds: 16 rows x 4 chunks per wave-instruction)
  if constexpr (!SW) {
    const int lrow = lane >> 2, lch = cpch<32>(lrow, lane & 3);
    for (int q = wave; q < WROWS / 16; q += 8) {
      const int tc = q >> 1, n = (q & 1) * 16 + lrow;
      const int tp = tc / NCH, c = tc - (tc / NCH) * NCH;
      glds16c(reinterpret_cast<const f16*>(p.W) + (size_t)n * p.ldw + tp * p.cc + c * 32 + lch * 8, sW + q * 16 * 64);
    }
  }

  if (tid < 64) {
    const float* src = tid < 32 ? p.bias : p.w2;
    sBias[tid] = (src && (tid < 32 || EM == E_HEAD)) ? src[tid & 31] : 0.f;
  }

  // tile geometry: image, tile row / column, virtual origin, source rows [sy0, sy0 + nsr)
  struct Geo {
    int b, ty, tx, iy0, ix0, sy0, nsr;
  };
  auto geo = [&](int tt) {
    Geo g;
    g.tx = tt % tiles_x;
    const int r = tt / tiles_x;
    g.ty = r % tiles_y;
    g.b = r / tiles_y;
    g.iy0 = g.ty * UTH - 1;
    g.ix0 = g.tx * UTW - 1;
    int a0, a1, b0, b1;
    float l0, l1;
    ac_index(usy, g.iy0 < 0 ? 0 : g.iy0, p.ch, a0, a1, l0, l1);
    const int last = g.iy0 + UPH - 1 < p.uh - 1 ? g.iy0 + UPH - 1 : p.uh - 1;
    ac_index(usy, last, p.ch, b0, b1, l0, l1);
    g.sy0 = a0;
    g.nsr = b1 - a0 + 1 < USR ? b1 - a0 + 1 : USR;
    return g;
  };

  // Both passes map a thread to a fixed (patch column, 8-channel chunk) --
  // CL = 72 pairs -- and one of RG = 7 row groups (504 of the 512 threads),
  // stepping over rows: the column's source index, weight and bounds are
  // computed once per tile, not per item.
  constexpr int CL = UPW * 4, RG = NT / CL;
  static_assert(RG * 2 >= USR && RG * 3 >= UPH, "row groups cover the H rows (2 each) and the patch rows (3)");
  // ---- pass H operands of item (tile g, chunk c): HI (source row, patch
  // column, chunk) items per thread, both source columns loaded into
  // registers -- issued one item ahead, under the previous item's pass V,
  // MFMAs and epilogue
  constexpr int HI = 2;
  f16x8 ha[HI], hb[HI];
  f16 hw = (f16)0.0f;
  bool hs[HI], hin = false;
  auto h_issue = [&](const Geo& g, int c, int tid) {
    const f16* img = reinterpret_cast<const f16*>(p.A) + (size_t)g.b * p.ch * p.cw * p.cc;
    const int cl = tid % CL, rg = tid / CL;
    const int lc = cl & 3, col = cl >> 2;
    const int ix = g.ix0 + col;
    hin = rg < RG && ix >= 0 && ix < p.uw;
    int x0 = 0, x1 = 0;
    float lx0, lx1 = 0.f;
    if (hin) ac_index(usx, ix, p.cw, x0, x1, lx0, lx1);
    hw = (f16)lx1;
    const unsigned o0 = (unsigned)x0 * (unsigned)p.cc + (unsigned)(c * 32 + lc * 8);
    const unsigned o1 = (unsigned)x1 * (unsigned)p.cc + (unsigned)(c * 32 + lc * 8);
#pragma unroll
    for (int k = 0; k < HI; ++k) {
      const int sr = rg + k * RG;
      hs[k] = rg < RG && sr < g.nsr;
      const unsigned r = (unsigned)(g.sy0 + (hin && hs[k] ? sr : 0)) * rowstride;
      // (out-of-map columns load a valid pixel and are zeroed at the commit:
      // a select here would wait for the load)
      ha[k] = *reinterpret_cast<const f16x8*>(img + (r + o0));
      hb[k] = *reinterpret_cast<const f16x8*>(img + (r + o1));
    }
  };
  auto h_commit = [&](int tid) {
    const int cl = tid % CL, rg = tid / CL;
    const int lc = cl & 3, col = cl >> 2;
#pragma unroll
    for (int k = 0; k < HI; ++k) {
      if (hs[k]) {
        *reinterpret_cast<f16x8*>(sH + uoff(rg + k * RG, col, lc)) =
            hin ? lerp8(ha[k], hb[k], hw) : zero8();
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Geo g = geo(t);
  int c = 0;
  h_issue(g, 0, tid);
  for (;;) {
    // the thread id through an opaque move: every lane-derived LDS address is
    // recomputed per item instead of being hoisted out of the tile loop (the
    // 18 tap addresses of the patch fragments alone would hold 18 VGPRs)
    int vt;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vt) : "v"(tid));
    const int vl = vt & 63;
    wait_vmc();  // this item's pass-H operands (and, first time, the weights) landed
    h_commit(vt);
    __syncthreads();  // H complete; every wave done with the previous item's MFMAs / staging
    if constexpr (SW) {
      // chunk c's weights (every wave has left the previous item's MFMAs),
      // issued from asm ahead of the next item's pass-H loads and waited
      // for by count before the second barrier
      const int lrow = vl >> 2, lch = cpch<32>(lrow, vl & 3);
      for (int q = wave; q < WROWS / 16; q += 8) {
        const int n = (q & 1) * 16 + lrow;
        glds16_asm(reinterpret_cast<const f16*>(p.W) + (size_t)n * p.ldw + (q >> 1) * p.cc + c * 32 + lch * 8,
                   __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(sW + q * 16 * 64)));
      }
    }
    // the next item's pass-H loads fly under this item's pass V, MFMAs and epilogue
    int tn = t, cn = c + 1;
    if (cn == NCH) {
      cn = 0;
      tn = t + tstep;
    }
    Geo gn = g;
    if (tn < tend) {
      gn = geo(tn);
      h_issue(gn, cn, vt);
    }
    // ---- pass V: the thread's (column, chunk) over rows rg, rg + RG, ...
    // (not unrolled: the next item's pass-H registers are live here)
    {
      const int cl = vt % CL, rg = vt / CL;
      const int lc = cl & 3, col = cl >> 2;
      const int ix = g.ix0 + col;
      const bool xin = ix >= 0 && ix < p.uw;
#pragma unroll 1
      for (int r = rg; r < UPH && rg < RG; r += RG) {
        const int iy = g.iy0 + r;
        f16x8 v = zero8();
        if (xin && iy >= 0 && iy < p.uh) {
          int y0, y1;
          float ly0, ly1;
          ac_index(usy, iy, p.ch, y0, y1, ly0, ly1);
          const f16x8 a = *reinterpret_cast<const f16x8*>(sH + uoff(y0 - g.sy0, col, lc));
          const f16x8 bb = *reinterpret_cast<const f16x8*>(sH + uoff(y1 - g.sy0, col, lc));
          v = lerp8(a, bb, (f16)ly1);
          if (p.relu_in) v = relu8(v);
        }
        *reinterpret_cast<f16x8*>(sP + uoff(r, col, lc)) = v;
      }
    }
    if constexpr (SW) {
      // this wave's weight DMAs landed: only the next item's 2 HI pass-H
      // loads, issued after them, may still be in flight
      if (tn < tend) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * HI) : "memory");
      else wait_vmc();
    }
    __syncthreads();
    // ---- 9 taps x one 32-deep k-step of chunk c
    {
      const int lane = vl, lc = vl >> 4;
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int ky = tp / 3, kx = tp - (tp / 3) * 3;
        f16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          fa[i] = *reinterpret_cast<const f16x8*>(sP + uoff(wave * TM + i + ky, (lane & 15) + kx, lc));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = j * 16 + (lane & 15);
          fb[j] = *reinterpret_cast<const f16x8*>(sW + ((SW ? tp : tp * NCH + c) * 32 + r) * 64 + cpch<32>(r, lc) * 16);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
        if constexpr (PERSIST) __builtin_amdgcn_sched_barrier(0);  // no fragment hoisting across taps (registers)
      }
    }
    if (c == NCH - 1) {
      // ---- epilogue of tile t: lane owns pixel (row wave*TM + i, column
      // lane & 15) and channels 16 j + 4 (lane >> 4) + r (tile_epilogue.h
      // store_tile semantics, bias from LDS)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int oy = g.ty * UTH + wave * TM + i, ox = g.tx * UTW + (vl & 15);
        const int m = (oy < Ho && ox < Wo) ? ((g.b * Ho + oy) * Wo + ox) : -1;
        if constexpr (EM == E_HEAD) {
          // (the positional-embedding variant in its own branch: its global
          // load's wait must not sit on the no-pe path, where it would drain
          // the next item's prefetch)
          auto hidden = [&](auto pe_tag) {
            constexpr bool PE = decltype(pe_tag)::value;
            float part = 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int n0 = j * 16 + (vl >> 4) * 4;
              const float4 bn = *reinterpret_cast<const float4*>(sBias + n0);
              const float4 w2 = *reinterpret_cast<const float4*>(sBias + 32 + n0);
              float h0 = acc[i][j][0] + bn.x, h1 = acc[i][j][1] + bn.y;
              float h2 = acc[i][j][2] + bn.z, h3 = acc[i][j][3] + bn.w;
              if constexpr (PE) {
                // (+ 0 where no embedding: the no-PE path skips the add -- it
                // changes only a -0 sum, which the ReLU below maps to +0 anyway)
                float pv[4] = {0.f, 0.f, 0.f, 0.f};
                if (m >= 0) {
                  const f16x4 q = *reinterpret_cast<const f16x4*>(reinterpret_cast<const f16*>(p.hpe) +
                                                                  (size_t)(m % p.hpe_pix) * 32 + n0);
#pragma unroll
                  for (int r = 0; r < 4; ++r) pv[r] = (float)q[r];
                }
                h0 += pv[0];
                h1 += pv[1];
                h2 += pv[2];
                h3 += pv[3];
              }
              // explicit fma chain: the contraction store_tile's loop gets
              // (packed-math vectorisation would otherwise split some of it)
              part = fmaf(h0 > 0.f ? h0 : 0.f, w2.x, part);
              part = fmaf(h1 > 0.f ? h1 : 0.f, w2.y, part);
              part = fmaf(h2 > 0.f ? h2 : 0.f, w2.z, part);
              part = fmaf(h3 > 0.f ? h3 : 0.f, w2.w, part);
            }
            return part;
          };
          float part = p.hpe ? hidden(std::true_type{}) : hidden(std::false_type{});
          part += __shfl_xor(part, 16, 64);
          part += __shfl_xor(part, 32, 64);
          if ((vl >> 4) == 0 && m >= 0) {
            const float z = part + p.b2;
            p.out32[m] = p.head_metric == 2 ? __expf(z)
                         : p.head_metric ? p.max_depth / (1.f + __expf(-z)) : (z > 0.f ? z : 0.f);
          }
        } else {
          if (m < 0) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n0 = j * 16 + (vl >> 4) * 4;
            const float4 bn = *reinterpret_cast<const float4*>(sBias + n0);
            float v[4] = {acc[i][j][0] + bn.x, acc[i][j][1] + bn.y, acc[i][j][2] + bn.z, acc[i][j][3] + bn.w};
            if (p.act == ACT_RELU) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
            } else if (p.act == ACT_GELU) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
            }
            const f16x4 h = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
            *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.out16) + (size_t)m * p.ldo + n0) = h;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (tn >= tend) break;
    t = tn;
    c = cn;
    g = gn;
  }
}

// switch "upconv" = 0: the upsampling convs stay on conv3_kernel (A/B, tests)
bool upconv_enabled() { return knob(KNOB_UPCONV) != 0; }

// every 16-row tile's 18 virtual rows must come from at most USR source
// rows: the device's fp32 index arithmetic (ac_scale, ac_index in geo())
// restated on the host for each tile row -- the exact span, not a bound
bool upconv_eligible(const GemmParams& p) {
#pragma clang fp contract(off)
  if (p.amode != A_CONV3_UP || p.N != 32 || p.stride != 1 || (p.cc & 31) || p.cc > 128) return false;
  if (p.emode != E_STORE && p.emode != E_HEAD) return false;
  if (p.emode == E_STORE && ((p.ldo & 3) || p.res0 || p.res1)) return false;
  if (p.uh < 2 || p.uw < 1 || p.ch < 1 || p.cw < 1 || p.oh != p.uh) return false;
  if (!upconv_enabled()) return false;
  const float sy = (float)(p.ch - 1) / (float)(p.uh - 1);
  const int tiles_y = (p.oh + UTH - 1) / UTH;
  for (int ty = 0; ty < tiles_y; ++ty) {
    const int iy0 = ty * UTH - 1;
    const int first = iy0 < 0 ? 0 : iy0;
    const int last = iy0 + UPH - 1 < p.uh - 1 ? iy0 + UPH - 1 : p.uh - 1;
    const int a0 = (int)(sy * (float)first);
    const int l0 = (int)(sy * (float)last);
    const int b1 = l0 + (l0 < p.ch - 1 ? 1 : 0);
    if (b1 - a0 + 1 > USR) return false;
  }
  return true;
}

// persistent grid: workgroups per CU the LDS allows x 256 CUs (grids up to
// that size run one tile per workgroup)
template <int NCH>
int upconv_grid() {
  constexpr int lds = UPATCH + UHBUF + 9 * (NCH > 1 ? 1 : NCH) * 32 * 64;
  const int per_cu = 163840 / lds < 4 ? 163840 / lds : 4;
  return 256 * (per_cu > 0 ? per_cu : 1);
}
template <int NCH, int EM>
void launch_upconv_n(const GemmParams& p, long long tiles, hipStream_t st) {
  const int grid = upconv_grid<NCH>();
  if (tiles > grid)
    hipLaunchKernelGGL((upconv_kernel<NCH, EM, true>), dim3((unsigned)grid), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL((upconv_kernel<NCH, EM, false>), dim3((unsigned)tiles), dim3(512), 0, st, p);
}

template <int EM>
hipError_t launch_upconv(const GemmParams& p, hipStream_t st) {
  const long long tiles = (long long)p.cb * ((p.oh + UTH - 1) / UTH) * ((p.ow + UTW - 1) / UTW);
  if (tiles <= 0) return hipSuccess;
  if (tiles >= (1ll << 31)) return hipErrorInvalidValue;
  switch (p.cc / 32) {
    case 1: launch_upconv_n<1, EM>(p, tiles, st); break;
    case 2: launch_upconv_n<2, EM>(p, tiles, st); break;
    case 3: launch_upconv_n<3, EM>(p, tiles, st); break;
    case 4: launch_upconv_n<4, EM>(p, tiles, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

bool conv_direct_supported(const GemmParams& p) {
  if (p.cc % 32) return false;
  if (p.amode == A_CONV3_UP) return p.stride == 1;
  return p.stride == 1 || p.stride == 2;
}

// The direct conv (conv3_kernel) reads an upsampled res1 in its epilogue
// (GemmParams::res1_up, switch "resize_fold"): true when launch_conv3 routes
// p there -- a stride-1 E_STORE 3x3 conv that the persistent 64-channel conv
// does not take -- and the map has at most 64 channels.  (launch_gemm checks
// the split-K and im2col routes first.)  ViT-S B = 1 (64 features): the
// three resize launches gone, 0.7493 -> 0.7463 ms per forward; ViT-L B = 1's
// 256-channel 148^2 conv paid more for the 32 gathers per pixel than the
// launch costs (3.187 -> 3.197 ms), so wider maps keep the launch
// (profiles/r06_resize_fold.txt).
bool conv3_takes_res1_up(const GemmParams& p) {
  return knob(KNOB_RESIZE_FOLD) && p.amode == A_CONV3 && p.emode == E_STORE && p.stride == 1 && p.N <= 64 &&
         conv_direct_supported(p) && conv64p_mode(p) < 0 && p.ldo == p.N && (p.N & 7) == 0 && p.res1_uh > 0 &&
         p.res1_uw > 0;
}

hipError_t launch_conv3(const GemmParams& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (!conv_direct_supported(p) || (p.N & 7) || (p.ldw & 63) || p.ldw < 9 * p.cc) return hipErrorInvalidValue;
  const bool up = p.amode == A_CONV3_UP;
  if (up && upconv_eligible(p)) return p.emode == E_HEAD ? launch_upconv<E_HEAD>(p, st) : launch_upconv<E_STORE>(p, st);
  const bool ck64 = (p.cc % 64) == 0 && p.stride == 1;
  if (p.emode == E_HEAD) {
    if (p.N != 32 || p.stride != 1) return hipErrorInvalidValue;
    if (up) return ck64 ? conv_tiles<64, 1, true, E_HEAD>(p, st) : conv_tiles<32, 1, true, E_HEAD>(p, st);
    return ck64 ? conv_tiles<64, 1, false, E_HEAD>(p, st) : conv_tiles<32, 1, false, E_HEAD>(p, st);
  }
  if (p.emode != E_STORE) return hipErrorInvalidValue;
  hipError_t err;
  if (!up && conv64p_launch(p, st, err)) return err;
  if (up) return ck64 ? conv_tiles<64, 1, true, E_STORE>(p, st) : conv_tiles<32, 1, true, E_STORE>(p, st);
  if (p.stride == 2) return conv_tiles<32, 2, false, E_STORE>(p, st);
  return ck64 ? conv_tiles<64, 1, false, E_STORE>(p, st) : conv_tiles<32, 1, false, E_STORE>(p, st);
}

}  // namespace mde
