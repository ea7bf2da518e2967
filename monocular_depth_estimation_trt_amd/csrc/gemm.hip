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
// Structure (cdna_hip_programming.md section 5, "step-3 structure"):
//  * BM x BN x 64 block tile, WM x WN waves (4), each wave (BM/WM) x (BN/WN)
//    as 16x16 MFMA tiles, two 32-deep MFMA k-substeps per K-step;
//  * operands staged global -> LDS with global_load_lds_dwordx4 (no VGPR
//    round trip), two LDS stages, one barrier per K-step; LDS rows are 128 B
//    (64 halves) with chunk swizzle c ^ (row & 7) applied on the SOURCE
//    address (the LDS image is lane-linear) and on the fragment read, which
//    makes the ds_read_b128 fragment reads conflict-free;
//  * implicit-im2col A: each lane computes its own source pixel; padding
//    taps read a zero line (a glds lane can't be masked, it can be redirected);
//  * the bilinear-upsampled conv A (A_CONV3_UP) is register-staged because
//    every element is a 4-tap blend;
//  * MFMA issued with W as the A operand, so each lane owns 4 consecutive
//    output columns of one row: the fused epilogue (tile_epilogue.h) stores
//    8 B (f16) / 16 B (f32) per lane straight from the accumulators.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"
#include "tile_epilogue.h"
#include "tuning.h"

#ifndef MDE_GEMM_BK
#define MDE_GEMM_BK 64
#endif
#ifndef MDE_XCD_REMAP
#define MDE_XCD_REMAP 1
#endif
#ifndef MDE_EPI_LDS
#define MDE_EPI_LDS 1  // row-major epilogues staged through LDS (whole-line stores)
#endif
#ifndef MDE_BK32_STAGES
#define MDE_BK32_STAGES 3  // ring depth of the BK 32 tiles (2: 33 KB, four workgroups per CU)
#endif
#ifndef MDE_GEMM_STAGES
#define MDE_GEMM_STAGES 2  // LDS ring depth for dense A (>2: counted-vmcnt pipeline)
#endif

// Phase-isolation hooks (MDE_EXP_NOLOOP / NOLOAD / NOMFMA / NOEPI) compile
// parts of the GEMM out and produce WRONG outputs: tools/ablate.py builds them
// as separate variant libraries only, with MDE_EXPERIMENT defined as well;
// _build.build_library never passes defines to the in-tree libmde_hip.so.
#if (defined(MDE_EXP_NOLOOP) || defined(MDE_EXP_NOLOAD) || defined(MDE_EXP_NOMFMA) || defined(MDE_EXP_NOEPI)) && \
    !defined(MDE_EXPERIMENT)
#error "MDE_EXP_* hooks need -DMDE_EXPERIMENT (variant libraries only, never the product build)"
#endif

namespace mde {

namespace {

__device__ __attribute__((aligned(64))) f16 g_zero_line[64];  // zero-initialised module global

MDE_DEV void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}

MDE_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int N>
MDE_DEV void wait_vm_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier that leaves LDS-DMA in flight (__syncthreads() would
// also drain vmcnt): own LDS reads retired, raw s_barrier, compiler fences.
MDE_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS tile geometry for a K-step of BK halves: rows of BK*2 bytes, 16-byte
// chunks; one glds wave-instruction (64 lanes x 16 B) fills RW rows.
template <int BK>
struct KGeo {
  static constexpr int ROWB = BK * 2;       // bytes per row
  static constexpr int CH = BK / 8;         // chunks per row
  static constexpr int RW = 64 / CH;        // rows per wave-instruction
  // physical chunk of logical chunk lc in row r (conflict-free ds_read_b128)
  static MDE_DEV int pch(int r, int lc) {
    if constexpr (BK == 64) return lc ^ (r & 7);
    else return lc ^ ((r >> 1) & 3);
  }
};

#ifdef MDE_GEMM_WPE  // tuning: minimum waves per SIMD (caps VGPRs so more workgroups share a CU)
#define MDE_GEMM_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MDE_GEMM_WPE)))
#else
#define MDE_GEMM_WPE_ATTR
#endif

// BK 32 (the short-K 128^2 dense stores): 3-stage ring = 48 KB and a half-size
// epilogue staging, capped at 168 VGPRs -- three workgroups per CU, so one
// workgroup's epilogue stores overlap the others' main loops
// STG > 0: ring depth forced (small grids: one workgroup per CU with
// STG - 1 K-steps in flight instead of two workgroups with one each)
// SPLIT: the fused split-K form (E_RESID / E_STORE over gridDim.y slices, the
// tail after the main loop) -- separate instantiations, so the whole-tile
// kernels carry none of its code or registers
template <int BM, int BN, int BK, int WM, int WN, int AM, int EM, int STG = 0, bool SPLIT = false>
__global__ void __launch_bounds__(WM * WN * 64) MDE_GEMM_WPE_ATTR
    __attribute__((amdgpu_waves_per_eu(STG == 0 && BK == 32 ? (WM * WN == 8 ? 4 : (MDE_BK32_STAGES > 2 ? 3 : 4)) : 1)))
    gemm_kernel(const GemmParams p) {
  using G = KGeo<BK>;
  constexpr int ROWB = G::ROWB, CH = G::CH;
  constexpr int NW = WM * WN;
  constexpr int NT = NW * 64;
  constexpr int TM = BM / (WM * 16);
  constexpr int TN = BN / (WN * 16);
  static_assert(TM * WM * 16 == BM && TN * WN * 16 == BN, "tile");
  // glds wave-instructions per tile (each fills RW rows); wave w issues
  // instructions w, w + NW, ... (APASS / BPASS slots, the last maybe partial)
  constexpr int AINS = BM / G::RW, BINS = BN / G::RW;
  static_assert(AINS * G::RW == BM && BINS * G::RW == BN, "tile rows vs glds rows");
  constexpr int APASS = (AINS + NW - 1) / NW, BPASS = (BINS + NW - 1) / NW;
  constexpr int STAGE = (BM + BN) * ROWB;
  // dense A: SG-deep ring, every wave issues exactly NPER glds per stage so a
  // counted vmcnt names "stage kt has landed"
  constexpr int SGWANT = STG > 0 ? STG : (BK == 32 ? MDE_BK32_STAGES : MDE_GEMM_STAGES);
  constexpr int SGMAX = 163840 / STAGE < SGWANT ? 163840 / STAGE : SGWANT;  // LDS limit
  // (implicit-im2col A too: its glds count per wave is the same every stage;
  // the register-staged upsampling A keeps the two-stage loop)
  constexpr int SG = (AM != A_CONV3_UP && AINS % NW == 0 && BINS % NW == 0 && SGMAX > 2) ? SGMAX : 2;
  constexpr int NPER = APASS + BPASS;
  static_assert(SG >= 2 && SG <= 4, "stages");
  // folded LayerNorm consumers: (mean, var) of the tile's rows behind the ring
  constexpr bool LNF = AM == A_DENSE && (EM == E_QKV || EM == E_STORE);
  constexpr int LNB = LNF ? BM * 8 : 0;
  // fused split-K: E_RESID / E_STORE launched with gridDim.y = S > 1 slices
  // (the split tail after the main loop; gridDim.y = 1 is the plain tile)
  constexpr bool FSPLIT = SPLIT && (EM == E_RESID || EM == E_STORE) && AM != A_CONV3_UP;
  static_assert(!SPLIT || FSPLIT, "fused split-K: E_RESID / E_STORE over dense or im2col A");
  __shared__ __attribute__((aligned(16))) char smem[SG * STAGE + LNB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int ntn = (p.N + BN - 1) / BN;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
  // (bid % 8 shares an L2), so give each XCD a contiguous run of tiles
  // (tn fastest) -- the N-tiles of one row block then share A in one L2.
  // Bijective for any grid size (cdna_hip_programming.md section 5).
  int bid = blockIdx.x, slice = blockIdx.y;
  if constexpr (EM == E_PARTIAL || FSPLIT) {  // (gridDim.y = 1: the same order as below)
    // split-K: remap over (slice, tile) so each XCD takes a contiguous run of
    // one slice's tiles -- its L2 then holds that K-slice of W and of the A
    // rows, not every slice of both (a slice-blind order streams all of W
    // through every XCD)
    if (MDE_XCD_REMAP) {
      const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
      slice = lin / gridDim.x;
      bid = lin - slice * gridDim.x;
    }
  } else {
    if (MDE_XCD_REMAP) bid = xcd_remap(bid, gridDim.x);
  }
  int tm, tn;
  tile_of(bid, (p.M + BM - 1) / BM, ntn, AM == A_DENSE ? tile_group_m(p.N, p.K, BM) : 1, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- glds lane geometry: lane -> (row within a wave-instruction, chunk)
  const int lrow = lane / CH;
  const int lch = G::pch(lrow, lane % CH);  // logical chunk (involution: pch(pch(c)) = c)

  // ---- A operand state ----
  const f16* arow[APASS];
  int iy0[APASS], ix0[APASS];
  bool rv[APASS];
  if constexpr (AM != A_CONV3_UP) {
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      const int r = (wave + i * NW) * G::RW + lrow;
      const int gm = m0 + r;
      rv[i] = gm < p.M;
      const int gmc = rv[i] ? gm : (p.M - 1);
      if constexpr (AM == A_DENSE) {
        const int ar = p.a_tok > 1 ? gmc + gmc / (p.a_tok - 1) + 1 : gmc;
        arow[i] = reinterpret_cast<const f16*>(p.A) + (size_t)ar * p.lda;
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
  }
  // register-staged A (A_CONV3_UP): thread -> 16B chunks (row, logical chunk)
  constexpr int UPC = (AM == A_CONV3_UP) ? (BM * CH) / NT : 1;
  static_assert(AM != A_CONV3_UP || (BM * CH) % NT == 0, "up-conv staging");
  const f16* urow[UPC];
  int uy0[UPC], ux0[UPC];
  bool uv[UPC];
  const int ulch = tid % CH;
  if constexpr (AM == A_CONV3_UP) {
#pragma unroll
    for (int i = 0; i < UPC; ++i) {
      const int r = tid / CH + i * (NT / CH);
      const int gm = m0 + r;
      uv[i] = gm < p.M;
      const int gmc = uv[i] ? gm : 0;
      const int hw = p.oh * p.ow;
      const int b = gmc / hw;
      const int rem = gmc - b * hw;
      const int oy = rem / p.ow, ox = rem - (rem / p.ow) * p.ow;
      uy0[i] = oy - 1;
      ux0[i] = ox - 1;
      urow[i] = reinterpret_cast<const f16*>(p.A) + (size_t)b * p.ch * p.cw * p.cc;
    }
  }
  // K-tiles [kt0, kt0 + nk): all of K, or this workgroup's split-K slice
  int nk = (p.K + BK - 1) / BK, kt0 = 0;
  if constexpr (EM == E_PARTIAL || FSPLIT) {
    const int per = (nk + (int)gridDim.y - 1) / (int)gridDim.y;
    kt0 = slice * per;
    nk = min(nk - kt0, per);  // >= 1: the launcher uses at most nk slices of ceil(nk / S) tiles
  }
#ifdef MDE_EXP_NOLOOP
  if (p.M > 0) nk = 0;
#endif

  // conv K position (tap, c0) of this lane's chunk at K-tile kt0, advanced by
  // BK per step
  int tap = 0, c0 = kt0 * BK + (AM == A_CONV3_UP ? ulch : lch) * 8;
  if constexpr (AM != A_DENSE) {
    tap = c0 / p.cc;
    c0 -= tap * p.cc;
  }
  float usy = 0.f, usx = 0.f;
  if constexpr (AM == A_CONV3_UP) {
    usy = ac_scale(p.ch, p.uh);
    usx = ac_scale(p.cw, p.uw);
  }

  // ---- B operand (weights [Npad][ldw], ldw % 64 == 0) ----
  const f16* wbase = reinterpret_cast<const f16*>(p.W) + (size_t)(n0 + wave * G::RW + lrow) * p.ldw + lch * 8;
  auto aslot = [&](int i) { return (wave + i * NW) * G::RW * ROWB; };  // LDS row offset of slot i

  f16x8 ru[UPC];

  auto issue = [&](int kt, int buf) {
#ifdef MDE_EXP_NOLOAD
    if (p.M > 0) return;
#endif
    char* sbase = smem + buf * STAGE;
    const int k0 = (kt + kt0) * BK;
#pragma unroll
    for (int i = 0; i < BPASS; ++i)
      if (BINS % NW == 0 || wave + i * NW < BINS)
        glds16(wbase + (size_t)i * NW * G::RW * p.ldw + k0, sbase + BM * ROWB + aslot(i));
    if constexpr (AM == A_DENSE) {
      const int k = k0 + lch * 8;
      const int kk = k < p.K ? k : 0;  // K tail: W is zero there, any finite A will do
#pragma unroll
      for (int i = 0; i < APASS; ++i)
        if (AINS % NW == 0 || wave + i * NW < AINS) glds16(arow[i] + kk, sbase + aslot(i));
    } else if constexpr (AM == A_CONV3) {
      const bool kv = (k0 + lch * 8) < p.K;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
      for (int i = 0; i < APASS; ++i) {
        const int iy = iy0[i] + ky, ix = ix0[i] + kx;
        const bool ok = rv[i] && kv && iy >= 0 && iy < p.ch && ix >= 0 && ix < p.cw;
        const f16* src = ok ? arow[i] + ((size_t)iy * p.cw + ix) * p.cc + c0 : g_zero_line;
        if (AINS % NW == 0 || wave + i * NW < AINS) glds16(src, sbase + aslot(i));
      }
    } else {  // A_CONV3_UP: blend 4 taps of the source map in registers
      const bool kv = (k0 + ulch * 8) < p.K;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
      for (int i = 0; i < UPC; ++i) {
        f16x8 v = zero8();
        const int iy = uy0[i] + ky, ix = ux0[i] + kx;
        if (uv[i] && kv && iy >= 0 && iy < p.uh && ix >= 0 && ix < p.uw) {
          int y0, y1, x0, x1;
          float ly0, ly1, lx0, lx1;
          ac_index(usy, iy, p.ch, y0, y1, ly0, ly1);
          ac_index(usx, ix, p.cw, x0, x1, lx0, lx1);
          const f16* base = urow[i] + c0;
          const f16x8 a = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * p.cw + x0) * p.cc);
          const f16x8 b = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * p.cw + x1) * p.cc);
          const f16x8 c = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * p.cw + x0) * p.cc);
          const f16x8 d = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * p.cw + x1) * p.cc);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = (f16)(ly0 * (lx0 * (float)a[j] + lx1 * (float)b[j]) + ly1 * (lx0 * (float)c[j] + lx1 * (float)d[j]));
        }
        ru[i] = v;
      }
    }
    if constexpr (AM != A_DENSE) {
      c0 += BK;
      while (c0 >= p.cc) { c0 -= p.cc; ++tap; }
    }
  };

  auto commit_up = [&](int buf) {
    if constexpr (AM == A_CONV3_UP) {
      char* sA = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < UPC; ++i) {
        const int r = tid / CH + i * (NT / CH);
        *reinterpret_cast<f16x8*>(sA + r * ROWB + G::pch(r, ulch) * 16) = ru[i];
      }
    }
  };

  // acc[i][j] holds C^T for the 16x16 block (m-block i, n-block j): the MFMA is
  // issued with W as its A operand, so lane l owns row m = .. + (l & 15) and the
  // four consecutive columns n = .. + 4(l >> 4) + r -- stores are 8/16 B wide.
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma_stage = [&](int cur) {
#ifdef MDE_EXP_NOMFMA
    if (p.M > 0) return;
#endif
    const char* sA = smem + cur * STAGE;
    const char* sB = sA + BM * ROWB;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      f16x8 fa[TM], fb[TN];
      const int lc = 4 * s + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 16 + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const f16x8*>(sA + r * ROWB + G::pch(r, lc) * 16);
        if constexpr (AM == A_CONV3) {
          if (p.relu_in) fa[i] = relu8(fa[i]);
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * TN * 16 + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const f16x8*>(sB + r * ROWB + G::pch(r, lc) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
    }
  };
  // folded LayerNorm: the tile's rows' (mean, var) from the producers'
  // slice partials.  Each wave takes BM / NW rows (no row loaded twice),
  // the 4 lanes that share a row (lane >> 4) take slices q, q + 4, ...
  // (D % 128 == 0, <= 32 slices), the loads issued behind the prologue's
  // stage 0 whose wait covers them; Chan et al.'s merge, then (mean, var)
  // to LDS behind the ring -- the prologue barrier publishes them.
  float4 c1v[TN];  // lnc1 of this lane's columns (an epilogue load would cost every tile an L2 round trip)
  auto ln_partial_loads = [&] {
    if constexpr (LNF) {
      if (p.lnst_in) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * TN * 16 + j * 16 + (lane >> 4) * 4;
          c1v[j] = *reinterpret_cast<const float4*>(p.lnc1 + (n < p.N ? n : 0));
        }
        const float2* st2 = reinterpret_cast<const float2*>(p.lnst_in);
        const float invd = 1.f / (float)(p.lnst_ns * 32);
        const int kp = p.lnst_ns >> 2;  // slices per lane (wave-uniform)
        constexpr int RPW = BM / NW;    // rows per wave: 16 or 32
        constexpr int G = (RPW + 15) / 16;
        // all loads first, unpredicated (slices past kp re-read slice q, an
        // L1 hit, and are masked below): one latency round trip, no branches
        float2 t[G][8];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int m = m0 + wave * RPW + g * 16 + (lane & 15);
          const int mr = m < p.M ? m : p.M - 1;
          const int mc = p.a_tok > 1 ? mr + mr / (p.a_tok - 1) + 1 : mr;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int sl = (lane >> 4) + (k < kp ? 4 * k : 0);
            t[g][k] = st2[(size_t)sl * p.lnst_rows + mc];
          }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int r = wave * RPW + g * 16 + (lane & 15);
          float mean, var;
          ln_merge_stats(t[g], kp, invd, mean, var);
          // only this wave's rows (RPW 8: lanes 8..15 hold the next wave's)
          if ((lane >> 4) == 0 && g * 16 + (lane & 15) < RPW)
            *reinterpret_cast<float2*>(smem + SG * STAGE + r * 8) = make_float2(mean, var);
        }
      }
    }
  };
  if constexpr (SG == 2) {
    issue(0, 0);
    commit_up(0);
    ln_partial_loads();
    wait_vm();
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
      mma_stage(cur);
      if (kt + 1 < nk) commit_up(cur ^ 1);
      wait_vm();
      __syncthreads();
    }
  } else {
    // SG-1 stages in flight; one barrier per K-step.  At step kt the stages
    // issued after kt are min(nk-1-kt, SG-2): wait until only they remain.
#pragma unroll
    for (int s = 0; s < SG - 1; ++s)
      if (s < nk) issue(s, s);
    ln_partial_loads();
    for (int kt = 0; kt < nk; ++kt) {
      const int after = min(nk - 1 - kt, SG - 2);
      if (after >= 2) wait_vm_n<2 * NPER>();
      else if (after == 1) wait_vm_n<NPER>();
      else wait_vm_n<0>();
      lds_barrier();  // stage kt visible to all waves; stage kt-1 fully consumed
      if (kt + SG - 1 < nk) issue(kt + SG - 1, (kt + SG - 1) % SG);
      mma_stage(kt % SG);
    }
  }

  // ---- fused split-K tail (gridDim.y = S > 1): each slice publishes its
  // fp32 accumulators to its slot of p.partial in register order (16-B words
  // thread-major per 16x16 block: coalesced), then bumps the tile's arrival
  // counter p.tile_cnt[bid].  The LAST of the S slices to arrive adds the
  // slots in slice order 0..S-1 -- the order of the reduce kernels, so the
  // sum does not depend on which slice arrives last -- re-zeroes the counter
  // for the next launch and runs the tile's own epilogue; the others exit.
  // No workgroup ever waits on another.  The slices of a tile sit on
  // different XCDs (slice-aware order above), so slots and counter go
  // through system-scope (sc0 sc1) accesses that bypass the per-XCD L2s
  // instead of a cache-wide __threadfence() write-back per slice.
  if constexpr (FSPLIT) {
    const int S = (int)gridDim.y;
    if (S > 1) {
      constexpr int NB = TM * TN;
      typedef unsigned long long u64;
      u64* const slots = reinterpret_cast<u64*>(p.partial);
      const size_t slot_words = (size_t)NB * NT * 2;
      auto word = [&](int s, int blk) {
        return slots + ((size_t)s * gridDim.x + bid) * slot_words + ((size_t)blk * NT + tid) * 2;
      };
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          u64* d = word(slice, i * TN + j);
          const f32x4 a = acc[i][j];
          __hip_atomic_store(d, (u64)__float_as_uint(a[0]) | ((u64)__float_as_uint(a[1]) << 32), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(d + 1, (u64)__float_as_uint(a[2]) | ((u64)__float_as_uint(a[3]) << 32), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      wait_vm();  // this wave's slot stores have completed
      __shared__ int s_last;
      __syncthreads();
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(p.tile_cnt + bid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_last = old == S - 1;
        if (old == S - 1) __hip_atomic_store(p.tile_cnt + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();
      if (!s_last) return;
      auto load = [&](int s, f32x4 (&v)[TM][TN]) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (s == slice) {
              v[i][j] = acc[i][j];
            } else {
              const u64* q = word(s, i * TN + j);
              const u64 lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              const u64 hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              v[i][j] = f32x4{__uint_as_float((unsigned)lo), __uint_as_float((unsigned)(lo >> 32)),
                              __uint_as_float((unsigned)hi), __uint_as_float((unsigned)(hi >> 32))};
            }
          }
      };
      // two slices per batch of loads (one memory round trip), added in order
      f32x4 sum[TM][TN];
      for (int s0 = 0; s0 < S; s0 += 2) {
        f32x4 va[TM][TN], vb[TM][TN];
        load(s0, va);
        if (s0 + 1 < S) load(s0 + 1, vb);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            sum[i][j] = s0 == 0 ? va[i][j] : sum[i][j] + va[i][j];
            if (s0 + 1 < S) sum[i][j] += vb[i][j];
          }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = sum[i][j];
    }
  }

#ifdef MDE_EXP_NOEPI
  if (p.M > 0) return;
#endif
  // ---- folded LayerNorm (GemmParams::lnst_in): A held the raw f16 residual
  // rows and W = W_ln * gamma; per row, mean and rstd from the producer's
  // 32-column partials (fp32), then acc := rstd * acc - rstd * mean * lnc1[n]
  // (the epilogue adds bias = b + W_ln beta).  mean and variance from the
  // slices' (sum, M2) by Chan et al.'s pairwise merge, fp32.
  if constexpr (AM == A_DENSE && (EM == E_QKV || EM == E_STORE)) {
    if (p.lnst_in) {
      // the rows' (mean, var), merged in the prologue (ln_partial_loads)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float2 mv = *reinterpret_cast<const float2*>(smem + SG * STAGE + (wm * TM * 16 + i * 16 + (lane & 15)) * 8);
        const float mean = mv.x;
        const float rstd = rsqrtf(__fadd_rn(mv.y, p.ln_eps));
        const float nm = -rstd * mean;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float4 c = c1v[j];
          acc[i][j][0] = fmaf(rstd, acc[i][j][0], nm * c.x);
          acc[i][j][1] = fmaf(rstd, acc[i][j][1], nm * c.y);
          acc[i][j][2] = fmaf(rstd, acc[i][j][2], nm * c.z);
          acc[i][j][3] = fmaf(rstd, acc[i][j][3], nm * c.w);
        }
      }
    }
  }

  // ---- epilogue: lane owns (m, n..n+3) per block ----
  int mrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * TM * 16 + i * 16 + (lane & 15);
    mrow[i] = m < p.M ? m : -1;
  }
  // LDS-staged epilogue when every wave's fp32 tile fits in the ring, or
  // (HALF) half of it: f16 rows / two fp32 row passes (store_tile_lds)
  constexpr bool STG_FULL = BM * BN * 4 <= SG * STAGE;
  constexpr int STG_HALF = !STG_FULL && BM * BN * 2 <= SG * STAGE;
  constexpr bool EPI_LDS = MDE_EPI_LDS && (STG_FULL || STG_HALF);
  bool staged = false;
  if constexpr (EPI_LDS) {
    if constexpr (SG > 2) lds_barrier();  // the ring's last stage may still be read by other waves
    const int m0w = m0 + wm * TM * 16;
    staged = store_tile_lds<EM, TM, TN, STG_HALF>(
        p, acc, [&](int row) { return m0w + row < p.M ? m0w + row : -1; }, n0 + wn * TN * 16, lane,
        smem + wave * (TM * 16) * (TN * 16) * (STG_HALF ? 2 : 4));
  }
  if (!staged) store_tile<EM, TM, TN>(p, acc, mrow, n0 + wn * TN * 16 + (lane >> 4) * 4, lane, slice);
}

template <int BM, int BN, int WM, int WN, int AM, int EM, int BKSEL = MDE_GEMM_BK, int STG = 0>
hipError_t run(const GemmParams& p, hipStream_t st) {
  const int gm = (p.M + BM - 1) / BM, gn = (p.N + BN - 1) / BN;
  const long long blocks = (long long)gm * gn;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BKSEL, WM, WN, AM, EM, STG>), dim3((unsigned)blocks), dim3(WM * WN * 64), 0,
                     st, p);
  return hipGetLastError();
}

// dense short-K stores (K <= 768) take the BK 32 / 3-stage / three-per-CU
// 128^2 kernel; 128^2 tiles once the grid holds at least kBigTileMin of them
constexpr int kBk32Kmax = 768;
constexpr long long kBigTileMin = 240;

// 64^2 tiles of a grid that fits two workgroups per CU run a 4-deep ring (64
// KB: 48 KB of K-steps in flight instead of 16): the batch-1 linears and
// split-K slices are latency-bound on their one K-step in flight.  Switch
// "deep64" (tuning.h).
bool deep64(long long wgs) { return knob(KNOB_DEEP64) && wgs <= 512; }

// 128^2 tiles of a grid under two workgroups per CU run 8 waves (2 x 4 of 64
// x 32): a lone workgroup per CU otherwise has one wave per SIMD to cover its
// own LDS reads and barrier waits.  ViT-L B=1 fc1 0.665 -> 0.635, fc2 (split
// slices) 0.830 -> 0.809 ms per forward (profiles/r03_v4_bench_vitl1w8).
// Switch "w8small".
bool w8small(long long wgs) { return knob(KNOB_W8SMALL) && wgs < 512; }

// Residual updates whose 64^2 grid is under one workgroup per CU (ViT-S
// batch 1: fc2 K 1536 and proj K 384 at 1370 x 384, 132 tiles) on 32 x 64
// tiles (258 workgroups, the whole K loop, 4-deep ring): no split-K slices
// and no reduce launch for fc2 (round 5 measured ViT-S B = 1 0.792 -> 0.765
// ms per forward, profiles/r05_b1_resid_narrow.txt; not bit-identical to the
// split path -- one K loop instead of three slices added in order).  Switch
// "narrow_resid".
bool narrow_resid(const GemmParams& p) {
  if (!knob(KNOB_NARROW_RESID) || p.amode != A_DENSE || p.emode != E_RESID) return false;
  const long long t64 = (long long)((p.M + 63) / 64) * ((p.N + 63) / 64);
  const long long t32 = (long long)((p.M + 31) / 32) * ((p.N + 63) / 64);
  return t64 < 256 && t32 >= 192 && t32 <= 512;
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
    if constexpr (AM == A_DENSE && EM == E_RESID) {
      // residual updates with at least two rounds of 256 x 128 tiles (8 waves,
      // BK 32 x 3 stages, two workgroups per CU): 25 % fewer L2 -> LDS bytes per
      // FLOP and twice the rows per workgroup for the read-modify-write
      // epilogue.  ViT-S B = 48, same box, two passes: proj 0.685 / 0.690 ->
      // 0.611 / 0.606 ms, fc2 1.493 / 1.503 -> 1.401 / 1.394 ms per forward,
      // qkv / fc1 unchanged on this tile (profiles/r03_v3_*)
      const long long t256 = (long long)((p.M + 255) / 256) * ((p.N + 127) / 128);
      if (t256 >= 512) return run<256, 128, 4, 2, AM, EM, 32>(p, st);
      // short-K residual updates (ViT-S proj, K 384) on 128 x 64 tiles: 48 KB
      // LDS with full fp32 staging, three workgroups per CU (B=28: proj
      // 0.427/0.431 -> 0.419/0.425 ms per forward, two same-box runs; fc2 at
      // K 1536 loses, 0.86 -> 0.97)
      if (p.K <= 384 && big >= kBigTileMin) return run<128, 64, 4, 1, AM, EM>(p, st);
      if (narrow_resid(p)) return run<32, 64, 2, 2, AM, EM, 64, 4>(p, st);
    }
    if (big >= kBigTileMin) {
      // short-K stores (ViT-S/B qkv, fc1: K 384 / 768 -> 6-12 K-steps, the
      // epilogue a third of the launch) gain from the third workgroup per CU
      // (B=28 ViT-S: fc1 1.30 -> 1.10 ms, qkv 0.97 -> 0.89 per forward); the
      // residual updates and K >= 1024 do not (fc2 0.85 -> 0.96 with two fp32
      // staging passes, proj 0.43 -> 0.45 even with f16 staging of the
      // update; ViT-L B=8 qkv 2.56 -> 2.67)
      if constexpr (AM == A_DENSE && (EM == E_STORE || EM == E_QKV)) {
        if (p.K <= kBk32Kmax) return run<128, 128, 2, 2, AM, EM, 32>(p, st);
        if (w8small(big)) return run<128, 128, 2, 4, AM, EM>(p, st);
      }
      // the patch embed (K 672) and the resize-layer ConvTs (K 48 / 96) too:
      // ViT-S B = 48, per layer, two same-box runs: patch_embed 86.4 / 85.8 ->
      // 83.5 / 83.8 us, convT4 57.8 / 59.1 -> 48.6 / 50.6, convT2 34.7 / 34.8
      // -> 31.4 / 32.4 (profiles/r05_patch_convt_bk32.txt)
      if constexpr (AM == A_DENSE && (EM == E_PATCH || EM == E_CONVT)) {
        if (p.K <= kBk32Kmax) return run<128, 128, 2, 2, AM, EM, 32>(p, st);
      }
      return run<128, 128, 2, 2, AM, EM>(p, st);
    }
    if constexpr (AM == A_DENSE) {
      const long long t64 = (long long)((p.M + 63) / 64) * ((p.N + 63) / 64);
      if (deep64(t64)) return run<64, 64, 2, 2, AM, EM, 64, 4>(p, st);
      // (a 3-deep ring for grids of 512-768 tiles measured no gain: ViT-S B=1
      // fc1, 528 tiles, 0.134 -> 0.136 ms per forward, profiles/r03_v11_*)
    }
    return run<64, 64, 2, 2, AM, EM>(p, st);
  }
}

// Direct-conv tiles are 8 x 16 output pixels per image: on small maps most of
// a tile is padding (19^2 -> 47 % useful).  The implicit-im2col GEMM tiles the
// flattened B*oh*ow pixel axis instead, which wins for stride-2 convs and for
// wide-K convs on maps that fill the 8 x 16 grid badly (MI355X, B=32: the
// 37^2 -> 19^2 s2 384->384 conv 0.161 -> 0.069 ms, 19^2 384->64 0.047 ->
// 0.042; narrow 64-channel convs stay direct: 0.015 vs 0.022).
bool prefer_im2col(const GemmParams& p) {
  if (p.amode != A_CONV3 || p.emode != E_STORE) return false;
  if (p.stride == 2) return true;
  const double tiles = (double)((p.oh + 7) / 8 * 8) * (double)((p.ow + 15) / 16 * 16);
  return p.cc >= 256 && (double)p.oh * p.ow < 0.6 * tiles;
}

// E_STORE split-K: slices of the K loop on 64^2 tiles into the fp32
// workspace, then launch_splitk_store sums them in slice order and runs the
// epilogue (deterministic).  For grids that leave most of the chip idle: the
// small-batch DPT convs on 19^2 / 37^2 / 74^2 maps walk K = 9 Cin (up to
// 9216) in a few dozen workgroups (ViT-L B = 1: layer3_rn 30 direct-conv
// workgroups x 16 channel chunks, 129 us).  Returns the slice count (1 = no split).
int store_split_slices(const GemmParams& p) {
  if (p.emode != E_STORE || !p.partial || p.partial_cap == 0 || p.lnst_in || p.lnst_out) return 1;
  if (p.amode != A_DENSE && p.amode != A_CONV3) return 1;
  if (p.amode == A_CONV3 && p.stride != 1 && p.stride != 2) return 1;
  if (!knob(KNOB_SPLITK)) return 1;
  const int nk = (p.K + 63) / 64;
  const long long t64 = (long long)((p.M + 63) / 64) * ((p.N + 63) / 64);
  // workgroups of the unsplit launch
  long long wgs;
  if (p.amode == A_CONV3 && conv_direct_supported(p) && !prefer_im2col(p)) {
    const int bn = p.N <= 32 ? 32 : (p.N <= 64 ? 64 : 128);
    wgs = (long long)p.cb * ((p.oh + 7) / 8) * ((p.ow + 15) / 16) * ((p.N + bn - 1) / bn);
  } else {
    const long long big = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128);
    wgs = big >= kBigTileMin ? big : t64;
  }
  // at least 12 K-steps: the 64-channel convs of the ViT-S DPT (K 576, 9
  // steps) run better unsplit (ViT-S B=1 0.925 -> 0.902 ms per forward with
  // 12 vs 8; 16: 0.909)
  if (nk < 12) return 1;
  int S;
  if (wgs >= 256) {
    // a grid just over one workgroup per CU with a long K loop -- ViT-S B =
    // 48 layer4_rn, 271 64^2 tiles x 54 K-steps, 43 us at one workgroup per
    // CU -- takes two slices (2-stage ring, all resident)
    if (wgs >= 384 || nk < 48) return 1;
    S = 2;
  } else {
    // fill two workgroups per CU without spilling into a third: the slices then
    // run the 4-deep ring (deep64), which a 513th workgroup would forfeit
    S = (int)((512 + t64 - 1) / t64);
    if (512 / t64 >= 2) S = (int)(512 / t64);  // (independent of the "deep64" switch: same slices either way)
  }
  S = S < nk / 4 ? S : nk / 4;  // >= 4 K-steps per slice
  S = S < 16 ? S : 16;
  while (S > 1 && (size_t)S * p.M * p.N > p.partial_cap) --S;
  if (S <= 1) return 1;
  const int per = (nk + S - 1) / S;
  return (nk + per - 1) / per;  // every slice non-empty
}

// the fused split-K form (GemmParams::tile_cnt) applies: switch on, counters
// for every tile and S slots of BM x BN fp32 per tile in `partial`
bool fused_split(const GemmParams& p, long long tiles, int S, int BM, int BN) {
  return knob(KNOB_SPLITK_FUSED) && p.tile_cnt && tiles <= p.tile_cnt_cap &&
         (size_t)S * (size_t)tiles * (size_t)BM * BN <= p.slot_cap && ((uintptr_t)p.partial & 15) == 0;
}

template <int AM>
hipError_t launch_split_store(const GemmParams& p, int S, hipStream_t st) {
  const unsigned tiles = (unsigned)(((p.M + 63) / 64) * ((p.N + 63) / 64));
  if (fused_split(p, tiles, S, 64, 64)) {
    if (deep64((long long)tiles * S))
      hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, AM, E_STORE, 4, true>), dim3(tiles, (unsigned)S),
                         dim3(256), 0, st, p);
    else
      hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, AM, E_STORE, 0, true>), dim3(tiles, (unsigned)S),
                         dim3(256), 0, st, p);
    return hipGetLastError();
  }
  GemmParams q = p;
  q.emode = E_PARTIAL;
  q.x32 = p.partial;
  q.ldo = p.N;
  if (deep64((long long)tiles * S))
    hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, AM, E_PARTIAL, 4>), dim3(tiles, (unsigned)S), dim3(256),
                       0, st, q);
  else
    hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, AM, E_PARTIAL>), dim3(tiles, (unsigned)S), dim3(256), 0,
                       st, q);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_splitk_store(p.partial, S, p, st);
}

// folded-LayerNorm operands consistent with the problem (launch_gemm)
bool lnst_valid(const GemmParams& p) {
  if (p.lnst_out && !MDE_EPI_LDS) return false;
  return !((p.lnst_ns * 32 != (p.lnst_out ? p.N : p.K)) ||
           (p.lnst_in && (p.lnst_ns > 32 || (p.lnst_ns & 3) ||
                          p.lnst_rows != (p.a_tok > 1 ? p.M / (p.a_tok - 1) * p.a_tok : p.M) ||
                          (p.a_tok > 1 && p.M % (p.a_tok - 1)))) ||
           (p.lnst_out && p.lnst_rows < (p.emode == E_PATCH ? p.M / p.npatch * p.T : p.M)) ||
           (p.lnst_in && (!p.lnc1 || p.amode != A_DENSE)) || (p.lnst_out && !p.xh));
}

}  // namespace

int gemm_store_split_slices(const GemmParams& p) { return store_split_slices(p); }

hipError_t launch_gemm(const GemmParams& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.res1_up) {
    // res1 = upsample(res1_up): read through it by the direct conv's
    // epilogue, or written into res1 first for every other route
    if (!p.res1 || p.amode != A_CONV3 || p.emode != E_STORE || p.res1_uh <= 0 || p.res1_uw <= 0 || (p.N & 7))
      return hipErrorInvalidValue;
    GemmParams q = p;
    if (store_split_slices(p) <= 1 && !prefer_im2col(p) && conv3_takes_res1_up(p)) {
      q.res1 = nullptr;
      return launch_conv3(q, st);
    }
    const hipError_t e = launch_resize(p.res1_up, const_cast<h16*>(p.res1), p.cb, p.res1_uh, p.res1_uw, p.N, p.oh,
                                       p.ow, st);
    if (e != hipSuccess) return e;
    q.res1_up = nullptr;
    return launch_gemm(q, st);
  }
  if (p.K <= 0 || (p.K & 7) || (p.N & 7) || (p.ldw & 63) || p.ldw < ((p.K + 63) / 64) * 64)
    return hipErrorInvalidValue;
  if (p.amode == A_DENSE && ((p.lda & 7) || p.lda < p.K)) return hipErrorInvalidValue;
  if (p.a_tok == 1 || p.a_tok < 0 || (p.a_tok > 1 && (p.amode != A_DENSE || p.emode != E_STORE || !p.lnst_in)))
    return hipErrorInvalidValue;
  if (p.amode != A_DENSE && (p.cc & 7)) return hipErrorInvalidValue;
  if ((p.emode == E_STORE || p.emode == E_RESID || p.emode == E_PATCH) && (p.ldo & 7)) return hipErrorInvalidValue;
  // E_CONVT stores 16 B per output pixel (f16x8 at pixel*ldo + co): ldo and
  // the base must keep every such store 16-B aligned (Depth Pro writes into
  // concat slots, out16 = base + sd0)
  if (p.emode == E_CONVT && ((p.cout & 7) || (p.ldo & 7) || p.ldo < p.cout || ((uintptr_t)p.out16 & 15)))
    return hipErrorInvalidValue;
  if (p.emode == E_HEAD && (p.N != 32 || p.amode == A_DENSE)) return hipErrorInvalidValue;
  if (const int S = store_split_slices(p); S > 1) {
    if ((p.ldo & 7) || ((uintptr_t)p.partial & 15)) return hipErrorInvalidValue;
    return p.amode == A_DENSE ? launch_split_store<A_DENSE>(p, S, st) : launch_split_store<A_CONV3>(p, S, st);
  }
  if (p.amode != A_DENSE && conv_direct_supported(p) && !prefer_im2col(p))
    return launch_conv3(p, st);
  if ((p.emode == E_RESID || p.emode == E_PATCH) && p.xh && ((uintptr_t)p.xh & 15)) return hipErrorInvalidValue;
  if (p.emode == E_RESID && p.splitk > 1 && p.partial && p.amode == A_DENSE && !narrow_resid(p)) {
    // small M, long K (B = 1 fc2: 132 64^2 tiles x 24 K-steps): S slices of
    // the K loop fill the chip, a second kernel adds them in slice order.
    // When 128^2 tiles x 4 slices still give >= 320 workgroups (ViT-L /
    // VGGT B = 1: 88 tiles), the 128^2 tiles halve the L2 -> LDS bytes per
    // FLOP of the 64^2 ones; `partial` holds 4 slices (engine contract)
    const int nk = (p.K + 63) / 64;
    const long long t128 = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128);
    const bool big = t128 * 4 >= 320 && nk >= 16;
    int S = big ? 4 : (p.splitk < nk ? p.splitk : nk);
    if (!big) {  // keep the 64^2 slices within two workgroups per CU (deep ring; same slices with "deep64" off)
      const long long t64 = (long long)((p.M + 63) / 64) * ((p.N + 63) / 64);
      while (S > 2 && t64 * S > 512) --S;
    }
    const int per = (nk + S - 1) / S;
    S = (nk + per - 1) / per;  // every slice non-empty
    const long long t64 = (long long)((p.M + 63) / 64) * ((p.N + 63) / 64);
    if (fused_split(p, big ? t128 : t64, S, big ? 128 : 64, big ? 128 : 64)) {
      // one launch: the slices' tails add the slots and run the E_RESID
      // epilogue (LN partials included) on the tile's last slice
      if (big && w8small(t128 * S)) {
        hipLaunchKernelGGL((gemm_kernel<128, 128, MDE_GEMM_BK, 2, 4, A_DENSE, E_RESID, 0, true>),
                           dim3((unsigned)t128, (unsigned)S), dim3(512), 0, st, p);
      } else if (big) {
        hipLaunchKernelGGL((gemm_kernel<128, 128, MDE_GEMM_BK, 2, 2, A_DENSE, E_RESID, 0, true>),
                           dim3((unsigned)t128, (unsigned)S), dim3(256), 0, st, p);
      } else if (deep64(t64 * S)) {
        hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, A_DENSE, E_RESID, 4, true>), dim3((unsigned)t64, (unsigned)S),
                           dim3(256), 0, st, p);
      } else {
        hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, A_DENSE, E_RESID, 0, true>), dim3((unsigned)t64, (unsigned)S),
                           dim3(256), 0, st, p);
      }
      return hipGetLastError();
    }
    GemmParams q = p;
    q.emode = E_PARTIAL;
    q.x32 = p.partial;
    q.ldo = p.N;
    q.bias = nullptr;
    q.ls = nullptr;
    q.lnst_out = nullptr;  // the reduce kernel writes the LN partials
    if (big && w8small(t128 * S)) {
      hipLaunchKernelGGL((gemm_kernel<128, 128, MDE_GEMM_BK, 2, 4, A_DENSE, E_PARTIAL>), dim3((unsigned)t128, (unsigned)S),
                         dim3(512), 0, st, q);
    } else if (big) {
      hipLaunchKernelGGL((gemm_kernel<128, 128, MDE_GEMM_BK, 2, 2, A_DENSE, E_PARTIAL>), dim3((unsigned)t128, (unsigned)S),
                         dim3(256), 0, st, q);
    } else {
      const unsigned tiles = (unsigned)(((p.M + 63) / 64) * ((p.N + 63) / 64));
      if (deep64((long long)tiles * S))
        hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, A_DENSE, E_PARTIAL, 4>), dim3(tiles, (unsigned)S),
                           dim3(256), 0, st, q);
      else
        hipLaunchKernelGGL((gemm_kernel<64, 64, MDE_GEMM_BK, 2, 2, A_DENSE, E_PARTIAL>), dim3(tiles, (unsigned)S),
                           dim3(256), 0, st, q);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_splitk_resid(p.partial, S, p.M, p.N, p.bias, p.ls, p.x32, p.xh, p.ldo, st, p.lnst_out);
  }
  if (p.lnst_out || p.lnst_in) {
    // folded LayerNorm: the 128^2 / 64^2 kernels of this file (partials per
    // 32-column slice from the LDS-staged epilogue, the fold after the main loop;
    // a tile that falls back to the direct epilogue writes NaN partials)
    if (!lnst_valid(p)) return hipErrorInvalidValue;
    if (panel_gemm_eligible(p)) return launch_panel_gemm(p, st);
  } else if (panel_gemm_eligible(p)) {
    return launch_panel_gemm(p, st);
  } else if (gemm256_eligible(p)) {
    return launch_gemm256(p, st);
  }
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
