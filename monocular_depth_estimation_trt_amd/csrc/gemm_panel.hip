// Short-K token-major GEMMs at large batch (the ViT-S fc1 and qkv: K = 384,
// GELU / q-k-V^T head split, LayerNorm folded) for gfx950: A-stationary row panels, W chunks streamed
// through LDS, each unit's MFMAs interleaved with the previous unit's
// epilogue in the same wave.
//
//   C[M,N] = act(A[M,384] * W[N,384]^T + bias) (fp16 operands, fp32
//   accumulation), with the folded-LayerNorm consumer fix-up -- the 128^2
//   kernel's fp32 operations in the same order, so the outputs are
//   bit-identical to it (tests/test_gpu_ops.py test_panel_gemm_bit_exact).
//
// Why (tools/bench_kernels.py phase-isolation
// builds, B = 48): the 128^2 BK 32 kernel moves 192 KB of operands through
// LDS per tile (its main loop is LDS-DMA bound at ~85 GB/s per CU) and its
// three workgroups per CU run their main loops and epilogues in step:
// fc1 154 us = main loop 116 + epilogue 47.  Here
//  * a workgroup (8 waves, one per CU) owns whole 256-row panels of A; each
//    wave keeps its 32 rows x 384 K in VGPRs (24 MFMA B-operand fragments,
//    loaded once per panel straight from HBM) -- A never passes through LDS;
//  * W (<= 1.2 MB, resident in every XCD's L2) streams in 64-column chunks
//    (48 KB) through a 2-slot LDS ring: 48 KB of LDS-DMA per 256 x 64 output
//    unit instead of the 192 KB two 128^2 tiles of the same size take;
//  * every wave runs unit j's 96 MFMAs and, in the same instruction stream,
//    unit j-1's epilogue from the other accumulator set: one 16 x 16 block
//    (fold, bias, GELU, f16, 8-B store) per k-substep, so the VALU work fills
//    the MFMA shadows and both pipes stay busy (a ping-pong of two wave
//    groups -- tools/experiments/gemm_pingpong.hip -- left the MFMA pipe idle
//    half the time: one epilogue wave per SIMD was latency-bound at 2x its
//    MFMA segment);
//  * one barrier per unit: chunk j + 1's DMA is issued after it and waited
//    (vmcnt(0)) at the end of the unit, when the epilogue's stores are at
//    least four k-substeps old;
//  * the workgroups are persistent: each takes a contiguous range of the
//    (panel, chunk) units, so a panel's A is loaded once or twice per CU.
//
// Reference ops covered: a9 qkv, a12 fc1 + GELU (the a8 / a10
// LayerNorms folded).  The f16-residual form (proj: xh += ls * (.), with the
// LN partials of the rows written) is built too but taken only at switch
// "panel" = 2: at N = 384 a panel has 6 units and its load is not amortised
// (slower than the whole-row tile in the engine).
// PX_TRACE builds (tools/panel_trace.py) record s_memtime per unit segment.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"
#include "tuning.h"

namespace mde {

namespace {

constexpr int PK = 384;              // K
constexpr int PKS = PK / 32;         // MFMA k-substeps (12)
constexpr int PKSEG = PK / 64;       // 128-B LDS row segments of a W row (6)
constexpr int PBN = 64;              // output columns per unit = W rows per chunk
constexpr int PBM = 256;             // panel rows: 8 waves x 32
constexpr int PCHB = PBN * PK * 2;   // one W chunk in LDS: 48 KB
#ifndef PX_SLOTS
#define PX_SLOTS 3
#endif
constexpr int PSLOTS = PX_SLOTS;     // W ring depth: chunk j + PSLOTS - 1 issued at the top of unit j
constexpr int PLEAD = PSLOTS - 1;    // units between a chunk's issue and its use
constexpr int PNMAX = 1536;          // widest N (bias / lnc1 table)
constexpr int PTAB = PSLOTS * PCHB;  // bias / lnc1 table offset
constexpr int PLDS = PTAB + 2 * PNMAX * 4;  // 156 KB at 3 slots (108 KB at 2)
static_assert(PLDS <= 163840, "LDS");
// (round 6: the GELU on scalar registers instead of packed f32 pairs spilled
// 41 VGPRs in the LN-fold fc1 and ran slower; the packed form stays)
#ifndef PEPI_STRIDE
#define PEPI_STRIDE 1  // k-substeps between the epilogue's block pairs
#endif
#ifndef PEPI_OFF1
#define PEPI_OFF1 6    // first epilogue substep of waves 4-7 (waves 0-3: 0)
#endif

// One wave's share of a W chunk: 6 LDS-DMAs (global_load_lds_dwordx4, SGPR
// base + 32-bit VGPR offset form) -- rows lane >> 3 of its 8-row slice, row
// segment ks of 128 B from base + 128 ks + off into the LDS image at
// lds + 8192 ks.  Issued from inline asm on purpose: a compiler-visible
// LDS-DMA counts as a pending LGKM event in the compiler's wait insertion,
// which then turns every counted lgkmcnt of the MFMA stream into lgkmcnt(0)
// (each substep stalled on the fragment reads just issued for the next).
// The six segment bases are wave-uniform SGPR pairs and the lane offset one
// VGPR that is never written here (no address register reuse; the form is
// covered by tools/dma_war_probe.hip); m0 is restored.
#define PGLDS_SEG(B, MOFF) \
  "s_add_u32 m0, %[l], " MOFF "\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[off], %[" B "]\n\t"
MDE_DEV void pglds_chunk(const char* base, unsigned off, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %[keep], m0\n\t"
      PGLDS_SEG("b0", "0x0") PGLDS_SEG("b1", "0x2000") PGLDS_SEG("b2", "0x4000")
      PGLDS_SEG("b3", "0x6000") PGLDS_SEG("b4", "0x8000") PGLDS_SEG("b5", "0xa000")
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [off] "v"(off), [b0] "s"(base), [b1] "s"(base + 128), [b2] "s"(base + 256), [b3] "s"(base + 384),
        [b4] "s"(base + 512), [b5] "s"(base + 640), [l] "s"(lds)
      : "memory");
}
#undef PGLDS_SEG

// s_waitcnt vmcnt(0) as an instruction the compiler's wait insertion sees
// (an asm wait is opaque to it: loads it thinks pending at the loop head get
// a vmcnt(0) at their first use in EVERY unit -- with the W chunk DMA issued
// just before, that drained the ring each unit).  gfx9 simm16: vmcnt [3:0] +
// [15:14] = 0, expcnt [6:4] = 7, lgkmcnt [11:8] = 15
MDE_DEV void pwait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// s_waitcnt vmcnt(N) (N < 64; expcnt / lgkmcnt not waited), the same way
template <int N>
MDE_DEV void pwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

// raw workgroup barrier: LDS-DMA stays in flight (__syncthreads would drain vmcnt)
MDE_DEV void pbarrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// target of the stores of rows >= M (keeps the epilogue branch-free, so it
// stays in the MFMA stream's basic block)
__device__ __attribute__((aligned(16))) f16x4 g_psink[64];
__device__ __attribute__((aligned(16))) uint4 g_psink8[64];  // (panel32's 16-B stores)

#ifdef PX_TRACE
// timing build only (tools/panel_trace.py): per (block < 8, wave, unit <
// 96) the s_memtime after the unit's barrier and before its end-of-unit wait
// (slot 3: s_memrealtime, 100 MHz, at the unit start -- the clock check)
__device__ unsigned long long g_ptrace[8][8][96][4];
#define PTRACE(SG, K)                                                     \
  if (blockIdx.x < 8 && (SG) >= 0 && (SG) < 96) {                         \
    const unsigned long long tt = __builtin_amdgcn_s_memtime();           \
    if (lane == 0) g_ptrace[blockIdx.x][wave][(SG)][(K)] = tt;            \
    if ((K) == 0) {                                                       \
      const unsigned long long rt = __builtin_amdgcn_s_memrealtime();     \
      if (lane == 0) g_ptrace[blockIdx.x][wave][(SG)][3] = rt;            \
    }                                                                     \
  }
#else
#define PTRACE(SG, K)
#endif

template <int EM, int ACT, bool FOLD>
__global__ void __launch_bounds__(512) panel_gemm_kernel(const GemmParams p, int nch, int npan) {
  __shared__ __attribute__((aligned(16))) char smem[PLDS];
  float* tab_b = reinterpret_cast<float*>(smem + PTAB);
  float* tab_c = tab_b + PNMAX;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, hq = lane >> 4;
  // the workgroup's units (panel-major (panel, chunk) pairs): q = npan / G
  // whole panels first -- each panel's A is loaded by one workgroup, once --
  // then the leftover panels' units spread evenly over all workgroups as a
  // tail (at B = 48: 257 panels, 256 workgroups -> 24 units each plus one
  // tail unit for 24 of them).  npan < G: all units are tail (an even split).
  const int G = gridDim.x, g = blockIdx.x;
#ifndef PX_PART
// 1: whole panels per workgroup + an even tail (A read once: qkv 295 -> ~205
// MB, fc1 341 -> ~255 MB per B = 48 launch); 0 (default): every workgroup an
// even contiguous share of all units, two panels for most.  Measured in the
// graph (round 6, same box): the whole-panel form made the NEXT kernels
// slower (the 256 x 128 residual GEMMs +40 us, attention +15 us per forward)
// by more than it saved, step 5724 (0) vs 5685 (1) img/s
#define PX_PART 0
#endif
  const int q = PX_PART ? npan / G : 0;
  const int m0 = g * q * nch, nm = q * nch;
  const int tb = q * G * nch, T = nch * npan - tb;
  const int t0 = tb + (int)((long long)g * T / G);
  const int nu = nm + tb + (int)((long long)(g + 1) * T / G) - t0;
  auto gunit = [&](int j) __attribute__((always_inline)) { return j < nm ? m0 + j : t0 + (j - nm); };

  // per-column bias and folded-LN column sums, read by every epilogue
  // (E_RESID: tab_c holds the layer scale instead)
  for (int i = tid; i < p.N; i += 512) {
    tab_b[i] = p.bias ? p.bias[i] : 0.f;
    tab_c[i] = FOLD ? p.lnc1[i] : (EM == E_RESID ? p.ls[i] : 0.f);
  }

  // ---- W chunk DMA: wave w fills rows 8w .. 8w + 7 of every 128-B row
  // segment; lane -> (row lane >> 3, physical chunk lane & 7) fetches logical
  // chunk (lane & 7) ^ row (swizzle on the source: conflict-free ds_read_b128)
  const int drow = lane >> 3;
  const unsigned woff = (unsigned)((drow * p.ldw + (((lane & 7) ^ drow) * 8)) * 2);  // bytes
  static_assert(PKSEG == 6 && PBN == 64, "pglds_chunk: 6 row segments of 64 rows");
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)smem) + wave * 1024;
  auto issue = [&](int rel) __attribute__((always_inline)) {  // local unit rel -> slot rel % PSLOTS
    // (wave-uniform operands made explicitly scalar: the asm takes SGPRs)
    const int c = __builtin_amdgcn_readfirstlane(gunit(rel) % nch);
    pglds_chunk(reinterpret_cast<const char*>(p.W) + (size_t)(c * PBN + 8 * wave) * p.ldw * 2, woff,
                __builtin_amdgcn_readfirstlane(lds0 + (rel % PSLOTS) * PCHB));
  };

  // ---- A: this wave's 32 panel rows as MFMA B-operand fragments ----
  // af[ib][s]: row 16 ib + (lane & 15), k = 32 s + 8 (lane >> 4) .. +8
  f16x8 af[2][PKS];
  auto row_of = [&](int pnl, int ib) __attribute__((always_inline)) { return pnl * PBM + wave * 32 + ib * 16 + l15; };
  auto load_panel = [&](int pnl) __attribute__((always_inline)) {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int m = row_of(pnl, ib);
      const f16* src = reinterpret_cast<const f16*>(p.A) + (size_t)(m < p.M ? m : p.M - 1) * p.lda + 8 * hq;
#pragma unroll
      for (int s = 0; s < PKS; ++s) af[ib][s] = *reinterpret_cast<const f16x8*>(src + 32 * s);
    }
  };
  // folded LayerNorm: (mean, rstd) of the lane's two rows from the
  // producers' 32-column slice partials, merged as the 128^2 kernel does
  // (ln_merge_stats): the 4 lanes of a row take slices q, q + 4, ..
  auto panel_stats = [&](int pnl, float (&mean_o)[2], float (&rstd_o)[2]) __attribute__((always_inline)) {
    const float2* st2 = reinterpret_cast<const float2*>(p.lnst_in) + (unsigned)(hq * p.lnst_rows);
    const int kp = p.lnst_ns >> 2;
    const float invd = 1.f / (float)(p.lnst_ns * 32);  // as gemm.hip computes it (device division)
    float2 t[2][8];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int m = row_of(pnl, ib);
      const int mr = m < p.M ? m : p.M - 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[ib][k] = st2[(unsigned)((k < kp ? 4 * k : 0) * p.lnst_rows + mr)];
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      float var;
      ln_merge_stats(t[ib], kp, invd, mean_o[ib], var);
      rstd_o[ib] = rsqrtf(__fadd_rn(var, p.ln_eps));
    }
  };

  // ---- epilogue of one 16 x 16 block (ib, jb) of a unit: lane owns row
  // 16 ib + (lane & 15), columns 16 jb + 4 (lane >> 4) .. +3 -- fold, bias,
  // activation, one rounding to f16, an 8-B store.  Branch-free (rows >= M
  // and the dummy epilogue of a workgroup's first unit store to the sink), so
  // it stays in the basic block of its substep's MFMAs.
  struct ColB {
    float4 b, c;
  };
  auto col_read = [&](int c, int jb) __attribute__((always_inline)) {
    const int n = c * PBN + jb * 16 + hq * 4;
    ColB r;
    r.b = *reinterpret_cast<const float4*>(tab_b + n);
    r.c = (FOLD || EM == E_RESID) ? *reinterpret_cast<const float4*>(tab_c + n) : float4{0.f, 0.f, 0.f, 0.f};
    return r;
  };
  // E_RESID: the f16 residual values a unit's epilogue updates, loaded during
  // that unit (after its chunk DMA, drained by its end-of-unit wait) and
  // consumed by the epilogue in the next unit -- a load consumed inside the
  // unit that issued it would wait for the (older) chunk DMA as well
  f16x4 rres[8];
  auto res_load2 = [&](int b0, int pnl, int c) __attribute__((always_inline)) {  // blocks b0, b0 + 1
    if constexpr (EM == E_RESID) {
#pragma unroll
      for (int b = b0; b < b0 + 2; ++b) {
        const int m = row_of(pnl, b >> 2);
        const int mr = m < p.M ? m : p.M - 1;
        rres[b] = *reinterpret_cast<const f16x4*>(reinterpret_cast<const f16*>(p.xh) + (size_t)mr * p.ldo + c * PBN +
                                                  (b & 3) * 16 + hq * 4);
      }
    }
  };
  // the 4 outputs of block (ib, jb) of unit (pnl, c), one rounding to f16;
  // rows >= M and the dummy epilogue of a run's first unit go to the sink.
  // E_STORE: one 8-B store at (m, n .. n+3).  E_QKV (chunk c = head c % heads
  // of q, k or v): q (scaled) / k rows [b*heads + h][t][64] take the 8 B at
  // dh .. dh+3; V^T [b*heads + h][64][Tpad] takes 4 scalar stores at key
  // position vt_pos(t) of rows dh .. dh+3
  auto store4 = [&](int ib, int jb, int pnl, int c, float y0, float y1, float y2, float y3, bool live,
                    const float4& ls) __attribute__((always_inline)) {
    const int m = row_of(pnl, ib);
    const bool ok = live && m < p.M;
    f16x4 h = {(f16)y0, (f16)y1, (f16)y2, (f16)y3};
    if constexpr (EM == E_STORE) {
      const int n = c * PBN + jb * 16 + hq * 4;
      f16x4* dst = ok ? reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.out16) + (size_t)m * p.ldo + n) : g_psink + lane;
      *dst = h;
    } else if constexpr (EM == E_RESID) {
      // xh += ls * (acc + bias): fp32 update, one rounding (the 128^2 kernel's)
      const f16x4 x = rres[ib * 4 + jb];
      h = f16x4{(f16)((float)x[0] + ls.x * y0), (f16)((float)x[1] + ls.y * y1), (f16)((float)x[2] + ls.z * y2),
                (f16)((float)x[3] + ls.w * y3)};
      const int n = c * PBN + jb * 16 + hq * 4;
      f16x4* dst = ok ? reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.xh) + (size_t)m * p.ldo + n) : g_psink + lane;
      *dst = h;
    } else {
      const int which = c / p.heads, hh = c - which * p.heads;
      const int mm = ok ? m : 0;
      const int b = mm / p.T, t = mm - b * p.T;
      const int dh = jb * 16 + hq * 4;
      if (which < 2) {
        const float sc = which == 0 ? p.qscale : 1.f;
        h = f16x4{(f16)(y0 * sc), (f16)(y1 * sc), (f16)(y2 * sc), (f16)(y3 * sc)};
        f16* base = which == 0 ? reinterpret_cast<f16*>(p.q) : reinterpret_cast<f16*>(p.k);
        f16x4* dst = ok ? reinterpret_cast<f16x4*>(base + ((size_t)(b * p.heads + hh) * p.Tpad + t) * 64 + dh)
                        : g_psink + lane;
        *dst = h;
      } else {
        f16* row = reinterpret_cast<f16*>(p.vt) + ((size_t)(b * p.heads + hh) * 64 + dh) * p.Tpad + vt_pos(t);
        f16* sink = reinterpret_cast<f16*>(g_psink + lane);
        const size_t tp = p.Tpad;
        *(ok ? row : sink) = h[0];
        *(ok ? row + tp : sink) = h[1];
        *(ok ? row + 2 * tp : sink) = h[2];
        *(ok ? row + 3 * tp : sink) = h[3];
      }
    }
    return h;
  };
  // E_RESID with lnst_out: the folded-LN partials of the f16 values written,
  // per row and 32-column slice (sum, M2 about the slice mean): a block pair
  // (jb, jb + 1) is one slice; the 4 lanes of a row (lane >> 4) hold its 32
  // values.  Same definition as the 128^2 kernel's (tile_epilogue.h
  // ln_partials); the summation groups differ, so equal to fp32 rounding.
  auto ln_slice = [&](int ib, int pnl, int slice, const f16x4& h0, const f16x4& h1, bool live)
                      __attribute__((always_inline)) {
    float s1 = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) s1 += (float)h0[r];
#pragma unroll
    for (int r = 0; r < 4; ++r) s1 += (float)h1[r];
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    const float ms = s1 * (1.f / 32.f);
    float s2 = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = (float)h0[r] - ms;
      s2 += d * d;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = (float)h1[r] - ms;
      s2 += d * d;
    }
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    const int m = row_of(pnl, ib);
    float2* dst = (live && m < p.M && hq == 0)
                      ? reinterpret_cast<float2*>(p.lnst_out + ((size_t)slice * p.lnst_rows + m) * 2)
                      : reinterpret_cast<float2*>(g_psink + lane);
    *dst = make_float2(s1, s2);
  };
  // two blocks (2 x 4 values) in lockstep: each step of gelu_erf2 for all
  // four value pairs before the next (the same operations per value, so
  // bit-identical), four independent dependency chains for the in-order wave
  auto epi_pair = [&](int b0, int pnl, int c, const f32x4 (&accP)[2][4], const float (&pmean)[2],
                      const float (&prstd)[2], const ColB (&cb)[2], bool live) __attribute__((always_inline)) {
    f32x2 x[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = b0 + e, ib = b >> 2, jb = b & 3;
      f32x4 v = accP[ib][jb];
      if constexpr (FOLD) {
        const float rstd = prstd[ib], nm = -prstd[ib] * pmean[ib];
        v[0] = fmaf(rstd, v[0], nm * cb[e].c.x);
        v[1] = fmaf(rstd, v[1], nm * cb[e].c.y);
        v[2] = fmaf(rstd, v[2], nm * cb[e].c.z);
        v[3] = fmaf(rstd, v[3], nm * cb[e].c.w);
      }
      v[0] += cb[e].b.x; v[1] += cb[e].b.y; v[2] += cb[e].b.z; v[3] += cb[e].b.w;
      x[2 * e] = f32x2{v[0], v[1]};
      x[2 * e + 1] = f32x2{v[2], v[3]};
    }
    f32x2 y[4];
    if constexpr (ACT == ACT_GELU) {
      const f32x2 cc = {0.001014263055f, 0.001014263055f}, cb2 = {-0.106775724f, -0.106775724f},
                  ca = {-2.301121339f, -2.301121339f};
      f32x2 xc[4], x2[4], t[4], d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xc[q] = f32x2{__builtin_amdgcn_fmed3f(x[q][0], -8.f, 8.f), __builtin_amdgcn_fmed3f(x[q][1], -8.f, 8.f)};
#pragma unroll
      for (int q = 0; q < 4; ++q) x2[q] = xc[q] * xc[q];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = __builtin_elementwise_fma(cc, x2[q], cb2);
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = __builtin_elementwise_fma(t[q], x2[q], ca);
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = xc[q] * t[q];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = f32x2{1.f + __builtin_amdgcn_exp2f(t[q][0]), 1.f + __builtin_amdgcn_exp2f(t[q][1])};
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = f32x2{__builtin_amdgcn_rcpf(d[q][0]), __builtin_amdgcn_rcpf(d[q][1])};
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = x[q] * d[q];
    } else if constexpr (ACT == ACT_RELU) {
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = f32x2{x[q][0] > 0.f ? x[q][0] : 0.f, x[q][1] > 0.f ? x[q][1] : 0.f};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = x[q];
    }
    f16x4 hw[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = b0 + e, ib = b >> 2, jb = b & 3;
      hw[e] = store4(ib, jb, pnl, c, y[2 * e][0], y[2 * e][1], y[2 * e + 1][0], y[2 * e + 1][1], live, cb[e].c);
    }
    if constexpr (EM == E_RESID) {
      if (p.lnst_out) ln_slice(b0 >> 2, pnl, c * 2 + ((b0 & 3) >> 1), hw[0], hw[1], live);
    }
  };

  // ---- one unit: MFMAs of unit j into accC (chunk in slot j & 1), with the
  // epilogue of unit j - 1 (accP, its panel / chunk / LN stats) spread over
  // the first 8 k-substeps, one block each.  W fragments one substep ahead
  // (two register sets); sched_barrier per substep keeps the compiler from
  // hoisting all 48 fragment reads (192 VGPRs) and keeps each epilogue block
  // beside its substep's 8 MFMAs.
  const int cx = (hq ^ (lane & 7)) << 4;  // physical chunk of logical chunk hq in rows r (r & 7 = lane & 7)
  auto unit = [&](auto off_tag, int slot, f32x4(&accC)[2][4], const f32x4(&accP)[2][4], bool epi, int ppnl, int pc,
                  const float (&pmean)[2], const float (&prstd)[2], int cpnl, int cc) __attribute__((always_inline)) {
    constexpr int OFF = decltype(off_tag)::value;
    const char* sw = smem + slot * PCHB + l15 * 128;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) accC[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // (E_RESID: one set -- its residual values take the 16 VGPRs of the
    // second; the fragments are then read at the top of their own substep)
    constexpr int WB = EM == E_RESID ? 1 : 2;
    f16x8 wf[WB][4];
    auto rd = [&](int s, f16x8(&w)[4]) __attribute__((always_inline)) {
      const int off = (s >> 1) * 8192 + (cx ^ ((s & 1) << 6));  // logical chunk 4 (s & 1) + hq
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) w[jb] = *reinterpret_cast<const f16x8*>(sw + off + jb * 2048);
    };
    if constexpr (WB == 2) rd(0, wf[0]);
#pragma unroll
    for (int s = 0; s < PKS; ++s) {
      if constexpr (WB == 2) {
        if (s + 1 < PKS) rd(s + 1, wf[(s + 1) & 1]);
      } else {
        rd(s, wf[0]);
      }
      // the epilogue's 4 block pairs run in substeps OFF, OFF + E, .. OFF + 3E
      constexpr int E = PEPI_STRIDE;
      const bool ep = s >= OFF && ((s - OFF) % E) == 0 && (s - OFF) / E < 4;
      const int q = (s - OFF) / E;
      ColB cb[2];
      if (ep) cb[0] = col_read(pc, (2 * q) & 3), cb[1] = col_read(pc, (2 * q + 1) & 3);
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) accC[ib][jb] = mfma16x16x32(wf[s % WB][jb], af[ib][s], accC[ib][jb]);
      // blocks 2s, 2s + 1 of the previous unit in substeps 0 .. 3: its stores
      // are then at least 8 substeps old at the end-of-unit wait
      if (ep) {
        epi_pair(2 * q, ppnl, pc, accP, pmean, prstd, cb, epi);
        // (E_RESID) those two blocks' registers now take this unit's
        // residual values -- landed by the end-of-unit wait, used next unit
        res_load2(2 * q, cpnl, cc);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

#ifndef PX_PRIO
#define PX_PRIO 1
#endif
#if PX_PRIO
  // static priority for the second-dispatched half (MI355X_MICROARCH.md
  // "Two waves per SIMD" item 4): in-kernel trace, the lagging half's work
  // per unit 7026 -> 4301 ticks (the other half's 5005 -> 7026), graph fc1
  // 1.48 -> 1.45 ms per B = 48 forward
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  // ---- prologue: chunks 0 .. PLEAD - 1 in flight ----
#pragma unroll
  for (int r = 0; r < PLEAD; ++r)
    if (r < nu) issue(r);
  // ---- the unit loop, one copy per epilogue placement: the two waves of a
  // SIMD (w, w + 4) run their epilogue VALU in different k-substeps, so one's
  // VALU-heavy substeps meet the other's MFMA-only ones (the same substeps
  // for both left the SIMD alternately VALU- and MFMA-bound and one of the
  // pair idling at the unit barrier).  The branch sits outside the loop: a
  // per-unit branch between two unit bodies merged both accumulator sets at
  // every join and spilled.  Both copies run the same barrier sequence.
  auto run = [&](auto off_tag) __attribute__((always_inline)) {
    f32x4 acc0[2][4], acc1[2][4];  // the two accumulator sets: a unit's MFMAs / the previous unit's epilogue
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) acc1[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lmean[2] = {0.f, 0.f}, lrstd[2] = {1.f, 1.f};  // this panel's LN stats
    int ppnl = 0, pc = 0;                                 // panel and chunk of the unit whose epilogue runs next
    // outer loop: one run of units per A panel (af loop-invariant inside)
    auto epi_all = [&](const f32x4(&accP)[2][4]) __attribute__((always_inline)) {  // a unit's whole epilogue, standalone
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const ColB cb[2] = {col_read(pc, (2 * q) & 3), col_read(pc, (2 * q + 1) & 3)};
        epi_pair(2 * q, ppnl, pc, accP, lmean, lrstd, cb, true);
      }
    };
    int j = 0;
    while (j < nu) {
      const int gu = gunit(j), pnl = gu / nch;
      // the run: this panel's units inside the current (main or tail) range
      const int jend = min(j < nm ? nm : nu, j + (pnl + 1) * nch - gu);
      // the previous panel's last epilogue runs here, on its own (once per
      // panel switch): the stats registers then hold one panel at a time
      if (j > 0) epi_all(acc1);
      load_panel(pnl);
      if constexpr (FOLD) panel_stats(pnl, lmean, lrstd);
      pwait_vm0();  // A and every issued chunk landed (once per panel)
      const int j0 = j;
      // one unit: chunk jj visible to all waves after the barrier, and slot
      // (jj + PLEAD) % PSLOTS (unit jj - 1's) read by all, so chunk jj + PLEAD
      // goes into it.  At the end, chunk jj + 1 must have landed: it was issued
      // at the top of unit jj + 1 - PLEAD, and every unit since issued at least
      // 8 vector-memory ops after it (the epilogue's stores; E_QKV's V^T
      // chunks 32), so vmcnt(8 PLEAD) waits for it and leaves the newer chunk
      // DMAs and this unit's stores in flight (an older store waited for too
      // is long done)
      auto step = [&](int jj, f32x4(&accC)[2][4], const f32x4(&accP)[2][4]) __attribute__((always_inline)) {
        pbarrier();
        PTRACE(jj, 0)
        if (jj + PLEAD < nu) issue(jj + PLEAD);
        const int cc = gunit(jj) - pnl * nch;
        unit(off_tag, jj % PSLOTS, accC, accP, jj > j0, pnl, pc, lmean, lrstd, pnl, cc);
        ppnl = pnl;
        pc = cc;
        PTRACE(jj, 1)
        if constexpr (EM == E_RESID) pwait_vm0();  // (its residual loads: consumed next unit)
        else pwait_vm<8 * PLEAD>();
        PTRACE(jj, 2)
      };
      // two units per iteration with the accumulator roles swapped: no copy
      // of the 32 accumulator registers per unit
      for (; j + 1 < jend; j += 2) {
        step(j, acc0, acc1);
        step(j + 1, acc1, acc0);
      }
      if (j < jend) {
        step(j, acc0, acc1);
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) acc1[ib][jb] = acc0[ib][jb];
        ++j;
      }
    }
    epi_all(acc1);  // the last unit's epilogue
  };
  if (wave < 4) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, PEPI_OFF1>{});
}


// ---------------------------------------------------------------------------
// panel32_kernel (switch "panel32"): the same A-stationary panels, W ring and
// unit loop as panel_gemm_kernel, with
//  * v_mfma_f32_32x32x16_f16: a unit is 2 x 24 MFMAs per wave instead of
//    96 of 16x16x32 -- an MFMA holds the SIMD's vector issue for 8 cycles
//    whatever its size (MI355X_MICROARCH.md cycle constants), so the issue
//    slots the MFMAs take halve, and they are what the epilogue's VALU
//    competes for (in-kernel trace: the two waves of a SIMD share one issue
//    port and the unit length is their summed issue time);
//  * the folded LayerNorm's mean term as the accumulator's INITIAL value,
//    acc0 = -mean * c1 (per row x per column), so the epilogue is
//    y = rstd * acc + c2 (one fma) instead of rstd * acc - rstd * mean * c1 + c2
//    (mul, fma, add).  Not bit-identical to the 128^2 kernel (other fp32
//    association): tests/test_gpu_ops.py::test_panel32_matches_tile_kernel
//    bounds the difference by the f16 output rounding.
// Measured (round 6, B = 48, same box): per layer qkv 1.22 -> 1.12-1.17 ms,
// fc1 1.55-1.59 -> 1.53-1.57 ms per forward, but the graph step unchanged
// within its +-1 % noise over five pairs, and the in-graph clock of the last
// fc1 (tools/graph_clock.py, s_memtime / s_memrealtime) 1.91 GHz against 2.02
// for panel_gemm_kernel: fewer ticks per unit (7622 vs 7751) at a lower clock
// (the denser body draws more power -- MI355X_MICROARCH.md DVFS item 4), 3.98
// vs 3.84 us per unit.  Off by default (switch "panel32").  A two-workgroups-
// per-CU form (4 waves each, separate barrier domains) measured slower still
// (fc1 1.68 ms per forward) and was removed.
// W LDS image: 6 segments of 64 rows x 128 B, logical 16-B chunk lc of row r
// at physical chunk lc ^ ((r >> 1) & 7): the 32-row x 2-chunk operand reads
// are conflict-free in every ds_read_b128 lane group.
// Lane layout (32x32x16): W fragment = 32 output columns x 16 k (row l & 31,
// k 8 (l >> 5) .. +7); A fragment = the wave's 32 rows x 16 k (row l & 31);
// the accumulator of n-block nb holds row l & 31, columns nb * 32 + 8 g +
// 4 (l >> 5) + i in register 4 g + i.
constexpr int P3KS = PK / 16;  // 32x32x16 k-steps per unit (24)
#ifndef P3_OFF1
#define P3_OFF1 12  // first epilogue k-step of waves 4-7 (waves 0-3: 0)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
MDE_DEV f32x16 pmfma32(const f16x8& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int EM, int ACT, bool FOLD>
__global__ void __launch_bounds__(512) panel32_kernel(const GemmParams p, int nch, int npan) {
  static_assert(EM == E_STORE || EM == E_QKV, "panel32: E_STORE / E_QKV");
  __shared__ __attribute__((aligned(16))) char smem[PLDS];
  float* tab_b = reinterpret_cast<float*>(smem + PTAB);
  float* tab_c = tab_b + PNMAX;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, hh = lane >> 5;
  // units: an even contiguous share of the (panel, chunk) pairs
  const int U = nch * npan;
  const int u0 = (int)((long long)blockIdx.x * U / gridDim.x);
  const int nu = (int)((long long)(blockIdx.x + 1) * U / gridDim.x) - u0;

  for (int i = tid; i < p.N; i += 512) {
    tab_b[i] = p.bias ? p.bias[i] : 0.f;
    tab_c[i] = FOLD ? p.lnc1[i] : 0.f;
  }

  // ---- W chunk DMA: wave w fills rows 8w .. 8w + 7 of each 128-B row
  // segment; lane -> (row 8w + (lane >> 3), physical chunk lane & 7) fetches
  // logical chunk (lane & 7) ^ ((row >> 1) & 7)
  const int drow = lane >> 3;
  const unsigned woff =
      (unsigned)((drow * p.ldw + (((lane & 7) ^ (((8 * wave + drow) >> 1) & 7)) * 8)) * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)smem) + wave * 1024;
  auto issue = [&](int rel) __attribute__((always_inline)) {
    const int c = __builtin_amdgcn_readfirstlane((u0 + rel) % nch);
    pglds_chunk(reinterpret_cast<const char*>(p.W) + (size_t)(c * PBN + 8 * wave) * p.ldw * 2, woff,
                __builtin_amdgcn_readfirstlane(lds0 + (rel % PSLOTS) * PCHB));
  };

  // ---- A: the wave's 32 panel rows, k-step s = k 16 s + 8 hh .. +7
  f16x8 af[P3KS];
  auto row_of = [&](int pnl) __attribute__((always_inline)) { return pnl * PBM + wave * 32 + l31; };
  auto load_panel = [&](int pnl) __attribute__((always_inline)) {
    const int m = row_of(pnl);
    const f16* src = reinterpret_cast<const f16*>(p.A) + (size_t)(m < p.M ? m : p.M - 1) * p.lda + 8 * hh;
#pragma unroll
    for (int s = 0; s < P3KS; ++s) af[s] = *reinterpret_cast<const f16x8*>(src + 16 * s);
  };
  // folded LayerNorm statistics: computed in panel_gemm_kernel's lane layout
  // (4 lanes per row, ln_merge_stats -- bit-identical statistics), then lane
  // l takes those of its row wave * 32 + (l & 31) = 16 ib + (l & 15) from
  // lane l & 15, slot ib
  auto stats_load = [&](int pnl, float2 (&t)[2][8]) __attribute__((always_inline)) {
    const int l15 = lane & 15, hq = lane >> 4;
    const float2* st2 = reinterpret_cast<const float2*>(p.lnst_in) + (unsigned)(hq * p.lnst_rows);
    const int kp = p.lnst_ns >> 2;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int m = pnl * PBM + wave * 32 + ib * 16 + l15;
      const int mr = m < p.M ? m : p.M - 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[ib][k] = st2[(unsigned)((k < kp ? 4 * k : 0) * p.lnst_rows + mr)];
    }
  };
  auto stats_merge = [&](const float2 (&t)[2][8], float& mean_o, float& rstd_o) __attribute__((always_inline)) {
    const int kp = p.lnst_ns >> 2;
    const float invd = 1.f / (float)(p.lnst_ns * 32);
    float mn[2], rs[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      float var;
      ln_merge_stats(t[ib], kp, invd, mn[ib], var);
      rs[ib] = rsqrtf(__fadd_rn(var, p.ln_eps));
    }
    const int src = lane & 15;
    const float m0 = __shfl(mn[0], src), m1 = __shfl(mn[1], src);
    const float r0 = __shfl(rs[0], src), r1 = __shfl(rs[1], src);
    mean_o = (l31 >> 4) ? m1 : m0;
    rstd_o = (l31 >> 4) ? r1 : r0;
  };

  // ---- epilogue of group pair q (0..3) of a unit: n-block nb = q >> 1,
  // groups g0 = 2 (q & 1) and g0 + 1; the lane holds columns nb * 32 + 8 g +
  // 4 hh .. +3 of its row for g = g0, g0 + 1.  After the fp32 epilogue one
  // v_permlane32_swap per 32-bit word gives lane l < 32 the 8 columns of g0
  // and lane l + 32 those of g0 + 1: a 16-B store per lane, each row's 32
  // bytes in one instruction (8-B stores were the unit's store-issue bound,
  // MI355X_MICROARCH.md "attention epilogue store tail" / cdna_hip T21).
  // Branch-free: rows >= M and a run's first (dummy) epilogue go to the sink.
  auto epi_pair32 = [&](int q, int pnl, int c, const f32x16 (&accP)[2], float prstd, bool live)
                        __attribute__((always_inline)) {
    const int nb = q >> 1, g0 = 2 * (q & 1);
    f32x2 x[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int g = g0 + e;
      const float4 b = *reinterpret_cast<const float4*>(tab_b + c * PBN + nb * 32 + 8 * g + 4 * hh);
      const float v0 = accP[nb][4 * g], v1 = accP[nb][4 * g + 1], v2 = accP[nb][4 * g + 2], v3 = accP[nb][4 * g + 3];
      if constexpr (FOLD) {
        x[2 * e] = f32x2{fmaf(prstd, v0, b.x), fmaf(prstd, v1, b.y)};
        x[2 * e + 1] = f32x2{fmaf(prstd, v2, b.z), fmaf(prstd, v3, b.w)};
      } else {
        x[2 * e] = f32x2{v0 + b.x, v1 + b.y};
        x[2 * e + 1] = f32x2{v2 + b.z, v3 + b.w};
      }
    }
    f32x2 y[4];
    if constexpr (ACT == ACT_GELU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = gelu_erf2(x[i]);
    } else if constexpr (ACT == ACT_RELU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = f32x2{x[i][0] > 0.f ? x[i][0] : 0.f, x[i][1] > 0.f ? x[i][1] : 0.f};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = x[i];
    }
    const int m = row_of(pnl);
    const bool ok = live && m < p.M;
    typedef f16 f16x2 __attribute__((ext_vector_type(2)));
    auto pk = [](float a, float b) __attribute__((always_inline)) {
      return __builtin_bit_cast(unsigned, f16x2{(f16)a, (f16)b});
    };
    // the 8 columns of group g0 + hh, one 16-B store (A = group g0's words, B = g0 + 1's)
    auto swap_store = [&](f16* rowbase, float sc) __attribute__((always_inline)) {
      const unsigned a0 = pk(y[0][0] * sc, y[0][1] * sc), a1 = pk(y[1][0] * sc, y[1][1] * sc);
      const unsigned b0 = pk(y[2][0] * sc, y[2][1] * sc), b1 = pk(y[3][0] * sc, y[3][1] * sc);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      const uint4 v = {s0[0], s1[0], s0[1], s1[1]};
      uint4* dst = ok ? reinterpret_cast<uint4*>(rowbase + nb * 32 + 8 * (g0 + hh)) : g_psink8 + lane;
      *dst = v;
    };
    if constexpr (EM == E_STORE) {
      swap_store(reinterpret_cast<f16*>(p.out16) + (size_t)(ok ? m : 0) * p.ldo + c * PBN, 1.f);
    } else {
      const int which = c / p.heads, hd = c - which * p.heads;
      const int mm = ok ? m : 0;
      const int bi = mm / p.T, t = mm - bi * p.T;
      if (which < 2) {
        f16* base = which == 0 ? reinterpret_cast<f16*>(p.q) : reinterpret_cast<f16*>(p.k);
        swap_store(base + ((size_t)(bi * p.heads + hd) * p.Tpad + t) * 64, which == 0 ? p.qscale : 1.f);
      } else {
        f16* sink = reinterpret_cast<f16*>(g_psink8 + lane);
        const size_t tp = p.Tpad;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int n0 = nb * 32 + 8 * (g0 + e) + 4 * hh;
          f16* row = reinterpret_cast<f16*>(p.vt) + ((size_t)(bi * p.heads + hd) * 64 + n0) * p.Tpad + vt_pos(t);
          *(ok ? row : sink) = (f16)y[2 * e][0];
          *(ok ? row + tp : sink) = (f16)y[2 * e][1];
          *(ok ? row + 2 * tp : sink) = (f16)y[2 * e + 1][0];
          *(ok ? row + 3 * tp : sink) = (f16)y[2 * e + 1][1];
        }
      }
    }
  };

  // W fragment addresses: k-step s reads logical chunk 2 (s & 3) + hh of
  // segment s >> 2 in row nb * 32 + l31, physical chunk (2 (s & 3)) ^ x with
  // x = hh ^ ((l31 >> 1) & 7): four lane bases, the rest immediates
  const int xsw = hh ^ ((l31 >> 1) & 7);
  auto unit = [&](auto off_tag, int slot, f32x16(&accC)[2], const f32x16(&accP)[2], bool epi, int pnl, int pc,
                  float cmean, float prstd, int cc) __attribute__((always_inline)) {
    constexpr int OFF = decltype(off_tag)::value;
    const char* sw = smem + slot * PCHB + l31 * 128;
    // accumulator start: -mean * c1 of this unit's columns (fold), else 0
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      if constexpr (FOLD) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 c1 = *reinterpret_cast<const float4*>(tab_c + cc * PBN + nb * 32 + 8 * g + 4 * hh);
          accC[nb][4 * g] = -cmean * c1.x;
          accC[nb][4 * g + 1] = -cmean * c1.y;
          accC[nb][4 * g + 2] = -cmean * c1.z;
          accC[nb][4 * g + 3] = -cmean * c1.w;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) accC[nb][r] = 0.f;
      }
    }
    f16x8 wf[2][2];
    auto rd = [&](int s, f16x8(&w)[2]) __attribute__((always_inline)) {
      const char* b = sw + (((2 * (s & 3)) ^ xsw) << 4) + (s >> 2) * 8192;
      w[0] = *reinterpret_cast<const f16x8*>(b);
      w[1] = *reinterpret_cast<const f16x8*>(b + 4096);
    };
    rd(0, wf[0]);
#pragma unroll
    for (int s = 0; s < P3KS; ++s) {
      if (s + 1 < P3KS) rd(s + 1, wf[(s + 1) & 1]);
      // the previous unit's epilogue: group pairs q = 0..3 at k-steps OFF + 3 q
      const int rel = s - OFF;
      const bool ep = rel >= 0 && rel < 12 && (rel % 3) == 0;
      accC[0] = pmfma32(wf[s & 1][0], af[s], accC[0]);
      accC[1] = pmfma32(wf[s & 1][1], af[s], accC[1]);
      if (ep) epi_pair32(rel / 3, pnl, pc, accP, prstd, epi);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  PTRACE(95, 0)  // (trace builds: kernel entry)
#if PX_PRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
  for (int r = 0; r < PLEAD; ++r)
    if (r < nu) issue(r);
  auto run = [&](auto off_tag) __attribute__((always_inline)) {
    f32x16 acc0[2], acc1[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[0][r] = acc1[1][r] = 0.f;
    float lmean = 0.f, lrstd = 1.f;
    int pc = 0;
    auto epi_all = [&](const f32x16(&accP)[2], int pnl) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) epi_pair32(q, pnl, pc, accP, lrstd, true);
    };
    int j = 0, ppnl = 0;
    while (j < nu) {
      const int pnl = (u0 + j) / nch;
      const int jend = min(nu, (pnl + 1) * nch - u0);
      if (j > 0) epi_all(acc1, ppnl);
      PTRACE(j > 0 ? 93 : 91, 0)  // (trace: panel switch / first panel start)
      // the LN statistics' loads, then the panel's A; wait for everything
      // older than the 24 A loads (the chunk DMAs in flight, the statistics)
      // and let the first unit's k-steps wait for their own A fragments (the
      // compiler counts those loads): the panel load overlaps the unit's
      // first MFMAs instead of draining in front of them
      float2 st[2][8];
      if constexpr (FOLD) stats_load(pnl, st);
      load_panel(pnl);
      pwait_vm<P3KS>();
      if constexpr (FOLD) stats_merge(st, lmean, lrstd);
      PTRACE(j > 0 ? 94 : 92, 0)  // (trace: statistics landed)
      const int j0 = j;
      auto step = [&](int jj, f32x16(&accC)[2], const f32x16(&accP)[2]) __attribute__((always_inline)) {
        pbarrier();
        PTRACE(jj, 0)
        if (jj + PLEAD < nu) issue(jj + PLEAD);
        const int cc = (u0 + jj) - pnl * nch;
        unit(off_tag, jj % PSLOTS, accC, accP, jj > j0, pnl, pc, lmean, lrstd, cc);
        pc = cc;
        // chunk jj + 1 landed: it was issued at the top of unit jj - 1; since
        // then units jj - 1 and jj each issued >= 4 stores (one 16-B store per
        // group pair; E_QKV's V^T chunks 32 scalar ones) and, unless near the
        // end, chunk jj + 2's 6 DMAs
        static_assert(PLEAD == 2, "panel32: the counts below assume a 3-slot ring");
        PTRACE(jj, 1)
        if (jj + PLEAD < nu) pwait_vm<4 + 6 + 4>();
        else pwait_vm<4 + 4>();
        PTRACE(jj, 2)
      };
      // the run's first unit peeled off the loop: its k-steps wait for their
      // own A fragments (a loop would wait for all of them at its head)
      step(j, acc0, acc1);  // -> acc0
      ++j;
      for (; j + 1 < jend; j += 2) {
        step(j, acc1, acc0);
        step(j + 1, acc0, acc1);
      }
      if (j < jend) {
        step(j, acc1, acc0);  // -> acc1
        ++j;
      } else {
        acc1[0] = acc0[0];
        acc1[1] = acc0[1];
      }
      ppnl = pnl;
    }
    epi_all(acc1, ppnl);
    pwait_vm0();
    PTRACE(90, 0)  // (trace: kernel end, stores drained)
  };
  if (wave < 4) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, P3_OFF1>{});
}


}  // namespace

// CUs of the current device, cached per device id (persistent grids size
// themselves by it; hipGetDevice is per host thread, so each thread asks
// about the device it launches on)
int cu_count() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];  // 0 = not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev < kMaxDev) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
  if (dev < kMaxDev) cache[dev].store(v, std::memory_order_relaxed);  // racing threads store the same value
  return v;
}

#ifdef PX_TRACE
extern "C" int mde_debug_panel_trace(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptrace), sizeof(g_ptrace));
}
#endif

bool panel_gemm_eligible(const GemmParams& p) {
  if (!knob(KNOB_PANEL)) return false;
  if (p.amode != A_DENSE || p.K != PK || p.a_tok != 0 || (p.lnst_out && p.emode != E_RESID) || p.splitk > 1)
    return false;
  if (p.N % PBN || p.N > PNMAX || (p.lda & 7) || p.lda < PK || p.ldw < PK || (p.ldw & 63)) return false;
  if (p.lnst_in && (!p.lnc1 || p.lnst_ns != PK / 32 || p.lnst_rows != p.M)) return false;
  // whole CUs of work: at least 64 panels (B >= 12 ViT-S images)
  if ((p.M + PBM - 1) / PBM < 64) return false;
  if (p.emode == E_STORE)
    return p.out16 && !p.res0 && !p.res1 && !(p.ldo & 3) && !((uintptr_t)p.out16 & 7) && p.ldo >= p.N &&
           (p.act == ACT_NONE || p.act == ACT_RELU || p.act == ACT_GELU);
  // the f16-residual form (DA-V2 fp16 engines), no LN fold on its input: only
  // at "panel" = 2 -- bit-exact but slower than the whole-row 128 x 384 tile
  // in the engine (N = 384 gives 6 units per panel: the panel switch is not
  // amortised)
  if (p.emode == E_RESID)
    return knob(KNOB_PANEL) == 2 && p.xh && p.ls && !p.lnst_in && !(p.ldo & 3) && !((uintptr_t)p.xh & 7) && p.ldo >= p.N && !p.partial &&
           (!p.lnst_out || (p.lnst_ns * 32 == p.N && p.lnst_rows >= p.M));
  if (p.emode == E_QKV)
    return p.heads > 0 && p.heads * 64 * 3 == p.N && p.T > 0 && p.Tpad >= p.T && !(p.Tpad & 15) && p.q && p.k && p.vt &&
           !((uintptr_t)p.q & 7) && !((uintptr_t)p.k & 7) && p.act == ACT_NONE;
  return false;
}

hipError_t launch_panel_gemm(const GemmParams& p, hipStream_t st) {
  const int nch = p.N / PBN, npan = (p.M + PBM - 1) / PBM;
  const int U = nch * npan;
  const int G = U < cu_count() ? U : cu_count();
  const dim3 g(G), b(512);
  if (knob(KNOB_PANEL32) && (p.emode == E_STORE || p.emode == E_QKV)) {
    if (p.emode == E_QKV) {
      if (p.lnst_in) hipLaunchKernelGGL((panel32_kernel<E_QKV, ACT_NONE, true>), g, b, 0, st, p, nch, npan);
      else hipLaunchKernelGGL((panel32_kernel<E_QKV, ACT_NONE, false>), g, b, 0, st, p, nch, npan);
    } else if (p.lnst_in) {
      if (p.act == ACT_GELU) hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_GELU, true>), g, b, 0, st, p, nch, npan);
      else if (p.act == ACT_RELU) hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_RELU, true>), g, b, 0, st, p, nch, npan);
      else hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_NONE, true>), g, b, 0, st, p, nch, npan);
    } else {
      if (p.act == ACT_GELU) hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_GELU, false>), g, b, 0, st, p, nch, npan);
      else if (p.act == ACT_RELU) hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_RELU, false>), g, b, 0, st, p, nch, npan);
      else hipLaunchKernelGGL((panel32_kernel<E_STORE, ACT_NONE, false>), g, b, 0, st, p, nch, npan);
    }
    return hipGetLastError();
  }
  if (p.emode == E_RESID) {
    hipLaunchKernelGGL((panel_gemm_kernel<E_RESID, ACT_NONE, false>), g, b, 0, st, p, nch, npan);
  } else if (p.emode == E_QKV) {
    if (p.lnst_in) hipLaunchKernelGGL((panel_gemm_kernel<E_QKV, ACT_NONE, true>), g, b, 0, st, p, nch, npan);
    else hipLaunchKernelGGL((panel_gemm_kernel<E_QKV, ACT_NONE, false>), g, b, 0, st, p, nch, npan);
  } else if (p.lnst_in) {
    if (p.act == ACT_GELU) hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_GELU, true>), g, b, 0, st, p, nch, npan);
    else if (p.act == ACT_RELU) hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_RELU, true>), g, b, 0, st, p, nch, npan);
    else hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_NONE, true>), g, b, 0, st, p, nch, npan);
  } else {
    if (p.act == ACT_GELU) hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_GELU, false>), g, b, 0, st, p, nch, npan);
    else if (p.act == ACT_RELU) hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_RELU, false>), g, b, 0, st, p, nch, npan);
    else hipLaunchKernelGGL((panel_gemm_kernel<E_STORE, ACT_NONE, false>), g, b, 0, st, p, nch, npan);
  }
  return hipGetLastError();
}

}  // namespace mde
