// Short-K token-major GEMMs at large batch (ViT-S qkv and fc1: K = 384) for
// gfx950: A-stationary row panels, W chunks streamed through LDS, two
// ping-pong wave groups.
//
//   C[M,N] = A[M,384] * W[N,384]^T (fp16 operands, fp32 accumulation), with
//   the folded-LayerNorm consumer fix-up and the E_STORE (bias + GELU/ReLU) /
//   E_QKV (head-split q, k, V^T) epilogues of the 128^2 kernel -- the same
//   fp32 operations in the same order, so the outputs are bit-identical to it.
//
// Why (tools/bench_kernels.py phase-isolation
// builds, B = 48): the 128^2 BK 32 kernel moves 192 KB of operands through
// LDS per tile and runs its LDS-DMA, MFMA and epilogue phases one after the
// other -- fc1 154 us = main loop 116 (DMA alone 54, MFMA alone 51) +
// epilogue 47.  Here
//  * a workgroup (8 waves, one per CU: 156 KB of LDS) owns whole 256-row
//    panels of A; each wave keeps its 32 rows x 384 K in VGPRs (24 MFMA
//    B-operand fragments, loaded once per panel straight from HBM) -- A
//    never passes through LDS and is read from HBM exactly once;
//  * W (<= 1.2 MB, resident in every XCD's L2) streams in 64-column chunks
//    (48 KB) through a 3-slot LDS ring: per 256 x 64 output unit 48 KB of
//    LDS-DMA instead of the 192 KB two 128^2 tiles of the same size take;
//  * waves 0-3 (group 0, one per SIMD) and 4-7 (group 1) alternate: while
//    one group runs a unit's 96 MFMAs per wave, the other runs the previous
//    unit's epilogue (VALU + stores) on the same SIMDs, one barrier per
//    half-step ("segment").  Each wave issues its share of the W chunk two
//    units ahead at the start of its MFMA segment and waits for it
//    (vmcnt(0)) at the start of its next epilogue segment -- its stores of
//    the epilogue before are two segments old by then, so the drain costs
//    nothing and no counted wait has to order loads against stores;
//  * the workgroups are persistent: each takes a contiguous range of the
//    (panel, chunk) units, so a panel's A is loaded once or twice per CU.
//
// Reference ops covered: a9 qkv, a12 fc1 + GELU (with the
// a8/a10 LayerNorms folded in).
#include <cstdlib>

#include "mde_device.h"
#include "mde_ops.h"
#include "tuning.h"

namespace mde {

namespace {

constexpr int PK = 384;              // K
constexpr int PKS = PK / 32;         // MFMA k-substeps (12)
constexpr int PKSEG = PK / 64;       // 128-B LDS row segments of a W row (6)
constexpr int PBN = 64;              // output columns per unit = W rows per chunk
constexpr int PBM = 256;             // panel rows: 2 groups x 4 waves x 32
constexpr int PCHB = PBN * PK * 2;   // one W chunk in LDS: 48 KB
constexpr int PSLOTS = 3;            // W ring depth
constexpr int PNMAX = 1536;          // widest N (bias / lnc1 table)
constexpr int PTAB = PSLOTS * PCHB;                 // bias / lnc1 table offset
constexpr int PSTG = PTAB + 2 * PNMAX * 4;          // epilogue staging: 4 x (8 rows x 128 B)
constexpr int PLDS = PSTG + 4 * 1024;               // 160 KB, the whole LDS

// One group-0 wave's share of a W chunk: 12 LDS-DMAs (global_load_lds_dwordx4,
// 64-bit vaddr form) -- rows 8h + (lane >> 3) of its 16-row slice (source
// pointers s0 / s1 for h = 0 / 1), row segment ks of 128 B from src + 128 ks
// into the LDS image at lds + 1024 h + 8192 ks.  Issued from inline asm on
// purpose: a compiler-visible LDS-DMA counts as a pending LGKM event in the
// compiler's wait insertion, which then turns every counted lgkmcnt of the
// MFMA segment that follows into lgkmcnt(0) (each substep stalled on the
// fragment reads just issued for the next).  The address pairs are advanced
// after each issue (the vaddr64 form reads them at issue:
// tools/dma_war_probe.hip); m0 is restored.
#define PGLDS_SEG(H, MOFF)                                                  \
  "s_add_u32 m0, %[l], " MOFF "\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[a" H "], off\n\t" \
  "v_lshl_add_u64 %[a" H "], %[a" H "], 0, %[st]\n\t"
// base: the wave's first W row of the chunk (wave-uniform, SGPRs); off: the
// lane's byte offset (row (lane >> 3) and swizzled chunk); rows + 8 at +row8
// bytes.  The 64-bit lane addresses are formed inside the block, so no
// address pair stays live (or spilled) across the unit loop.
MDE_DEV void pglds_chunk(const void* base, unsigned off, unsigned long long row8, unsigned lds) {
  unsigned keep;
  unsigned long long a0, a1;
  asm volatile(
      "s_mov_b32 %[keep], m0\n\t"
      "v_lshl_add_u64 %[a0], %[off], 0, %[b]\n\t"
      "v_lshl_add_u64 %[a1], %[off], 0, %[b8]\n\t"
      PGLDS_SEG("0", "0x0") PGLDS_SEG("1", "0x400")
      PGLDS_SEG("0", "0x2000") PGLDS_SEG("1", "0x2400")
      PGLDS_SEG("0", "0x4000") PGLDS_SEG("1", "0x4400")
      PGLDS_SEG("0", "0x6000") PGLDS_SEG("1", "0x6400")
      PGLDS_SEG("0", "0x8000") PGLDS_SEG("1", "0x8400")
      PGLDS_SEG("0", "0xa000") PGLDS_SEG("1", "0xa400")
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep), [a0] "=&v"(a0), [a1] "=&v"(a1)
      : [off] "v"((unsigned long long)off), [b] "s"((unsigned long long)base), [b8] "s"((unsigned long long)base + row8),
        [l] "s"(lds), [st] "s"(128ull)
      : "memory");
}
#undef PGLDS_SEG

// s_waitcnt vmcnt(0) as an instruction the compiler's wait insertion sees
// (an asm wait is opaque to it: loads it thinks pending at the loop head get
// a vmcnt(0) at their first use in EVERY segment -- with the W chunk DMA
// issued just before, that drained the ring each MFMA segment).  gfx9
// simm16: vmcnt [3:0] + [15:14] = 0, expcnt [6:4] = 7, lgkmcnt [11:8] = 15
MDE_DEV void pwait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// vmcnt(12): all but this wave's last 12 vector-memory ops (one W chunk's DMAs)
MDE_DEV void pwait_vm12() { __builtin_amdgcn_s_waitcnt(0x0F7C); }

// raw workgroup barrier: LDS-DMA stays in flight (__syncthreads would drain vmcnt)
MDE_DEV void pbarrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#ifdef PX_TRACE
// timing build only (tools/panel_trace.py): per (block < 8, wave, segment <
// 96) the s_memtime at segment start (after its barrier) and at the end of
// the segment's work (before the next barrier)
__device__ unsigned long long g_ptrace[8][8][96][2];
#define PTRACE(SG, K)                                                              \
  if (blockIdx.x < 8 && (SG) >= 0 && (SG) < 96) {                                             \
    const unsigned long long tt = __builtin_amdgcn_s_memtime();                    \
    if (lane == 0) g_ptrace[blockIdx.x][wave][(SG)][(K)] = tt;                       \
  }
#else
#define PTRACE(SG, K)
#endif

template <int EM>
__global__ void __launch_bounds__(512) panel_gemm_kernel(const GemmParams p, int nch, int npan, float invd) {
  __shared__ __attribute__((aligned(16))) char smem[PLDS];
  float* tab_b = reinterpret_cast<float*>(smem + PTAB);
  float* tab_c = tab_b + PNMAX;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3;
  const int l15 = lane & 15, hq = lane >> 4;
  const int U = nch * npan;
  const int u0 = (int)((long long)blockIdx.x * U / gridDim.x);
  const int nu = (int)((long long)(blockIdx.x + 1) * U / gridDim.x) - u0;
  const bool fold = p.lnst_in != nullptr;

  // per-column bias and folded-LN column sums, read by every epilogue
  for (int i = tid; i < p.N; i += 512) {
    tab_b[i] = p.bias ? p.bias[i] : 0.f;
    tab_c[i] = fold ? p.lnc1[i] : 0.f;
  }

  // ---- W chunk DMA, group 0 only: wave wq fills rows 16 wq .. 16 wq + 15 of
  // every 128-B row segment; lane -> (row lane >> 3 (+8), physical chunk
  // lane & 7) fetches logical chunk (lane & 7) ^ row (swizzle on the source:
  // conflict-free ds_read_b128).  Group 1 never issues vector-memory loads in
  // the loop, so group 0's counted wait names "chunk j + 1 has landed".
  const int drow = lane >> 3;
  // (a 32-bit lane byte offset: one VGPR kept across the loop)
  const unsigned woff = (unsigned)((drow * p.ldw + (((lane & 7) ^ drow) * 8)) * 2);
  static_assert(PKSEG == 6 && PBN == 64, "pglds_chunk: 6 row segments of 64 rows");
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)smem) + wq * 2048;
  auto issue = [&](int rel) __attribute__((always_inline)) {  // unit u0 + rel -> slot rel % 3
    const int c = (u0 + rel) % nch;
    const f16* base = reinterpret_cast<const f16*>(p.W) + (size_t)(c * PBN + 16 * wq) * p.ldw;
    pglds_chunk(base, woff, (unsigned long long)p.ldw * 16, lds0 + (rel % PSLOTS) * PCHB);
  };

  // ---- A: this wave's 32 panel rows as MFMA B-operand fragments ----
  // af[ib][s]: row 16 ib + (lane & 15), k = 32 s + 8 (lane >> 4) .. +8
  f16x8 af[2][PKS];
  float lmean[2] = {0.f, 0.f}, lrstd[2] = {1.f, 1.f};  // LN stats of the rows whose epilogues run now
  auto row_of = [&](int pnl, int ib) __attribute__((always_inline)) { return pnl * PBM + grp * 128 + wq * 32 + ib * 16 + l15; };
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
  // producers' 32-column slice partials -- the 128^2 kernel's merge
  // (gemm.hip ln_partial_loads): the 4 lanes of a row take slices q, q+4, ..
  auto panel_stats = [&](int pnl, float (&mean_o)[2], float (&rstd_o)[2]) {
    // slice sl = hq + 4 k of row mr at st2[sl * rows + mr]: the lane part
    // (hq * rows) in the base, the k part scalar (no 64-bit offsets per slice
    // kept live across the unit loop)
    const float2* st2 = reinterpret_cast<const float2*>(p.lnst_in) + (unsigned)(hq * p.lnst_rows);
    const int kp = p.lnst_ns >> 2;
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
      ln_merge_stats(t[ib], kp, invd, mean_o[ib], var);  // the 128^2 kernel's merge, bit for bit
      rstd_o[ib] = rsqrtf(__fadd_rn(var, p.ln_eps));
    }
  };

  // ---- one unit's MFMAs: acc[ib][jb] over the chunk in slot rel % 3.
  // VT: operands swapped (the V third of E_QKV) -- the lane then owns four
  // consecutive rows of one column, i.e. four consecutive tokens of one V^T row
  f32x4 acc[2][4];
  const int cx = (hq ^ (lane & 7)) << 4;  // physical chunk of logical chunk hq in rows r (r & 7 = lane & 7)
  auto mma = [&](int rel, auto vt_tag) __attribute__((always_inline)) {
    constexpr bool VT = decltype(vt_tag)::value;
    const char* sw = smem + (rel % PSLOTS) * PCHB + l15 * 128;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) acc[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W fragments one substep ahead (two register sets): the reads of
    // substep s + 1 issue before the MFMAs of s; sched_barrier keeps the
    // compiler from hoisting all 48 reads (192 VGPRs) to the top
    f16x8 wf[2][4];
    auto rd = [&](int s, f16x8(&w)[4]) {
      const int off = (s >> 1) * 8192 + (cx ^ ((s & 1) << 6));  // logical chunk 4 (s & 1) + hq
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) w[jb] = *reinterpret_cast<const f16x8*>(sw + off + jb * 2048);
    };
    rd(0, wf[0]);
#pragma unroll
    for (int s = 0; s < PKS; ++s) {
      if (s + 1 < PKS) rd(s + 1, wf[(s + 1) & 1]);
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
          acc[ib][jb] = VT ? mfma16x16x32(af[ib][s], wf[s & 1][jb], acc[ib][jb])
                           : mfma16x16x32(wf[s & 1][jb], af[ib][s], acc[ib][jb]);
      // the next substep's 4 reads first, then this substep's 8 MFMAs (left
      // to itself the scheduler sinks the reads behind 6 of the MFMAs and the
      // next substep waits on them)
      if (s + 1 < PKS) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- epilogues (the 128^2 kernel's fp32 operations, same order) ----
  // Row-major outputs leave through LDS in whole 128-B lines: the lane's
  // f16x4 of row 16 ib + (lane & 15), columns 16 jb + 4 hq .. +3, are parked
  // 8 rows at a time in this wave's 1 KB slice (rows 8 h .. 8 h + 7 written by
  // the lanes that own them), read back as one 16-B chunk per lane (row
  // lane >> 3, columns 8 (lane & 7) ..) and stored by whole rows -- the direct
  // 8-B stores touch 16 partial lines per instruction and ran the epilogue
  // alone at a third of the staged rate.  Only one group is in its epilogue
  // segment at a time, so the slices are per wave-in-group.
  char* stg = smem + PSTG + wq * 1024;
  auto park_row8 = [&](int h, const f16x4 (&hv)[4]) __attribute__((always_inline)) {
    if ((l15 >> 3) == h) {
      const int r = l15 & 7;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int u = 4 * jb + hq;  // 8-B column quad
        *reinterpret_cast<f16x4*>(stg + r * 128 + ((((u >> 1) ^ r) << 4) | ((u & 1) << 3))) = hv[jb];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int rr = lane >> 3, cc = lane & 7;
    return *reinterpret_cast<const f16x8*>(stg + rr * 128 + ((cc ^ rr) << 4));
  };
  auto fold_bias = [&](int ib, int n, f32x4 v) __attribute__((always_inline)) {
    const float4 bn = *reinterpret_cast<const float4*>(tab_b + n);
    if (fold) {
      const float4 c1 = *reinterpret_cast<const float4*>(tab_c + n);
      const float nm = -lrstd[ib] * lmean[ib];
      v[0] = fmaf(lrstd[ib], v[0], nm * c1.x);
      v[1] = fmaf(lrstd[ib], v[1], nm * c1.y);
      v[2] = fmaf(lrstd[ib], v[2], nm * c1.z);
      v[3] = fmaf(lrstd[ib], v[3], nm * c1.w);
    }
    v[0] += bn.x; v[1] += bn.y; v[2] += bn.z; v[3] += bn.w;
    return v;
  };
  auto act_store = [&](int rel, auto act_tag) __attribute__((always_inline)) {  // E_STORE
    constexpr int ACT = decltype(act_tag)::value;
    const int u = u0 + rel, pnl = u / nch, c = u - pnl * nch;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      f16x4 hv[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        f32x4 v = fold_bias(ib, c * PBN + jb * 16 + hq * 4, acc[ib][jb]);
        if constexpr (ACT == ACT_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
        } else if constexpr (ACT == ACT_GELU) {
          const f32x2 lo = gelu_erf2(f32x2{v[0], v[1]}), hi = gelu_erf2(f32x2{v[2], v[3]});
          v = f32x4{lo[0], lo[1], hi[0], hi[1]};
        }
        hv[jb] = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f16x8 row8 = park_row8(h, hv);
        const int m = row_of(pnl, ib) - l15 + 8 * h + (lane >> 3);
        if (m < p.M)
          *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.out16) + (size_t)m * p.ldo + c * PBN + 8 * (lane & 7)) = row8;
      }
      __builtin_amdgcn_sched_barrier(0);  // one row block's temporaries at a time
    }
  };
  auto qk_store = [&](int rel) __attribute__((always_inline)) {  // E_QKV q / k third: token rows of one head
    const int u = u0 + rel, pnl = u / nch, c = u - pnl * nch;
    const int which = c / p.heads, hh = c - which * p.heads;
    const float sc = which == 0 ? p.qscale : 1.f;
    f16* dst0 = which == 0 ? reinterpret_cast<f16*>(p.q) : reinterpret_cast<f16*>(p.k);
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      f16x4 hv[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const f32x4 v = fold_bias(ib, c * PBN + jb * 16 + hq * 4, acc[ib][jb]);
        hv[jb] = f16x4{(f16)(v[0] * sc), (f16)(v[1] * sc), (f16)(v[2] * sc), (f16)(v[3] * sc)};
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f16x8 row8 = park_row8(h, hv);
        const int m = row_of(pnl, ib) - l15 + 8 * h + (lane >> 3);
        const int b = m / p.T, t = m - b * p.T;
        if (m < p.M)
          *reinterpret_cast<f16x8*>(dst0 + ((size_t)(b * p.heads + hh) * p.Tpad + t) * 64 + 8 * (lane & 7)) = row8;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto v_store = [&](int rel) __attribute__((always_inline)) {  // E_QKV V third (swapped MFMA): lane owns (tokens m .. m+3, dh)
    const int u = u0 + rel, pnl = u / nch, c = u - pnl * nch;
    const int hh = c - 2 * p.heads;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      // rows 16 ib + 4 hq + r of the wave: their LN stats live in lanes 4 hq + r
      float mean4[4], rstd4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mean4[r] = __shfl(lmean[ib], 4 * hq + r, 64);
        rstd4[r] = __shfl(lrstd[ib], 4 * hq + r, 64);
      }
      const int m0 = pnl * PBM + grp * 128 + wq * 32 + ib * 16 + hq * 4;
      const int b0 = m0 / p.T, t0 = m0 - b0 * p.T;
      const bool quad = (t0 & 3) == 0 && t0 + 3 < p.T && m0 + 3 < p.M;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int dh = jb * 16 + l15;
        const int n = c * PBN + dh;
        const float bn = tab_b[n], c1 = tab_c[n];
        f32x4 v = acc[ib][jb];
        if (fold) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaf(rstd4[r], v[r], (-rstd4[r] * mean4[r]) * c1);
        }
        f16x4 h;
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)(v[r] + bn);
        f16* row = reinterpret_cast<f16*>(p.vt) + ((size_t)(b0 * p.heads + hh) * 64 + dh) * p.Tpad;
        if (quad) {
          *reinterpret_cast<f16x4*>(row + vt_pos(t0)) = h;
        } else if (!(t0 & 1) && !(p.T & 1) && m0 + 3 < p.M) {
          // t0 = 2 mod 4 (every other image when T = 2 mod 4): two token
          // pairs, each contiguous under vt_pos; T even, so an image
          // boundary falls between the pairs, never inside one
          const size_t img = (size_t)p.heads * 64 * p.Tpad;
          const int t2 = t0 + 2;
          typedef f16 f16x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<f16x2*>(row + vt_pos(t0)) = f16x2{h[0], h[1]};
          f16* r2 = t2 < p.T ? row + vt_pos(t2) : row + img + vt_pos(t2 - p.T);
          *reinterpret_cast<f16x2*>(r2) = f16x2{h[2], h[3]};
        } else {
          const size_t img = (size_t)p.heads * 64 * p.Tpad;  // one image's V^T
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = t0 + r;
            if (m0 + r < p.M) {
              if (t < p.T) row[vt_pos(t)] = h[r];
              else row[img + vt_pos(t - p.T)] = h[r];
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto is_vt = [&](int rel) __attribute__((always_inline)) {
    if constexpr (EM == E_QKV) return ((u0 + rel) % nch) >= 2 * p.heads;
    return false;
  };
  auto epilogue = [&](int rel) __attribute__((always_inline)) {
    if constexpr (EM == E_QKV) {
      if (is_vt(rel)) v_store(rel);
      else qk_store(rel);
    } else {
      if (p.act == ACT_GELU) act_store(rel, std::integral_constant<int, ACT_GELU>{});
      else if (p.act == ACT_RELU) act_store(rel, std::integral_constant<int, ACT_RELU>{});
      else act_store(rel, std::integral_constant<int, ACT_NONE>{});
    }
  };

  auto mma_unit = [&](int j) __attribute__((always_inline)) {
#ifndef PX_NOPRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#ifdef PX_NOMMA
    if (p.M < 0)
#endif
    if (is_vt(j)) mma(j, std::true_type{});
    else mma(j, std::false_type{});
#ifndef PX_NOPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };
  auto epi_unit = [&](int j) __attribute__((always_inline)) {
#ifdef PX_EPIPRIO
    __builtin_amdgcn_s_setprio(2);
#endif
#ifndef PX_NOEPI
    epilogue(j);
#else
    if (p.M < 0) epilogue(j);
#endif
#ifdef PX_EPIPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // ---- prologue: chunks 0 and 1 in flight ----
  if (grp == 0) {
    issue(0);
    if (nu > 1) issue(1);
  }
  pwait_vm0();
  pbarrier();  // chunks 0 / 1 and the column table visible to every wave

  // ---- segments 0 .. 2 nu, one barrier each; unit j: group 0 runs its MFMAs
  // in segment 2j and its epilogue in 2j + 1, group 1 one segment later.
  // Outer loop: one run of units per A panel (af loop-invariant inside).
  int j = 0;
  while (j < nu) {
    const int pnl = (u0 + j) / nch;
    const int jend = min(nu, (pnl + 1) * nch - u0);
    load_panel(pnl);
    float nmean[2] = {0.f, 0.f}, nrstd[2] = {1.f, 1.f};
    if (fold) panel_stats(pnl, nmean, nrstd);
    pwait_vm0();  // A landed (once per panel)
    const int j0 = j;
    if (grp == 0 || j0 == 0) {
      lmean[0] = nmean[0], lmean[1] = nmean[1];
      lrstd[0] = nrstd[0], lrstd[1] = nrstd[1];
    }
    for (; j < jend; ++j) {
      PTRACE(2 * j - 1, 1)
      pbarrier();  // segment 2j
      PTRACE(2 * j, 0)
      if (grp == 0) {
        // slot (j + 2) % 3 held unit j - 1, whose last reader (group 1's
        // MFMA segment 2j - 1) ended at this barrier
        if (j + 2 < nu) issue(j + 2);
        mma_unit(j);
      } else if (j > 0) {
        epi_unit(j - 1);
        if (j == j0) {  // the previous panel's last epilogue is done: this panel's stats
          lmean[0] = nmean[0], lmean[1] = nmean[1];
          lrstd[0] = nrstd[0], lrstd[1] = nrstd[1];
        }
      }
      PTRACE(2 * j, 1)
      pbarrier();  // segment 2j + 1
      PTRACE(2 * j + 1, 0)
      if (grp == 0) {
        // chunk j + 1 (issued in segment 2j - 2, read from segment 2j + 2 on)
        // has landed: everything but chunk j + 2's 12 DMAs, which are this
        // wave's youngest vector-memory ops (the stores of epilogue j - 1
        // before them are two segments old)
#ifndef PX_NOWAIT
        if (j + 2 < nu) pwait_vm12();
        else pwait_vm0();
#endif
        epi_unit(j);
      } else {
        mma_unit(j);
      }
    }
  }
  PTRACE(2 * nu - 1, 1)
  pbarrier();  // segment 2 nu
  PTRACE(2 * nu, 0)
  if (grp == 1) epi_unit(nu - 1);
  PTRACE(2 * nu, 1)
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

}  // namespace

#ifdef PX_TRACE
extern "C" int mde_debug_panel_trace(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptrace), sizeof(g_ptrace));
}
#endif

bool panel_gemm_eligible(const GemmParams& p) {
  if (!knob(KNOB_PANEL)) return false;
  if (p.amode != A_DENSE || p.K != PK || p.a_tok != 0 || p.lnst_out || p.splitk > 1) return false;
  if (p.N % PBN || p.N > PNMAX || (p.lda & 7) || p.lda < PK || p.ldw < PK || (p.ldw & 63)) return false;
  if (p.lnst_in && (!p.lnc1 || p.lnst_ns != PK / 32 || p.lnst_rows != p.M)) return false;
  // whole CUs of work: at least 64 panels (B >= 12 ViT-S images)
  if ((p.M + PBM - 1) / PBM < 64) return false;
  if (p.emode == E_STORE) {
    return p.out16 && !p.res0 && !p.res1 && !(p.ldo & 7) && !((uintptr_t)p.out16 & 15) && p.ldo >= p.N &&
           (p.act == ACT_NONE || p.act == ACT_RELU || p.act == ACT_GELU);
  }
  if (p.emode == E_QKV) {
    return p.heads > 0 && p.heads * 64 * 3 == p.N && p.T > 0 && !(p.Tpad & 3) && p.Tpad >= p.T && p.q && p.k &&
           p.vt && !((uintptr_t)p.q & 15) && !((uintptr_t)p.k & 15) && !((uintptr_t)p.vt & 7);
  }
  return false;
}

hipError_t launch_panel_gemm(const GemmParams& p, hipStream_t st) {
  const int nch = p.N / PBN, npan = (p.M + PBM - 1) / PBM;
  const int U = nch * npan;
  const int G = U < cu_count() ? U : cu_count();
  // the folded LN's 1 / D, rounded as the 128^2 kernel's device division
  const float invd = p.lnst_ns > 0 ? 1.f / (float)(p.lnst_ns * 32) : 0.f;
  if (p.emode == E_QKV)
    hipLaunchKernelGGL(panel_gemm_kernel<E_QKV>, dim3(G), dim3(512), 0, st, p, nch, npan, invd);
  else
    hipLaunchKernelGGL(panel_gemm_kernel<E_STORE>, dim3(G), dim3(512), 0, st, p, nch, npan, invd);
  return hipGetLastError();
}

}  // namespace mde
