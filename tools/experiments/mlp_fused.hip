// EXPERIMENT, not part of libmde_hip (round 4, measured slower; DESIGN.md
// section 9 "Round 4: the fused MLP").  Built only by tools/mlp_probe.hip,
// whose synthetic run checks it against a CPU restatement and stamps its
// phases.  At ViT-S B = 48 the fused launch took 3.80 ms per forward against
// 3.1 ms for the unfused fc1 + fc2: a workgroup streams all 2.36 MB of the
// block's MLP weights through L2 -> LDS at ~13 B/clk/CU (1325 clocks per 16 KB
// stage against 512 MFMA clocks), and 514 workgroups at one per CU take 3
// rounds.  The weight ring's LDS-DMA is buffer_load ... lds (see mblds below)
// with its address registers kept live (see ka[] in the kernel).
//
// Fused DINOv2 MLP for the f16-residual ViT-S blocks at large batch (gfx950):
//
//   x += ls2 * (fc2(GELU(fc1(LN2(x)))) + b2)          
//
// One launch per block in place of fc1 (which wrote the 4D-wide hidden layer
// to HBM) and fc2 (which read it back): 2 x 202 MB per block at B = 48.  A
// 512-thread workgroup owns 128 token rows; wave w owns 16 of them for the
// whole MLP, so nothing but the weights moves through LDS:
//   * the wave's 16 raw f16 residual rows live in registers as the twelve
//     K = 32 A fragments of fc1 (48 VGPRs), the LayerNorm folded in as in the
//     unfused fc1 (pack._fold_ln: W1 * gamma, the rows' mean / rstd from the
//     per-32-column partials the previous residual writer left, acc := rstd *
//     acc - rstd * mean * c1 + c2);
//   * the hidden layer runs in 24 chunks of 64 columns: the chunk's fc1
//     accumulators (4 16x16 blocks) get fold + GELU and are rounded to f16 --
//     the same rounding the unfused fc1 store made -- straight into fc2's A
//     fragments: with W1 as the MFMA A operand a lane owns row m and 4
//     consecutive hidden columns of each block, i.e. columns {4g..4g+3} and
//     {16+4g..16+4g+3} of each 32-column K slice -- fc2's weights are packed
//     with that K permutation (pack.py `fc2.wp`), so no lane exchange;
//   * fc2's 16 x 384 fp32 accumulators (96 VGPRs) stay in registers over all
//     12 chunks; the epilogue adds ls2 * (acc + b2) to the f16 residual rows
//     (one rounding) and writes the next LayerNorm's partials.
// The weights stream through an 8-slot ring of 16 KB stages (3 of W1 -- 64
// hidden rows x 128 K -- then 3 of W2 -- 128 output rows x the chunk's 64
// hidden columns -- per 64-column hidden chunk, 144 per pass) filled by
// global_load_lds with the GEMM's 128-B-row chunk swizzle, seven stages (112
// KB) in flight per CU, one barrier per stage, counted vmcnt.  Per stage a
// wave issues 16 v_mfma_f32_16x16x32_f16 (two waves per SIMD: 512 MFMA cycles
// per 16 KB): one workgroup per CU, MFMA- and L2->LDS-bound in about equal
// measure, where the two unfused GEMMs were bound by their tiles' L2 -> LDS
// traffic (every 128^2 tile re-reading its A rows) and the hidden round trip.
#include "../../monocular_depth_estimation_trt_amd/csrc/mde_device.h"
#include "../../monocular_depth_estimation_trt_amd/csrc/mde_ops.h"

namespace mde {

// Fused MLP of the f16-residual ViT-S blocks (this file): xh [M][384] +=
// ls2 * (fc2(GELU(fc1(LayerNorm(xh)))) + b2) with the LayerNorm folded into
// fc1 (w1 = fc1.wf [1536][ldw1], c1 / c2 = fc1.c1 / fc1.c2) and read from the
// partials lnst [12][lnst_rows][2], which the kernel then overwrites with the
// updated rows' partials; w2 = fc2.wp [384][ldw2] (fc2's K permuted per
// 32-column block, pack.py).
struct MlpParams {
  h16* xh = nullptr; int M = 0;
  float* lnst = nullptr; int lnst_rows = 0; float eps = 1e-6f;
  const h16* w1 = nullptr; int ldw1 = 0; const float* c1 = nullptr; const float* c2 = nullptr;
  const h16* w2 = nullptr; int ldw2 = 0; const float* b2 = nullptr; const float* ls2 = nullptr;
};
bool mlp_fused_supported(int D, int hidden);
hipError_t launch_mlp_fused(const MlpParams& p, hipStream_t st);


namespace {

constexpr int MD = 384, MHID = 1536, MHC = 64, MNCH = MHID / MHC;  // width, hidden, chunk, chunks
constexpr int MXF = MD / 32;                                      // fc1 A fragments per row group
constexpr int MSB = 128 * 128;                                    // stage bytes: 16 KB
constexpr int MNSLOT = 8;
// stages per chunk: 3 of W1 (64 hidden rows x 128 K halves, as two 64 x 64
// sub-tiles of 128-B rows) + 3 of W2 (one 128-column output group x the 64
// hidden columns each)
constexpr int MSPC = 6;
constexpr int MNST = MNCH * MSPC;     // 144 stages per pass
constexpr int MNWV = 8, MROWS = 128;  // waves per workgroup, token rows per workgroup

// LDS-DMA as buffer_load ... lds (MUBUF), not global_load_lds: hipcc counts a
// pending FLAT-encoded LDS-DMA as an out-of-order lgkm event, and then every
// ds_read wait in its shadow becomes lgkmcnt(0) -- no LDS read overlaps an
// MFMA.  The buffer form keeps the counted lgkmcnt(N) waits.
typedef __amdgpu_buffer_rsrc_t mrsrc_t;
MDE_DEV mrsrc_t mrsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
#ifndef MLP_GLDS
#define MLP_GLDS 0  // probe A/B: 1 = the FLAT global_load_lds form
#endif
MDE_DEV void mblds(const void* base, mrsrc_t r, unsigned off, void* lds) {
#if MLP_GLDS
  (void)r;
  __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(base) + off, lds, 16, 0, 0);
#else
  (void)base;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
#endif
}

// timing probe (tools/mlp_probe.hip defines MLP_PROBE 1): per-wave clock
// stamps of the kernel's phases into g_mlp_probe; compiled out otherwise
#ifndef MLP_PROBE
#define MLP_PROBE 0
#endif
#if MLP_PROBE
__device__ unsigned long long* g_mlp_probe;
#define MLP_CLK() __builtin_amdgcn_s_memtime()
#endif

MDE_DEV void mlp_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// wait until at most `after` stages (2 glds each per wave) are in flight
MDE_DEV void mlp_wait(int after) {
  switch (after) {
    case 6: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
mlp_fused_kernel(const MlpParams p) {
  static_assert(MNSLOT - 2 <= 6, "mlp_wait covers six stages in flight");
  // one LDS object: the ring, then fc1's fold columns (c1) and bias (c2),
  // staged once -- a global load inside the stage loop would make its
  // consumer wait out every ring load issued before it (vmcnt counts loads
  // and LDS-DMA together, in order).  A second __shared__ variable would give
  // the LDS accesses alias scopes, and the compiler then drains vmcnt before
  // every ring read (the ring would stop being a pipeline).
  __shared__ __attribute__((aligned(16))) char ring[MNSLOT * MSB + 2 * MHID * 4];
  float* const sc12 = reinterpret_cast<float*>(ring + MNSLOT * MSB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
#if MLP_PROBE
  unsigned long long pt[8], twait = 0;
  pt[0] = MLP_CLK();
  pt[7] = __builtin_amdgcn_s_memrealtime();
#endif
  const int row = blockIdx.x * 128 + wave * 16 + (lane & 15);
  const bool rv = row < p.M;
  const int rr = rv ? row : p.M - 1;
  const f16* xh = reinterpret_cast<const f16*>(p.xh);

  // ---- stage loader: a glds wave-instruction fills 8 rows x 128 B; a stage
  // is 16 of them, wave w issues w and w + 8 (lane-linear LDS image, the
  // swizzle on the source chunk)
  const int lrow = lane >> 3;
  const int lch = (lane & 7) ^ lrow;
  const mrsrc_t rw1 = mrsrc(p.w1), rw2 = mrsrc(p.w2);
  // the DMA's address registers are kept live until the next step: reusing
  // them at once (as ds_read destinations) raced the in-flight LDS-DMA
  // (nondeterministic outputs; the VGPR read of a VMEM address is not
  // finished at issue)
  unsigned ka[2] = {0u, 0u};
  auto issue = [&](int s) {
    const int c = s / MSPC, r = s - (s / MSPC) * MSPC;
    char* slot = ring + (s % MNSLOT) * MSB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ins = wave + 8 * i;  // sub-tile i of a W1 stage; rows 64 i + .. of a W2 stage
      ka[i] = r < 3 ? ((c * MHC + wave * 8 + lrow) * p.ldw1 + r * 128 + i * 64 + lch * 8) * 2
                    : (((r - 3) * 128 + ins * 8 + lrow) * p.ldw2 + c * MHC + lch * 8) * 2;
      mblds(r < 3 ? (const void*)p.w1 : (const void*)p.w2, r < 3 ? rw1 : rw2, ka[i], slot + ins * 1024);
    }
  };

  // ---- prologue: the wave's 16 raw residual rows as fc1 A fragments
  // (fragment f: columns 32 f + 8 g .. +7), and their LayerNorm statistics
  // from the per-32-column partials (lnst: [12][lnst_rows][2], Chan merge)
  f16x8 xf[MXF];
#pragma unroll
  for (int f = 0; f < MXF; ++f) xf[f] = *reinterpret_cast<const f16x8*>(xh + (size_t)rr * MD + 32 * f + 8 * g);
  float mean, rstd;
  {
    const float2* st2 = reinterpret_cast<const float2*>(p.lnst);
    float2 t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = st2[(size_t)(g + 4 * k) * p.lnst_rows + rr];
    float s1 = t[0].x + t[1].x + t[2].x;
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    mean = s1 * (1.f / MD);
    float m2 = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float d = t[k].x * (1.f / 32.f) - mean;
      m2 += t[k].y + 32.f * d * d;
    }
    m2 += __shfl_xor(m2, 16);
    m2 += __shfl_xor(m2, 32);
    rstd = rsqrtf(m2 * (1.f / MD) + p.eps);
  }
  const float nm = -rstd * mean;
  for (int i = tid; i < 2 * MHID / 4; i += 512) {
    const float* src = i < MHID / 4 ? p.c1 + 4 * i : p.c2 + (4 * i - MHID);
    const float4 v = *reinterpret_cast<const float4*>(src);
    *reinterpret_cast<float4*>(sc12 + 4 * i) = v;
  }
  // (every load above is consumed before the ring's first LDS-DMA is issued,
  // so the counted waits below see only the ring; the first step's barrier
  // publishes sc12)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if MLP_PROBE
  pt[1] = MLP_CLK();
#endif

#pragma unroll
  for (int s = 0; s < MNSLOT - 1; ++s) issue(s);

  f32x4 yacc[24];
#pragma unroll
  for (int b = 0; b < 24; ++b) yacc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 hacc[4];
  f16x8 hf[2];

  // fragment of stage row r (0..127), logical chunk lc (16 B)
  auto frag = [&](const char* sl, int r, int lc) -> f16x8 {
    return *reinterpret_cast<const f16x8*>(sl + r * 128 + ((lc ^ (r & 7)) << 4));
  };
  // one pipeline step: stage s landed and visible, the next refill issued
  auto step_in = [&](int s) -> const char* {
    asm volatile("" ::"v"(ka[0]), "v"(ka[1]));
#if MLP_PROBE
    const unsigned long long ta = MLP_CLK();
#endif
    mlp_wait(min(MNST - 1 - s, MNSLOT - 2));
    mlp_barrier();  // stage s visible to all; stage s - 1 fully consumed
#if MLP_PROBE
    twait += MLP_CLK() - ta;
    if (s == 0) pt[2] = MLP_CLK();
#endif
    if (s + MNSLOT - 1 < MNST) issue(s + MNSLOT - 1);
    return ring + (s % MNSLOT) * MSB;
  };

  for (int c = 0; c < MNCH; ++c) {
#pragma unroll
    for (int b = 0; b < 4; ++b) hacc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fc1: hidden columns c*64 .. +64, K = 384 in 3 stages of 128 (two 64-K sub-tiles)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const char* sl = step_in(c * MSPC + r);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          const int lc = 4 * sub + g;
#pragma unroll
          for (int b = 0; b < 4; ++b)
            hacc[b] = mfma16x16x32(frag(sl + kk * 8192, b * 16 + (lane & 15), lc), xf[4 * r + 2 * kk + sub], hacc[b]);
        }
    }
    // LayerNorm fold + bias + GELU, rounded to f16 = fc2's A fragments: fragment
    // q holds blocks 2q (elements 0..3) and 2q + 1 (4..7) of this lane's row
    // (c1, c2 of columns n = c*64 + 16 b + 4 g read by inline asm: a plain
    // LDS read here is not proven disjoint from the ring's LDS-DMA and would
    // get a compiler-inserted vmcnt(0), draining the ring once per chunk)
    f32x4 c1v[4], c2v[4];
    {
      const unsigned la = (unsigned)(uintptr_t)(sc12 + c * MHC + 4 * g);  // LDS offset (low half of the flat address)
      asm volatile(
          "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:64\n\t"
          "ds_read_b128 %2, %8 offset:128\n\tds_read_b128 %3, %8 offset:192\n\t"
          "ds_read_b128 %4, %8 offset:6144\n\tds_read_b128 %5, %8 offset:6208\n\t"
          "ds_read_b128 %6, %8 offset:6272\n\tds_read_b128 %7, %8 offset:6336\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=v"(c1v[0]), "=v"(c1v[1]), "=v"(c1v[2]), "=v"(c1v[3]), "=v"(c2v[0]), "=v"(c2v[1]), "=v"(c2v[2]),
            "=v"(c2v[3])
          : "v"(la)
          : "memory");
    }
    static_assert(MHID * 4 == 6144, "c2 offset in the asm above");
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 c1 = c1v[2 * q + h], c2 = c2v[2 * q + h];
        const f32x4 a = hacc[2 * q + h];
        const f32x2 lo = gelu_erf2(f32x2{fmaf(rstd, a[0], nm * c1[0]) + c2[0], fmaf(rstd, a[1], nm * c1[1]) + c2[1]});
        const f32x2 hi = gelu_erf2(f32x2{fmaf(rstd, a[2], nm * c1[2]) + c2[2], fmaf(rstd, a[3], nm * c1[3]) + c2[3]});
        hf[q][4 * h] = (f16)lo[0];
        hf[q][4 * h + 1] = (f16)lo[1];
        hf[q][4 * h + 2] = (f16)hi[0];
        hf[q][4 * h + 3] = (f16)hi[1];
      }
    }
    // fc2: output column group j (128 columns) x the chunk's 64 hidden columns
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const char* sl = step_in(c * MSPC + 3 + j);
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int lc = 4 * sub + g;
#pragma unroll
        for (int b = 0; b < 8; ++b)
          yacc[j * 8 + b] = mfma16x16x32(frag(sl, b * 16 + (lane & 15), lc), hf[sub], yacc[j * 8 + b]);
      }
    }
  }

#if MLP_PROBE
  pt[3] = MLP_CLK();
#endif
  // ---- epilogue: x += ls2 * (acc + b2), one rounding; the next LayerNorm's
  // partials per 32-column slice (columns {4g..} of blocks 2q, 2q + 1 across
  // the four lane groups of the row)
  f16* xo = reinterpret_cast<f16*>(p.xh) + (size_t)rr * MD;
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = (2 * q + h) * 16 + 4 * g;
      const f16x4 x4 = *reinterpret_cast<const f16x4*>(xo + n);
      const float4 ls = *reinterpret_cast<const float4*>(p.ls2 + n);
      const float4 bb = *reinterpret_cast<const float4*>(p.b2 + n);
      const f32x4 a = yacc[2 * q + h];
      const f16x4 o = {(f16)fmaf(ls.x, a[0] + bb.x, (float)x4[0]), (f16)fmaf(ls.y, a[1] + bb.y, (float)x4[1]),
                       (f16)fmaf(ls.z, a[2] + bb.z, (float)x4[2]), (f16)fmaf(ls.w, a[3] + bb.w, (float)x4[3])};
      if (rv) *reinterpret_cast<f16x4*>(xo + n) = o;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * h + e] = (float)o[e];
    }
    float s1 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s1 += v[e];
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    const float ms = s1 * (1.f / 32.f);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - ms;
      s2 += d * d;
    }
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    if (g == 0 && rv) *reinterpret_cast<float2*>(p.lnst + ((size_t)q * p.lnst_rows + rr) * 2) = make_float2(s1, s2);
  }
#if MLP_PROBE
  pt[4] = MLP_CLK();
  pt[5] = twait;
  pt[6] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    unsigned long long* o = g_mlp_probe + ((size_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = pt[k];
  }
#endif
}

}  // namespace

bool mlp_fused_supported(int D, int hidden) { return D == MD && hidden == MHID; }

hipError_t launch_mlp_fused(const MlpParams& p, hipStream_t st) {
  if (p.M <= 0) return hipSuccess;
  if (!p.xh || !p.lnst || !p.w1 || !p.w2 || !p.c1 || !p.c2 || !p.b2 || !p.ls2) return hipErrorInvalidValue;
  if (p.ldw1 < MD || (p.ldw1 & 63) || p.ldw2 < MHID || (p.ldw2 & 63) || p.lnst_rows < p.M) return hipErrorInvalidValue;
  if (((uintptr_t)p.xh & 15) || ((uintptr_t)p.w1 & 15) || ((uintptr_t)p.w2 & 15)) return hipErrorInvalidValue;
  const long long blocks = ((long long)p.M + 127) / 128;
  hipLaunchKernelGGL(mlp_fused_kernel, dim3((unsigned)blocks), dim3(512), 0, st, p);
  return hipGetLastError();
}

}  // namespace mde
