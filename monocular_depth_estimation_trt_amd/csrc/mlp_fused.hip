// Fused transformer MLP for ViT-S (D = 384, hidden = 1536) on gfx950:
//
//   x32[m, :] += ls2 * (GELU(Hn[m, :] W1^T + b1) W2^T + b2)
//
// (upstream DINOv2 Block: x + ls2(mlp(norm2(x)))), in
// ONE kernel: the 1536-wide hidden activation never leaves the CU.  The
// unfused pair spends its time outside the MFMAs -- fc1 has K = 384, six
// K-steps per 128^2 tile, so every tile pays a full load-latency prologue
// plus a 32 KB GELU epilogue, and the 134 MB hidden tensor (B = 32) is
// written and read back through HBM (profiles/r01_v11: fc1 451 TF/s, fc2
// 557 TF/s, 2.49 ms of an 8.15 ms step).
//
// One workgroup = 128 rows, 8 waves, 1 workgroup per CU.  The hidden
// dimension is walked in 12 chunks of 128:
//   phase 1 (6 stages, BK 64):  acc1[128x128] = Hn[128x384] . W1[chunk]^T
//            waves 2 (M) x 4 (N), 64 x 32 each; epilogue + b1, GELU, f16 ->
//            H[128][128] in LDS (two 64-wide halves, 128-B rows, chunk
//            swizzle c ^ (r & 7) -- the layout of a GEMM A tile)
//   phase 2 (4 stages, BK 32):  acc2[128x384] += H . W2[:, chunk]^T
//            waves 2 (M) x 4 (N), 64 x 96 each (96 fp32 accumulators/lane)
// All 120 stages run through one 3-slot LDS ring (32 KB slots: A + W1
// tiles, or a [384][32] W2 tile with 64-B rows, swizzle c ^ ((r >> 1) & 3)):
// stages t+1 and t+2 are in flight while stage t is multiplied, a counted
// vmcnt names "stage t has landed" (4 or 3 global_load_lds per wave per
// stage) and one raw barrier per stage orders the slot reuse.
// Numerics equal the unfused path: same K order, the hidden value rounded
// to f16 after the GELU exactly where fc1's epilogue stores it.
#include <cstdlib>

#include "mde_device.h"
#include "mde_ops.h"
#include "tile_epilogue.h"

namespace mde {

namespace {

constexpr int D = 384, HID = 1536, HC = 128, NCH = HID / HC;  // hidden chunk, chunks
constexpr int BM = 128, NW = 8;
constexpr int P1S = D / 64;       // phase-1 stages per chunk (BK 64)
constexpr int P2S = HC / 32;      // phase-2 stages per chunk (BK 32)
constexpr int SPC = P1S + P2S;    // stages per chunk
constexpr int NST = NCH * SPC;    // stages per workgroup
constexpr int SLOT = 32768;       // ring slot bytes
constexpr int HOFF = 3 * SLOT;    // H tile offset
constexpr int LDS_BYTES = HOFF + BM * HC * 2;  // 128 KB

MDE_DEV void glds(const void* src, void* lds_wave_base) { __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0); }

MDE_DEV void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// glds ops one wave issues for stage s (phase 1: 2 A + 2 W1; phase 2: 3 W2)
MDE_DEV int ops_of(int s) { return (s % SPC) < P1S ? 4 : 3; }

MDE_DEV void wait_vm(int n) {
  if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

MDE_DEV int sw64(int r, int lc) { return lc ^ (r & 7); }         // 128-B rows (BK 64)
MDE_DEV int sw32(int r, int lc) { return lc ^ ((r >> 1) & 3); }  // 64-B rows (BK 32)

__global__ void __launch_bounds__(NW * 64) mlp384_kernel(const MlpParams p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = blockIdx.x * BM;

  // ---- glds lane geometry ----
  // BK 64 tiles: 8 rows x 8 chunks per wave-instruction; BK 32: 16 rows x 4 chunks
  const int r64 = lane >> 3, c64 = sw64(r64, lane & 7);
  const int r32 = lane >> 2, c32 = sw32(r32, lane & 3);
  const f16* arow[2];
  const f16* w1row[2];
  const f16* w2row[3];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave + i * NW) * 8 + r64;  // tile row of wave-instruction wave + 8 i
    const int gm = m0 + r < p.M ? m0 + r : p.M - 1;
    arow[i] = reinterpret_cast<const f16*>(p.A) + (size_t)gm * D + c64 * 8;
    w1row[i] = reinterpret_cast<const f16*>(p.W1) + (size_t)r * D + c64 * 8;  // + chunk * HC * D
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = (wave + i * NW) * 16 + r32;
    w2row[i] = reinterpret_cast<const f16*>(p.W2) + (size_t)r * p.ldw2 + c32 * 8;
  }

  auto issue = [&](int s) {
    char* slot = smem + (s % 3) * SLOT;
    const int ch = s / SPC, st = s - ch * SPC;
    if (st < P1S) {
      const int k0 = st * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds(arow[i] + k0, slot + (wave + i * NW) * 8 * 128);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        glds(w1row[i] + (size_t)ch * HC * D + k0, slot + BM * 128 + (wave + i * NW) * 8 * 128);
    } else {
      const int k0 = ch * HC + (st - P1S) * 32;
#pragma unroll
      for (int i = 0; i < 3; ++i) glds(w2row[i] + k0, slot + (wave + i * NW) * 16 * 64);
    }
  };

  f32x4 acc1[4][2], acc2[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 6; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  char* const H = smem + HOFF;

  issue(0);
  issue(1);
  for (int t = 0; t < NST; ++t) {
    // issued so far: stages 0 .. t+1; stage t has landed once only stage
    // t+1's loads may still be outstanding
    wait_vm(t + 1 < NST ? ops_of(t + 1) : 0);
    bar();  // stage t visible to every wave; slot (t + 2) % 3 (stage t-1) no longer read
    if (t + 2 < NST) issue(t + 2);
    const char* slot = smem + (t % 3) * SLOT;
    const int ch = t / SPC, st = t - ch * SPC;
    if (st < P1S) {
      // ---- phase 1: acc1 += A[128 x 64] . W1c[128 x 64]^T ----
      const char* sA = slot;
      const char* sW = slot + BM * 128;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int lc = 4 * s + (lane >> 4);
        f16x8 fa[4], fb[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + (lane & 15);
          fa[i] = *reinterpret_cast<const f16x8*>(sA + r * 128 + sw64(r, lc) * 16);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = wn * 32 + j * 16 + (lane & 15);
          fb[j] = *reinterpret_cast<const f16x8*>(sW + r * 128 + sw64(r, lc) * 16);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc1[i][j] = mfma16x16x32(fb[j], fa[i], acc1[i][j]);
      }
      if (st == P1S - 1) {
        // ---- chunk epilogue: + b1, GELU, f16 -> H (the last H reader was
        // phase 2 of the previous chunk, six barriers ago) ----
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = wn * 32 + j * 16 + (lane >> 4) * 4;  // hidden column inside the chunk
          const float4 bb = *reinterpret_cast<const float4*>(p.b1 + ch * HC + n);
          const int half = n >> 6, cc = n & 63;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = wm * 64 + i * 16 + (lane & 15);
            f16x4 h;
            h[0] = (f16)gelu_erf(acc1[i][j][0] + bb.x);
            h[1] = (f16)gelu_erf(acc1[i][j][1] + bb.y);
            h[2] = (f16)gelu_erf(acc1[i][j][2] + bb.z);
            h[3] = (f16)gelu_erf(acc1[i][j][3] + bb.w);
            *reinterpret_cast<f16x4*>(H + half * (BM * 128) + r * 128 + sw64(r, cc >> 3) * 16 + (cc & 7) * 2) = h;
            acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
    } else {
      // ---- phase 2: acc2 += H[128 x 32] . W2c[384 x 32]^T ----
      const int q = st - P1S;  // 32-wide K step inside the chunk
      const char* sH = H + (q >> 1) * (BM * 128);
      const int lca = 4 * (q & 1) + (lane >> 4), lcb = lane >> 4;
      f16x8 fa[4], fb[6];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const f16x8*>(sH + r * 128 + sw64(r, lca) * 16);
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int r = wn * 96 + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const f16x8*>(slot + r * 64 + sw32(r, lcb) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc2[i][j] = mfma16x16x32(fb[j], fa[i], acc2[i][j]);
    }
  }

  // ---- epilogue: x32 += ls2 * (acc2 + b2) ----
  GemmParams g;
  g.emode = E_RESID;
  g.M = p.M;
  g.N = D;
  g.bias = p.b2;
  g.ls = p.ls2;
  g.x32 = p.x32;
  g.ldo = D;
  int mrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    mrow[i] = m < p.M ? m : -1;
  }
  store_tile<E_RESID, 4, 6>(g, acc2, mrow, wn * 96 + (lane >> 4) * 4, lane);
}

}  // namespace

bool mlp_fused_supported(int dim, int hidden, int ldw1, int ldw2) {
  return dim == D && hidden == HID && ldw1 == D && ldw2 == HID;
}

// MDE_FUSED_MLP: 0 never (default), 1 auto (enough 128-row blocks to fill
// the chip at one workgroup per CU), 2 whenever supported.  Read per call
// (tests toggle it between engines).  Off by default: measured on MI355X at
// B = 32 (profiles/r01_v12_dav2_layers_b32_fused.json) the fused launch takes
// 0.246 ms against 0.207 ms for fc1 + fc2 -- with two stages in flight per
// workgroup each 32 KB stage waits out a full L2 round trip (120 stages per
// workgroup), so the kernel is load-latency bound at 420 TF/s.
bool mlp_fused_enabled(int M) {
  const char* e = getenv("MDE_FUSED_MLP");
  const int mode = e ? atoi(e) : 0;
  if (mode == 0) return false;
  if (mode == 2) return true;
  return (M + BM - 1) / BM >= 256;
}

hipError_t launch_mlp_fused(const MlpParams& p, hipStream_t st) {
  if (p.M <= 0) return hipSuccess;
  if (!p.A || !p.W1 || !p.b1 || !p.W2 || !p.b2 || !p.ls2 || !p.x32 || p.ldw2 != HID) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mlp384_kernel, dim3((unsigned)((p.M + BM - 1) / BM)), dim3(NW * 64), 0, st, p);
  return hipGetLastError();
}

}  // namespace mde
