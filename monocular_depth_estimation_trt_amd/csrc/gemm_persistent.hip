// Persistent, software-pipelined dense GEMM for the token-major linear layers
// of the DA-V2 encoder (qkv, proj, fc1+GELU, fc2, patch embed) and the DPT
// 1x1 / ConvTranspose projections -- C[M,N] = A[M,K] W[N,K]^T, f16 in, fp32
// accumulate, fused epilogue (tile_epilogue.h).
//
// Why persistent: at these shapes K is 384..1536 (6..24 K-steps of 64), so a
// launch-per-tile GEMM spends a large share of each tile in its prologue
// (first loads exposed) and epilogue.  Here one workgroup per CU walks a list
// of tiles; the K-steps of consecutive tiles form ONE flattened stream with a
// 3-slot global_load_lds ring, two K-steps in flight, so the next tile's
// first loads are already landing while the current tile's epilogue runs.
//
// Tile 256 x 128 x 64, 8 waves (4 x 2, 64 x 64 each, 2 waves per SIMD), LDS
// 3 x 48 KB.  LDS images are lane-linear 128-B rows with the chunk swizzle on
// the source address (conflict-free ds_read_b128 fragments).  Waits are
// counted `s_waitcnt vmcnt(N)` + raw s_barrier so DMA stays in flight across
// barriers (a __syncthreads() would drain it).  Tiles are dealt XCD-aware:
// the 32 workgroups that share one XCD's L2 take a contiguous run of tiles
// (N fastest), so the N-tiles of a row block read A through one L2.
#include <cstdlib>
#include <cstring>

#include "mde_device.h"
#include "mde_ops.h"
#include "tile_epilogue.h"

namespace mde {

namespace {

constexpr int PBK = 64, PROWB = 128;

MDE_DEV void pglds(const void* src, void* lds_wave_base) { __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0); }

template <int N>
MDE_DEV void pwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

MDE_DEV void plds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN, int WM, int WN, int NST, int EM>
__global__ void __launch_bounds__(WM * WN * 64) gemm_persistent_kernel(const GemmParams p, int ntm, int ntn) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  static_assert(TM * WM * 16 == BM && TN * WN * 16 == BN, "tile");
  constexpr int AINS = BM / 8, BINS = BN / 8;  // 8-row glds wave-instructions per operand tile
  static_assert(AINS % NW == 0 && BINS % NW == 0, "uniform glds count per wave");
  constexpr int APW = AINS / NW, BPW = BINS / NW;
  constexpr int PER = APW + BPW;  // glds per wave per K-step
  constexpr int STAGE = (BM + BN) * PROWB;
  static_assert(NST == 3, "counted waits below assume a 3-slot ring");
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int lrow = lane >> 3;
  const int lch = (lane & 7) ^ lrow;  // logical K chunk this lane fetches (swizzle involution)

  // ---- this workgroup's tiles: slot = round * G + blockIdx.x, XCD-grouped
  const int G = gridDim.x;
  const int ntiles = ntm * ntn;
  const int rounds = (ntiles + G - 1) / G;
  auto tile_at = [&](int round) -> int {  // logical tile id, or -1
    const int base = round * G;
    const int cnt = ntiles - base < G ? ntiles - base : G;
    int b = blockIdx.x;
    if (b >= cnt) return -1;
    if (cnt == G && (G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);
    return base + b;
  };
  int my_tiles = 0;
  for (int r = 0; r < rounds; ++r) my_tiles += tile_at(r) >= 0;
  const int nk = (p.K + PBK - 1) / PBK;
  const int nsteps = my_tiles * nk;
  if (nsteps == 0) return;

  const f16* Ab = reinterpret_cast<const f16*>(p.A);
  const f16* Wb = reinterpret_cast<const f16*>(p.W);

  // issue the glds of flattened step g (tile g / nk, K-step g % nk) into slot
  auto issue = [&](int g, int slot) {
    const int lt = tile_at(g / nk);
    const int kt = g - (g / nk) * nk;
    const int tm = lt / ntn, tn = lt - (lt / ntn) * ntn;
    const int k = kt * PBK + lch * 8;
    const int kk = k < p.K ? k : 0;  // K tail: W is zero there
    char* sA = smem + slot * STAGE;
    char* sB = sA + BM * PROWB;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int ins = wave + i * NW;
      int gm = tm * BM + ins * 8 + lrow;
      gm = gm < p.M ? gm : p.M - 1;
      pglds(Ab + (size_t)gm * p.lda + kk, sA + ins * 8 * PROWB);
    }
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      const int ins = wave + i * NW;
      const int gn = tn * BN + ins * 8 + lrow;
      pglds(Wb + (size_t)gn * p.ldw + kt * PBK + lch * 8, sB + ins * 8 * PROWB);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  if (nsteps > 1) {
    issue(1, 1);
    pwait_vm<PER>();
  } else {
    pwait_vm<0>();
  }
  plds_barrier();

  int slot = 0;
  for (int g = 0; g < nsteps; ++g) {
    if (g + 2 < nsteps) issue(g + 2, slot == 0 ? 2 : slot - 1);
    const char* sA = smem + slot * STAGE;
    const char* sB = sA + BM * PROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lc = 4 * s + (lane >> 4);
      f16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 16 + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const f16x8*>(sA + r * PROWB + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * TN * 16 + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const f16x8*>(sB + r * PROWB + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
    }
    // step g+1 must have landed (its slot's old contents were released at the
    // previous barrier); the epilogue's stores below are younger than it
    if (g + 2 < nsteps) pwait_vm<PER>();
    else pwait_vm<0>();
    plds_barrier();
    slot = slot == 2 ? 0 : slot + 1;

    const int kt = g - (g / nk) * nk;
    if (kt == nk - 1) {
      const int lt = tile_at(g / nk);
      const int tm = lt / ntn, tn = lt - (lt / ntn) * ntn;
      int mrow[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = tm * BM + wm * TM * 16 + i * 16 + (lane & 15);
        mrow[i] = m < p.M ? m : -1;
      }
      store_tile<EM, TM, TN>(p, acc, mrow, tn * BN + wn * TN * 16 + (lane >> 4) * 4, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

int num_cus() {
  static int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
  }();
  return n;
}

template <int BM, int BN, int WM, int WN, int EM>
hipError_t run_persistent(const GemmParams& p, hipStream_t st) {
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int tiles = ntm * ntn;
  int G = num_cus();
  if (tiles < G) G = tiles;
  hipLaunchKernelGGL((gemm_persistent_kernel<BM, BN, WM, WN, 3, EM>), dim3(G), dim3(WM * WN * 64), 0, st, p, ntm,
                     ntn);
  return hipGetLastError();
}

}  // namespace

// Opt-in (MDE_GEMM_PERSISTENT=1): on MI355X at the DA-V2 shapes it measured
// equal or slightly slower than the per-tile kernel (and both at parity with
// hipBLASLt: tools/torch_mm_ref.py), so the per-tile kernel is the default.
bool gemm_persistent_enabled() {
  static const int v = [] {
    const char* e = getenv("MDE_GEMM_PERSISTENT");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v != 0;
}

hipError_t launch_gemm_persistent(const GemmParams& p, hipStream_t st) {
  switch (p.emode) {
    case E_STORE: return run_persistent<256, 128, 4, 2, E_STORE>(p, st);
    case E_QKV: return run_persistent<256, 128, 4, 2, E_QKV>(p, st);
    case E_RESID: return run_persistent<256, 128, 4, 2, E_RESID>(p, st);
    case E_PATCH: return run_persistent<256, 128, 4, 2, E_PATCH>(p, st);
    case E_CONVT: return run_persistent<256, 128, 4, 2, E_CONVT>(p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mde
