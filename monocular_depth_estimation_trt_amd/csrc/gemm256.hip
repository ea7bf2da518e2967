// Large dense GEMM for gfx950: 256 x 256 x 64 tiles, 8 waves, one workgroup
// per CU, a phase-interleaved software pipeline.
//
//   C[M,N] = A[M,K] * W[N,K]^T   (fp16 operands, fp32 accumulation, fused
//   epilogue of tile_epilogue.h: bias / GELU / ReLU / LayerScale residual /
//   q-k-v head split / pos-embed / ConvT pixel shuffle)
//
// Used for the token-major linear layers once there are enough 256^2 tiles
// to fill the chip (Depth Pro's patch encoder: 140 x 577 tokens x D 1024;
// DA-V2 ViT-L).  The 128^2 kernel of gemm.hip stalls there on its per-K-step
// vmcnt(0) + barrier; hipBLASLt reached 1.1-1.2 PF/s on those shapes where
// it reached 0.7-0.9 (tools/gemm_compare.py).
//
// Structure (cdna_hip_programming.md section 5, "256^2 8-phase template" and
// "Pipelining across barriers", re-derived for this kernel):
//  * 8 waves = 2 (M) x 4 (N); a wave owns 128 x 64 of C = 8 x 4 MFMA blocks.
//  * LDS: two buffers (even / odd K-tiles) of A[256][64] + W[256][64] f16,
//    128-B rows, chunk swizzle c ^ (row & 7) applied on the SOURCE address
//    of global_load_lds (lane-linear LDS image) and on the ds_read_b128.
//  * A K-tile is consumed in 4 phases; phase q multiplies A rows
//    {128 wr + 32 q .. +32} (2 blocks) by the wave's 4 W blocks (16 MFMAs).
//    W fragments are read once per tile, A fragments one phase ahead, each
//    right behind the MFMAs that free their registers.
//  * As soon as a region of the current buffer has been read for the last
//    time, the loads of K-tile t+2 into it are issued (W + A quarter 0 in
//    phase 0, A quarter q in phase q): the DMA stays in flight across the
//    phase barriers (raw s_barrier, counted s_waitcnt vmcnt(7) once per tile
//    -- never vmcnt(0) in steady state).
//  * One barrier per phase; MFMA clusters at s_setprio(1).
#include <cstdlib>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"
#include "tuning.h"
#include "tile_epilogue.h"

#ifndef MDE_EPI_LDS_256
#define MDE_EPI_LDS_256 1  // epilogue staged through LDS in two M halves (whole-line stores)
#endif

namespace mde {

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NW = 8;
constexpr int ROWB = BK * 2;         // 128 bytes per LDS row
constexpr int TILE_B = 256 * ROWB;   // one operand tile, 32 KB
constexpr int BUF_B = 2 * TILE_B;    // A + W

MDE_DEV void g256_glds(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}

MDE_DEV void g256_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
MDE_DEV void g256_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

MDE_DEV int g256_off(int row, int lc) { return row * ROWB + ((lc ^ (row & 7)) << 4); }

template <int EM>
__global__ void __launch_bounds__(NW * 64) gemm256_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_B];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // XCD-aware order: each XCD a contiguous run, N fastest
  int tm, tn;
  tile_of(bid, (p.M + BM - 1) / BM, ntn, tile_group_m(p.N, p.K, BM), tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // glds geometry: a wave-instruction fills 8 rows x 128 B; lane -> (row lrow,
  // physical chunk pc) fetches logical chunk pc ^ lrow (rows are 8-aligned)
  const int lrow = lane >> 3, lch = (lane & 7) ^ lrow;
  const f16* Ab = reinterpret_cast<const f16*>(p.A);
  const f16* Wb = reinterpret_cast<const f16*>(p.W);
  // per-lane element offsets (32-bit: M * lda and N * ldw stay below 2^31 here)
  // from wave-uniform bases, so the pointers do not cost 8 VGPR pairs
  int asrc[4];
  int aoff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 128 * (wave >> 2) + 32 * q + 8 * (wave & 3);  // first LDS row of this wave's slice
    const int gm = min(m0 + r + lrow, p.M - 1);                 // clamped: rows >= M are masked on store
    asrc[q] = gm * p.lda;
    aoff[q] = r * ROWB;
  }
  int wsrc[4];
  int woff[4];
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int r = 64 * r4 + 8 * wave;
    const int gn = min(n0 + r + lrow, p.N - 1);
    wsrc[r4] = gn * p.ldw + lch * 8;
    woff[r4] = TILE_B + r * ROWB;
  }
  const int nk = (p.K + BK - 1) / BK;
  auto issue_w = [&](int kt, int buf) {
    const int k0 = kt * BK;  // W is zero-padded to ldw >= K rounded up to 64
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) g256_glds(Wb + (wsrc[r4] + k0), smem + buf * BUF_B + woff[r4]);
  };
  auto issue_a = [&](int q, int kt, int buf) {
    const int k = kt * BK + lch * 8;
    const int kk = k < p.K ? k : 0;  // K tail: W is zero there, any finite A chunk of the row will do
    g256_glds(Ab + (asrc[q] + kk), smem + buf * BUF_B + aoff[q]);
  };

  // fragments: W blocks nb (rows 64 wc + 16 nb + l15), A blocks 2q+i (rows
  // 128 wr + 16(2q+i) + l15).  Single register sets: each phase issues its
  // MFMAs first and only then the ds_reads of the next phase into the same
  // registers (the reads' latency runs under the MFMA pipeline drain; the
  // hazard recognizer orders the WAR on the sources) -- 48 fragment VGPRs
  // instead of 96, no spills beside the 128 accumulators.
  const int l15 = lane & 15, hq = lane >> 4;
  f16x8 wf[4][2];  // [n block][k substep]
  f16x8 af[2][2];  // [block in quarter][k substep]
  auto read_w = [&](int buf) {
    const char* base = smem + buf * BUF_B + TILE_B;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = 64 * wc + 16 * nb + l15;
        wf[nb][s] = *reinterpret_cast<const f16x8*>(base + g256_off(row, 4 * s + hq));
      }
  };
  auto read_a = [&](int buf, int q) {
    const char* base = smem + buf * BUF_B;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = 128 * wr + 16 * (2 * q + i) + l15;
        af[i][s] = *reinterpret_cast<const f16x8*>(base + g256_off(row, 4 * s + hq));
      }
  };

  f32x4 acc[2][4][4];  // [M half][block in half][n block]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma_phase = [&](auto q_tag) {
    constexpr int q = decltype(q_tag)::value;
    constexpr int h = q / 2;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int bi = (2 * q + i) % 4;
          acc[h][bi][nb] = mfma16x16x32(wf[nb][s], af[i][s], acc[h][bi][nb]);
        }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);  // the next phase's ds_reads stay behind these MFMAs
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // one K-tile in buffer b (compile-time parity): 4 phases, one barrier each.
  // Phase q: refill the region of buffer b read for the last time in phase
  // q-1 with K-tile t+2, MFMAs of A quarter q, read the next phase's fragments.
  auto tile = [&](int t, auto buf_tag) {
    constexpr int b = decltype(buf_tag)::value;
    const bool pre = t + 2 < nk, nxt = t + 1 < nk;
    if (pre) {
      issue_w(t + 2, b);
      issue_a(0, t + 2, b);
    }
    mfma_phase(I0{});
    read_a(b, 1);
    g256_barrier();
    if (pre) issue_a(1, t + 2, b);
    mfma_phase(I1{});
    read_a(b, 2);
    g256_barrier();
    if (pre) issue_a(2, t + 2, b);
    mfma_phase(I2{});
    read_a(b, 3);
    // K-tile t+1 (issued during tile t-1) must have landed before phase 3
    // reads it; the 7 glds of tile t+2 issued since stay in flight
    if (pre) g256_vmcnt<7>();
    else g256_vmcnt<0>();
    g256_barrier();
    if (pre) issue_a(3, t + 2, b);
    mfma_phase(I3{});
    if (nxt) {
      read_w(b ^ 1);
      read_a(b ^ 1, 0);
    }
    g256_barrier();
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed, its W + A quarter 0 read
  issue_w(0, 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) issue_a(q, 0, 0);
  if (nk > 1) {
    issue_w(1, 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) issue_a(q, 1, 1);
    g256_vmcnt<8>();
  } else {
    g256_vmcnt<0>();
  }
  g256_barrier();
  read_w(0);
  read_a(0, 0);
  g256_barrier();  // every wave's reads of W / A quarter 0 retired before phase 0 refills them
  for (int t = 0; t < nk; t += 2) {
    tile(t, I0{});
    if (t + 1 < nk) tile(t + 1, I1{});
  }

  // ---- epilogue, one M half (64 rows per wave) at a time ----
  const int n0w = n0 + wc * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int m0w = m0 + 128 * wr + 64 * h;
    bool staged = false;
#if MDE_EPI_LDS_256
    staged = store_tile_lds<EM, 4, 4>(
        p, acc[h], [&](int row) { return m0w + row < p.M ? m0w + row : -1; }, n0w, lane,
        smem + wave * (64 * 64 * 4));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    if (!staged) {
      int mrow[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0w + 16 * i + l15;
        mrow[i] = m < p.M ? m : -1;
      }
      store_tile<EM, 4, 4>(p, acc[h], mrow, n0w + hq * 4, lane);
    }
  }
}

}  // namespace

bool gemm256_eligible(const GemmParams& p) {
  const int mode = knob(KNOB_GEMM256);  // 0: never, 1: auto (default), 2: always when legal
  if (mode == 0 || p.amode != A_DENSE || p.emode == E_HEAD) return false;
  if (p.M < 256 || p.N < 256) return false;
  // short K (ViT-S: 384): the prologue/epilogue of a one-workgroup-per-CU tile
  // is not hidden behind a second workgroup -- the 128^2 kernel wins there
  // (fc1 + GELU at B=32: 1.30 -> 1.37 ms)
  if (mode == 1 && p.K < 768) return false;
  const long long tiles = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256);
  if (mode == 2) return true;
  // one workgroup per CU: worth it when whole rounds of 256 tiles stay >= 80 %
  // busy (measured: 516 tiles = 2.02 rounds loses to the 128^2 kernel)
  const long long slots = (tiles + 255) / 256 * 256;
  return (double)p.M * p.N >= 0.8 * (double)slots * 65536.0;
}

hipError_t launch_gemm256(const GemmParams& p, hipStream_t st) {
  const long long blocks = (long long)((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  if (blocks <= 0) return hipSuccess;
  dim3 grid((unsigned)blocks), block(NW * 64);
  switch (p.emode) {
    case E_STORE: hipLaunchKernelGGL(gemm256_kernel<E_STORE>, grid, block, 0, st, p); break;
    case E_QKV: hipLaunchKernelGGL(gemm256_kernel<E_QKV>, grid, block, 0, st, p); break;
    case E_RESID: hipLaunchKernelGGL(gemm256_kernel<E_RESID>, grid, block, 0, st, p); break;
    case E_PATCH: hipLaunchKernelGGL(gemm256_kernel<E_PATCH>, grid, block, 0, st, p); break;
    case E_CONVT: hipLaunchKernelGGL(gemm256_kernel<E_CONVT>, grid, block, 0, st, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mde
