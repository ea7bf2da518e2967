// EXPERIMENT (round 5), not part of libmde_hip: a loader / consumer ring
// GEMM for the batch-1 shapes.
//
// The library's batch-1 GEMMs fill LDS at ~21 GB/s per CU (ViT-L B=1 qkv:
// 512 KB of operands per 128^2 tile in ~24 us): every wave both issues the
// K-step's LDS-DMA and computes, one barrier per K-step, so a CU has about
// one K-step in flight.  MI355X_MICROARCH.md's ring-gemm row measures 68
// GB/s per CU when dedicated loader waves keep K-steps in flight and the
// consumers only wait for a published slot.  This kernel is that structure
// for C[M][N] = A[M][K] W[N][K]^T (f16 in, fp32 accumulate, f16 out + bias):
//
//   * 512 threads: waves 0..3 consumers, 4..7 loaders (one of each per SIMD);
//   * tile BM x BN = (16 TM) x (64 TN): consumer c owns all BM rows and
//     columns [16 TN c, 16 TN (c+1)) -- W as the MFMA A operand, so a lane
//     owns 4 consecutive output columns of one row (the library's layout);
//   * K-steps of 32 (64-B LDS rows, chunk swizzle c ^ ((r >> 1) & 3) on the
//     DMA source and the fragment read), NS slots of (BM + BN) x 64 B;
//   * loader l issues its quarter of stage k into slot k % NS once every
//     consumer has released stage k - NS (free words), then publishes stage
//     k - INF (its counted vmcnt leaves INF stages in flight) in its full word;
//   * consumer c waits for the four full words of stage k, reads its
//     fragments, releases the slot (free word) after lgkmcnt(0), then issues
//     the MFMAs;
//   * every poll loop is bounded (a broken handshake ends the kernel with a
//     wrong result, never a hang) and counted in `stats`.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/ring_gemm tools/experiments/ring_gemm.hip
//   ./build/ring_gemm M N K [iters]      -> one JSON line (time, GB/s per CU, max error vs reference)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef RG_TM
#define RG_TM 9
#endif
#ifndef RG_TN
#define RG_TN 2
#endif
#ifndef RG_NS
#define RG_NS 8
#endif
#ifndef RG_INF
#define RG_INF 4
#endif
#ifndef RG_BK
#define RG_BK 32
#endif
#ifndef RG_GM
#define RG_GM 8
#endif
#ifndef RG_WAUX
#define RG_WAUX 0
#endif

constexpr int TM = RG_TM, TN = RG_TN, NS = RG_NS, INF = RG_INF, BK = RG_BK;
constexpr int BM = 16 * TM, BN = 64 * TN;
constexpr int ROWB = BK * 2;                 // bytes per LDS row
constexpr int CH = BK / 8;                   // 16-B chunks per row
constexpr int RW = 64 / CH;                  // rows per glds wave-instruction
constexpr int STAGE = (BM + BN) * ROWB;
constexpr int AINS = BM / RW, BINS = BN / RW;  // glds wave-instructions per stage
constexpr int INS = AINS + BINS;
static_assert(INS % 4 == 0 || true, "");
constexpr int LPER = (INS + 3) / 4;          // per loader wave (the last may be short)
constexpr int FLAGS = 2 * NS * 4 * 4;        // full[NS][4] + free[NS][4] words
static_assert(NS * STAGE + FLAGS <= 163840, "LDS");
static_assert(NS >= INF + 3, "slots: one to issue into, INF in flight, two published");

__device__ __forceinline__ int pch(int r, int lc) { return BK == 64 ? lc ^ (r & 7) : lc ^ ((r >> 1) & 3); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
  return (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
}

__device__ __forceinline__ void lds_store_flag(volatile int* f, int v) { *f = v; }
__device__ __forceinline__ int lds_load_flag(volatile int* f) { return *f; }

constexpr int SPIN_MAX = 1 << 20;

__global__ void __launch_bounds__(512) ring_gemm(const f16* __restrict__ A, const f16* __restrict__ W,
                                                 const float* __restrict__ bias, f16* __restrict__ C, int M, int N,
                                                 int K, int* __restrict__ stats) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE + FLAGS];
  volatile int* full = reinterpret_cast<volatile int*>(smem + NS * STAGE);  // [NS][4]
  volatile int* freew = full + NS * 4;                                       // [NS][4]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // row blocks in groups of RG_GM (the library's tile_group_m): an XCD's
  // run of workgroups covers GM row blocks x a few N tiles, both operands
  // L2-resident
  int tm, tn;
  {
    const int ntm = (M + BM - 1) / BM, gm = RG_GM;
    if (gm <= 1) {
      tm = bid / ntn;
      tn = bid - tm * ntn;
    } else {
      const int per = gm * ntn, g = bid / per, r = bid - g * per, mb = g * gm;
      const int gs = ntm - mb < gm ? ntm - mb : gm;
      tn = r / gs;
      tm = mb + (r - tn * gs);
    }
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / BK;
  if (tid < NS * 8) (tid < NS * 4 ? full : freew)[tid % (NS * 4)] = 0;
  __syncthreads();

  if (wave >= 4) {
    // ---------------- loader ----------------
    const int l = wave - 4;
    const int lrow = lane / CH, lchp = lane % CH;  // lane -> (row, physical chunk)
    int spins = 0;
    for (int k = 0; k < nk; ++k) {
      const int s = k % NS;
      if (k >= NS) {
        const int need = k - NS + 1;  // stage k - NS released
        for (;;) {
          int ok = 1;
#pragma unroll
          for (int c = 0; c < 4; ++c) ok &= lds_load_flag(freew + s * 4 + c) >= need;
          if (ok || ++spins > SPIN_MAX) break;
          __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
      }
      char* sb = smem + s * STAGE;
#pragma unroll
      for (int j = 0; j < LPER; ++j) {
        const int ins = l + 4 * j;  // wave-instruction index in the stage
        if (ins < INS) {
          const bool isA = ins < AINS;
          const int r = (isA ? ins : ins - AINS) * RW + lrow;  // row in the A or W tile
          const int lc = pch(r, lchp);
          if (isA) {
            const int gm = min(m0 + r, M - 1);
            __builtin_amdgcn_global_load_lds(A + (size_t)gm * K + k * BK + lc * 8, sb + ins * RW * ROWB, 16, 0, 0);
          } else {  // W padded to a multiple of BN rows
            __builtin_amdgcn_global_load_lds(W + (size_t)(n0 + r) * K + k * BK + lc * 8, sb + ins * RW * ROWB, 16, 0,
                                             RG_WAUX);
          }
        }
      }
      // publish stage k - INF: leave INF stages of this wave's DMAs in flight
      // (LPER or LPER - 1 per stage: the stage's instructions dealt round-robin)
      if (k >= INF) {
        if (l + 4 * (LPER - 1) < INS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF * LPER) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF * (LPER - 1)) : "memory");
        if (lane == 0) lds_store_flag(full + ((k - INF) % NS) * 4 + l, k - INF + 1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int k = max(0, nk - INF); k < nk; ++k)
      if (lane == 0) lds_store_flag(full + (k % NS) * 4 + l, k + 1);
    if (lane == 0 && spins > SPIN_MAX) atomicAdd(stats, 1);
    return;
  }

  // ---------------- consumer ----------------
  const int c = wave;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int spins = 0;
  for (int k = 0; k < nk; ++k) {
    const int s = k % NS;
    for (;;) {
      int ok = 1;
#pragma unroll
      for (int l = 0; l < 4; ++l) ok &= lds_load_flag(full + s * 4 + l) >= k + 1;
      if (ok || ++spins > SPIN_MAX) break;
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    const char* sA = smem + s * STAGE;
    const char* sB = sA + BM * ROWB;
    f16x8 fa[BK / 32][TM], fb[BK / 32][TN];
#pragma unroll
    for (int u = 0; u < BK / 32; ++u) {
      const int lc = 4 * u + (lane >> 4);  // logical chunk: K 8lc .. 8lc+7 of the step
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = i * 16 + (lane & 15);
        fa[u][i] = *reinterpret_cast<const f16x8*>(sA + r * ROWB + pch(r, lc) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = (c * TN + j) * 16 + (lane & 15);
        fb[u][j] = *reinterpret_cast<const f16x8*>(sB + r * ROWB + pch(r, lc) * 16);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_store_flag(freew + s * 4 + c, k + 1);
#pragma unroll
    for (int u = 0; u < BK / 32; ++u)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[u][j], fa[u][i], acc[i][j], 0, 0, 0);
  }
  if (lane == 0 && spins > SPIN_MAX) atomicAdd(stats, 1);
  // epilogue: lane owns row m0 + 16 i + (lane & 15), columns n .. n+3
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + (c * TN + j) * 16 + (lane >> 4) * 4;
      if (n >= N) continue;
      const float4 b = *reinterpret_cast<const float4*>(bias + n);
      const f16x4 h = {(f16)(acc[i][j][0] + b.x), (f16)(acc[i][j][1] + b.y), (f16)(acc[i][j][2] + b.z),
                       (f16)(acc[i][j][3] + b.w)};
      *reinterpret_cast<f16x4*>(C + (size_t)m * N + n) = h;
    }
  }
}

__global__ void ref_gemm(const f16* A, const f16* W, const float* bias, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N || m >= M) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(size_t)m * K + k] * (float)W[(size_t)n * K + k];
  C[(size_t)m * N + n] = s + bias[n];
}

__global__ void fill(f16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (f16)(((float)(x & 0xffff) / 65535.f - 0.5f) * scale);
  }
}

__global__ void touch(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] += 1.f;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 1370, N = argc > 2 ? atoi(argv[2]) : 3072, K = argc > 3 ? atoi(argv[3]) : 1024;
  const int iters = argc > 4 ? atoi(argv[4]) : 50;
  if (K % BK) { fprintf(stderr, "K %% BK\n"); return 1; }
  const int Np = (N + BN - 1) / BN * BN;
  f16 *A, *W, *C;
  float *bias, *R, *flush;
  int* stats;
  CHECK(hipMalloc(&A, (size_t)M * K * 2));
  CHECK(hipMalloc(&W, (size_t)Np * K * 2));
  CHECK(hipMalloc(&C, (size_t)M * N * 2));
  CHECK(hipMalloc(&bias, (size_t)Np * 4));
  CHECK(hipMalloc(&R, (size_t)M * N * 4));
  CHECK(hipMalloc(&stats, 4));
  const size_t FL = (size_t)128 << 20;  // 512 MB: evicts L2 and the Infinity Cache
  CHECK(hipMalloc(&flush, FL * 4));
  fill<<<2048, 256>>>(A, (size_t)M * K, 1, 2.f);
  fill<<<2048, 256>>>(W, (size_t)Np * K, 7, 2.f / sqrtf((float)K));
  CHECK(hipMemset(bias, 0, (size_t)Np * 4));
  CHECK(hipMemset(stats, 0, 4));
  CHECK(hipDeviceSynchronize());
  const int tiles = ((M + BM - 1) / BM) * (Np / BN);
  ring_gemm<<<tiles, 512>>>(A, W, bias, C, M, N, K, stats);
  CHECK(hipGetLastError());
  ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, W, bias, R, M, N, K);
  CHECK(hipDeviceSynchronize());
  std::vector<f16> hc((size_t)M * N);
  std::vector<float> hr((size_t)M * N);
  CHECK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  for (size_t i = 0; i < hc.size(); ++i) {
    maxerr = std::max(maxerr, (double)std::fabs((float)hc[i] - hr[i]));
    maxref = std::max(maxref, (double)std::fabs(hr[i]));
  }
  int st = 0;
  CHECK(hipMemcpy(&st, stats, 4, hipMemcpyDeviceToHost));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> warm, cold;
  for (int it = 0; it < iters; ++it) {
    CHECK(hipEventRecord(e0));
    ring_gemm<<<tiles, 512>>>(A, W, bias, C, M, N, K, stats);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    warm.push_back(ms);
  }
  for (int it = 0; it < std::max(5, iters / 5); ++it) {
    touch<<<4096, 256>>>(flush, FL);
    CHECK(hipEventRecord(e0));
    ring_gemm<<<tiles, 512>>>(A, W, bias, C, M, N, K, stats);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    cold.push_back(ms);
  }
  std::sort(warm.begin(), warm.end());
  std::sort(cold.begin(), cold.end());
  const double wm = warm[warm.size() / 2], cm = cold[cold.size() / 2];
  const double tile_bytes = (double)(BM + BN) * K * 2;
  printf("{\"GM\": %d, \"BK\": %d, \"waux\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"BM\": %d, \"BN\": %d, \"NS\": %d, \"INF\": %d, \"tiles\": %d, "
         "\"warm_us\": %.2f, \"cold_us\": %.2f, \"tflops_warm\": %.1f, \"GBps_per_cu_warm\": %.1f, "
         "\"GBps_per_cu_cold\": %.1f, \"max_abs_err\": %.3e, \"max_ref\": %.3e, \"spin_overflows\": %d}\n",
         RG_GM, BK, RG_WAUX, M, N, K, BM, BN, NS, INF, tiles, wm * 1e3, cm * 1e3, 2.0 * M * N * K / (wm * 1e-3) / 1e12,
         tile_bytes / (wm * 1e-3) / 1e9, tile_bytes / (cm * 1e-3) / 1e9, maxerr, maxref, st);
  return 0;
}
