// Dense f16 MFMA peak of this MI355X, measured (BASELINE.md:41-42).
//
// Every wave keeps 4 independent 32x32 fp32 accumulators and issues
// v_mfma_f32_32x32x16_f16 back to back on operands held in registers.  The
// operands are random f16 (N(0,1)-ish from a seeded LCG on the host), four
// different A/B pairs cycled so the multiplier inputs toggle every issue --
// zero or constant operands let the chip hold a higher clock than a real GEMM
// does (MI355X_MICROARCH.md "DVFS give-back" 1).  The 16x16x32 form is
// measured too.  Grid: 8 workgroups of 256 threads per CU (one wave per SIMD
// per workgroup; 2048 workgroups), long enough (≈0.1 s per launch) for the
// clock to settle; the figure reported is the median of the timed launches.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/mfma_peak tools/mfma_peak.hip
//   ./build/mfma_peak [iters]   -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void mfma32_loop(const half8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  half8 a0 = src[lane], a1 = src[64 + lane], a2 = src[128 + lane], a3 = src[192 + lane];
  half8 b0 = src[256 + lane], b1 = src[320 + lane], b2 = src[384 + lane], b3 = src[448 + lane];
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b2, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a3, b3, c3, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b2, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b3, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a3, b0, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma16_loop(const half8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  half8 a0 = src[lane], a1 = src[64 + lane], a2 = src[128 + lane], a3 = src[192 + lane];
  half8 b0 = src[256 + lane], b1 = src[320 + lane], b2 = src[384 + lane], b3 = src[448 + lane];
  floatx4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    // 16 MFMAs of 16x16x32 = the FLOPs of 8 of 32x32x16 per iteration
    #pragma unroll
    for (int r = 0; r < 2; ++r) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b2, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3, b3, c3, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b2, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b3, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3, b0, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, c3, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 100000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, threads = 256;

  // random f16 operands, seeded (LCG -> Irwin-Hall sum of 4 uniforms, ~N(0,1))
  std::vector<_Float16> h(512 * 8);
  unsigned long long st = 0x9E3779B97F4A7C15ull;
  for (auto& x : h) {
    float s = 0.f;
    for (int k = 0; k < 4; ++k) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      s += (float)((st >> 40) & 0xFFFFFF) / 16777216.0f;
    }
    x = (_Float16)((s - 2.0f) * 1.7320508f);
  }
  half8* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * sizeof(_Float16)));
  CHECK(hipMalloc(&out, (size_t)blocks * threads * sizeof(float)));
  CHECK(hipMemcpy(src, h.data(), h.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));

  // FLOPs per launch: waves x iters x 8 MFMAs x 2*32*32*16
  const double waves = (double)blocks * threads / 64;
  const double flop = waves * iters * 8 * 2.0 * 32 * 32 * 16;
  double res[2];
  for (int kind = 0; kind < 2; ++kind) {
    std::vector<double> tf;
    for (int rep = 0; rep < 12; ++rep) {   // first 4 launches warm the clock up, untimed
      CHECK(hipEventRecord(e0, 0));
      if (kind == 0) mfma32_loop<<<blocks, threads>>>(src, out, iters);
      else mfma16_loop<<<blocks, threads>>>(src, out, iters);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 4) tf.push_back(flop / (ms * 1e-3) / 1e12);
    }
    res[kind] = median(tf);
    fprintf(stderr, "[mfma_peak] %s: median %.1f TF/s (min %.1f max %.1f) over %zu launches of %.3f TFLOP\n",
            kind == 0 ? "32x32x16_f16" : "16x16x32_f16", res[kind], *std::min_element(tf.begin(), tf.end()),
            *std::max_element(tf.begin(), tf.end()), tf.size(), flop / 1e12);
  }
  std::vector<float> hout(16);
  CHECK(hipMemcpy(hout.data(), out, 16 * sizeof(float), hipMemcpyDeviceToHost));
  printf("{\"mfma_f16_32x32x16_tflops\": %.1f, \"mfma_f16_16x16x32_tflops\": %.1f, \"cus\": %d, "
         "\"workgroups\": %d, \"iters\": %d, \"operands\": \"random f16, 4 A/B pairs cycled\", "
         "\"spec_dense_tflops\": 2500.0, \"device\": \"%s\", \"check\": %g}\n",
         res[0], res[1], cus, blocks, iters, prop.gcnArchName, (double)hout[0]);
  return 0;
}
