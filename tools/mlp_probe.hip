// Phase timing of the fused MLP kernel (mlp.hip built with MLP_PROBE 1):
// synthetic ViT-S shapes (D 384, hidden 1536), M rows, one warm launch, then
// a timed launch whose per-wave clock stamps are summarised.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o build/mlp_probe tools/mlp_probe.hip
//   ./build/mlp_probe [M]          (default 65760 = ViT-S 518^2 x 48 images)
#define MLP_PROBE 1
#include "experiments/mlp_fused.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 65760;
  const int D = 384, H = 1536;
  std::vector<_Float16> x((size_t)M * D), w1((size_t)H * D), w2((size_t)D * H);
  unsigned s = 12345u;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 9) & 0xffff) / 65536.f - 0.5f; };
  for (auto& v : x) v = (_Float16)rnd();
  for (auto& v : w1) v = (_Float16)(rnd() * 0.1f);
  for (auto& v : w2) v = (_Float16)(rnd() * 0.05f);
  // LayerNorm partials consistent with mean 0.1 / var 1 per 32-column slice
  std::vector<float> lnst((size_t)12 * M * 2);
  for (size_t i = 0; i < lnst.size(); i += 2) { lnst[i] = 3.2f; lnst[i + 1] = 32.f; }
  std::vector<float> c1(H), c2(H), b2(D), ls2(D);
  for (int n = 0; n < H; ++n) { c1[n] = 0.3f * (n % 7); c2[n] = 0.2f * ((n % 5) - 2); }
  for (int n = 0; n < D; ++n) { b2[n] = 0.01f * ((n % 3) - 1); ls2[n] = 0.5f + 0.1f * (n % 4); }

  _Float16 *dx, *dw1, *dw2;
  float *dst, *dc1, *dc2, *db2, *dls2;
  CK(hipMalloc(&dx, x.size() * 2));
  CK(hipMalloc(&dw1, w1.size() * 2));
  CK(hipMalloc(&dw2, w2.size() * 2));
  CK(hipMalloc(&dst, lnst.size() * 4));
  CK(hipMalloc(&dc1, H * 4));
  CK(hipMalloc(&dc2, H * 4));
  CK(hipMalloc(&db2, D * 4));
  CK(hipMalloc(&dls2, D * 4));
  CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw1, w1.data(), w1.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw2, w2.data(), w2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc1, c1.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc2, c2.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db2, b2.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dls2, ls2.data(), D * 4, hipMemcpyHostToDevice));
  const int blocks = (M + mde::MROWS - 1) / mde::MROWS;
  const int nw = blocks * mde::MNWV;
  unsigned long long* dprobe;
  CK(hipMalloc(&dprobe, (size_t)nw * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(mde::g_mlp_probe), &dprobe, sizeof(dprobe)));

  mde::MlpParams p;
  p.xh = reinterpret_cast<mde::h16*>(dx);
  p.M = M;
  p.lnst = dst;
  p.lnst_rows = M;
  p.w1 = reinterpret_cast<const mde::h16*>(dw1);
  p.ldw1 = D;
  p.c1 = dc1;
  p.c2 = dc2;
  p.w2 = reinterpret_cast<const mde::h16*>(dw2);
  p.ldw2 = H;
  p.b2 = db2;
  p.ls2 = dls2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.f;
  for (int it = 0; it < 3; ++it) {
    CK(hipMemcpy(dst, lnst.data(), lnst.size() * 4, hipMemcpyHostToDevice));
    CK(hipEventRecord(e0, 0));
    CK(mde::launch_mlp_fused(p, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("launch %d: %.1f us (%d workgroups)\n", it, ms * 1000.f, blocks);
  }
  // correctness: the last launch's output rows vs a CPU restatement (LN stats
  // mean 0 / var 1, fold c1 / c2, erf GELU, fc2 over the packed K permutation)
  {
    std::vector<_Float16> y((size_t)M * D);
    CK(hipMemcpy(y.data(), dx, y.size() * 2, hipMemcpyDeviceToHost));
    // the kernel ran 3 times in place: rerun the reference 3 times on the checked rows
    const float rs = 1.f / std::sqrt(1.f + 1e-6f);
    auto kperm = [](int kp) {  // packed position -> natural hidden column
      const int q = kp / 32, w = kp % 32, g = w / 8, j = w % 8;
      return 32 * q + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
    };
    double maxerr = 0.0;
    int checked = 0;
    for (int row = 0; row < M; row += (row < 256 ? 1 : 997)) {
      std::vector<float> xr(D), h(H);
      for (int k = 0; k < D; ++k) xr[k] = (float)x[(size_t)row * D + k];
      for (int rep = 0; rep < 3; ++rep) {
        for (int n = 0; n < H; ++n) {
          double a = 0;
          for (int k = 0; k < D; ++k) a += (double)(float)w1[(size_t)n * D + k] * xr[k];
          const float t = rs * (float)a - rs * 0.1f * c1[n] + c2[n];
          h[n] = (float)(_Float16)(0.5f * t * (1.f + std::erf(t / std::sqrt(2.f))));
        }
        std::vector<float> o(D);
        for (int n = 0; n < D; ++n) {
          double a = 0;
          for (int kp = 0; kp < H; ++kp) a += (double)(float)w2[(size_t)n * H + kp] * h[kperm(kp)];
          o[n] = (float)(_Float16)(ls2[n] * ((float)a + b2[n]) + xr[n]);
        }
        xr = o;
      }
      for (int n = 0; n < D; ++n) maxerr = std::max(maxerr, (double)std::fabs((float)y[(size_t)row * D + n] - xr[n]));
      ++checked;
    }
    std::printf("check: %d rows, max |gpu - cpu| = %.4g\n", checked, maxerr);
    if (maxerr > 0.02) std::printf("CHECK FAILED\n");
  }
  std::vector<unsigned long long> pr((size_t)nw * 8);
  CK(hipMemcpy(pr.data(), dprobe, pr.size() * 8, hipMemcpyDeviceToHost));
  // per wave: prologue (0->1), first stage wait (1->2), loop (2->3),
  // epilogue (3->4), barrier+wait time inside the loop (5), wall (realtime 7->6)
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  std::vector<double> pro, first, loop, epi, wait, total, rstart, rlen;
  unsigned long long rt0 = ~0ull;
  for (int w = 0; w < nw; ++w) rt0 = std::min(rt0, pr[(size_t)w * 8 + 7]);
  for (int w = 0; w < nw; ++w) {
    const unsigned long long* q = &pr[(size_t)w * 8];
    pro.push_back((double)(q[1] - q[0]));
    first.push_back((double)(q[2] - q[1]));
    loop.push_back((double)(q[3] - q[2]));
    epi.push_back((double)(q[4] - q[3]));
    wait.push_back((double)q[5]);
    total.push_back((double)(q[4] - q[0]));
    rstart.push_back((double)(q[7] - rt0) / 100.0);  // 100 MHz realtime -> us
    rlen.push_back((double)(q[6] - q[7]) / 100.0);
  }
  std::printf("median clocks per wave: prologue %.0f, first stage %.0f, loop %.0f (of it waiting %.0f = %.1f%%), "
              "epilogue %.0f, total %.0f\n",
              med(pro), med(first), med(loop), med(wait), 100.0 * med(wait) / med(loop), med(epi), med(total));
  std::printf("per stage (144): %.0f clocks, waiting %.0f\n", med(loop) / 144.0, med(wait) / 144.0);
  std::printf("wall per workgroup: median %.2f us; start times: min %.2f median %.2f max %.2f us\n", med(rlen),
              *std::min_element(rstart.begin(), rstart.end()), med(rstart),
              *std::max_element(rstart.begin(), rstart.end()));
  // histogram of start times (rounds)
  int hist[16] = {0};
  const double mx = *std::max_element(rstart.begin(), rstart.end()) + 1e-9;
  for (double v : rstart) hist[std::min(15, (int)(v / mx * 16))]++;
  std::printf("start-time histogram (16 bins to %.1f us):", mx);
  for (int i = 0; i < 16; ++i) std::printf(" %d", hist[i] / mde::MNWV);
  std::printf("\n");
  return 0;
}
