// Device-side types and helpers shared by the gfx950 kernels (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mde {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MDE_DEV __device__ __forceinline__

MDE_DEV f32x4 mfma16x16x32(const f16x8& a, const f16x8& b, const f32x4& c) {
  // D[16x16] += A[16x32] * B[32x16]; lane l holds A[l&15][8(l>>4)+j],
  // B[8(l>>4)+j][l&15]; D row (l>>4)*4+r, col l&15.
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

MDE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, below f16 rounding):
// one exp + one reciprocal instead of the libm polynomial ladder.
MDE_DEV float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __frcp_rn(1.0f + 0.3275911f * ax);
  const float poly = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t +
                      0.254829592f) * t;
  const float y = 1.0f - poly * __expf(-ax * ax);
  return copysignf(y, x);
}

// GELU with the exact-erf definition (nn.GELU() default, upstream DINOv2 Mlp).
MDE_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// Storage position of key t in a V^T row: inside every 32-key group the keys
// are ordered [4 keys of sub-tile 0 | 4 keys of sub-tile 1] per 4-key lane
// slot, so the 8 keys one MFMA lane consumes in P.V ({32g+4h+0..3,
// 32g+16+4h+0..3}) are one contiguous 16-byte read.
MDE_DEV int vt_pos(int t) {
  const int k = t & 31;
  return (t & ~31) | ((k & 15) >> 2) << 3 | (k >> 4) << 2 | (k & 3);
}

MDE_DEV f16x8 zero8() {
  f16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (f16)0.0f;
  return z;
}

MDE_DEV f16x8 relu8(f16x8 v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = v[i] > (f16)0.0f ? v[i] : (f16)0.0f;
  return v;
}

}  // namespace mde
