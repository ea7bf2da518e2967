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

MDE_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

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
