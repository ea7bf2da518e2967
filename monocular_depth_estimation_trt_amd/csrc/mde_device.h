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

// GELU (exact-erf definition: nn.GELU() default, upstream DINOv2 Mlp) as
// x * sigmoid(x (a + b x^2 + c x^4)), x clamped to [-8, 8] inside the
// sigmoid argument; a, b, c minimax-fitted to the erf form (log2 e folded
// in): max |error| 2.6e-5 over all x in fp32 (fp16 output ulp is 9.8e-4 at
// 1..2).  6 VALU + v_exp_f32 + v_rcp_f32 instead of ~14 VALU + 2 transcendentals
// plus a correctly rounded division for the A&S 7.1.26 erf.
MDE_DEV float gelu_erf(float x) {
  const float xc = __builtin_amdgcn_fmed3f(x, -8.f, 8.f);
  const float x2 = xc * xc;
  const float z = xc * fmaf(fmaf(0.001014263055f, x2, -0.106775724f), x2, -2.301121339f);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}

// gelu_erf on two lanes' values at once: the polynomial on packed f32
// (v_pk_mul_f32 / v_pk_fma_f32: 5 instructions for both elements), the
// clamp, exp2 and reciprocal per element -- 11 VALU per pair instead of 18,
// bit-identical to gelu_erf (same fused operations in the same order)
typedef float f32x2 __attribute__((ext_vector_type(2)));
MDE_DEV f32x2 gelu_erf2(f32x2 x) {
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x[0], -8.f, 8.f), __builtin_amdgcn_fmed3f(x[1], -8.f, 8.f)};
  const f32x2 x2 = xc * xc;
  const f32x2 c = {0.001014263055f, 0.001014263055f}, b = {-0.106775724f, -0.106775724f},
              a = {-2.301121339f, -2.301121339f};
  const f32x2 z = xc * __builtin_elementwise_fma(__builtin_elementwise_fma(c, x2, b), x2, a);
  const f32x2 d = {1.f + __builtin_amdgcn_exp2f(z[0]), 1.f + __builtin_amdgcn_exp2f(z[1])};
  const f32x2 r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  return x * r;
}

// Folded-LayerNorm row statistics from the producers' 32-column slice
// partials (GemmParams::lnst_in): the 4 lanes that share a row (lane >> 4)
// hold slices q, q + 4, ... (k < kp of t[k]); Chan et al.'s merge across them,
// mean = sum / D and var = M2 / D (invd = 1 / D).  Every operation rounded
// explicitly (no contraction), so the GEMM kernels that fold LN (gemm.hip,
// gemm_panel.hip) compute bit-identical statistics whatever their code around.
MDE_DEV void ln_merge_stats(const float2 (&t)[8], int kp, float invd, float& mean, float& var) {
#pragma clang fp contract(off)
  float s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s1 = s1 + (k < kp ? t[k].x : 0.f);
  s1 = s1 + __shfl_xor(s1, 16);
  s1 = s1 + __shfl_xor(s1, 32);
  mean = s1 * invd;
  float m2 = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float d = t[k].x * (1.f / 32.f) - mean;
    m2 = m2 + (k < kp ? t[k].y + (32.f * d) * d : 0.f);
  }
  m2 = m2 + __shfl_xor(m2, 16);
  m2 = m2 + __shfl_xor(m2, 32);
  var = m2 * invd;
}

// PyTorch upsample_bilinear2d(align_corners=True) source index and weights
// (area_pixel_compute_scale / _source_index in fp32, then floor, clamp of the
// +1 neighbour, lambda = src - i0), each op rounded as on the CPU: contraction
// off, or the lambda would be taken from the unrounded product (errors up to
// 5e-4 relative on steep maps).
MDE_DEV float ac_scale(int in_size, int out_size) {
#pragma clang fp contract(off)
  return out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.f;
}

MDE_DEV void ac_index(float scale, int dst, int in_size, int& i0, int& i1, float& l0, float& l1) {
#pragma clang fp contract(off)
  const float f = scale * (float)dst;
  i0 = (int)f;
  i1 = i0 + (i0 < in_size - 1 ? 1 : 0);
  l1 = f - (float)i0;
  l0 = 1.f - l1;
}

// NHWC f16 bilinear upsample (align_corners=True) of channels [c0, c0 + 8)
// at output pixel (oy, ox) of an oh x ow map, from in [b][ih][iw][C]: the
// four taps blended in packed f16 in lerp form, a + (b - a) w, x then y
// (resize_kernel, and the E_STORE epilogue's resize-on-read of
// GemmParams::res1_up -- one function, so both give the same bits).  Each
// axis' two weights sum to exactly 1: a constant map stays constant.
typedef f16 f16x2u __attribute__((ext_vector_type(2)));
MDE_DEV f16x8 upsample8(const f16* __restrict__ in, int b, int ih, int iw, int C, int oh, int ow, int oy, int ox,
                        int c0) {
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  ac_index(ac_scale(ih, oh), oy, ih, y0, y1, ly0, ly1);
  ac_index(ac_scale(iw, ow), ox, iw, x0, x1, lx0, lx1);
  (void)lx0;
  (void)ly0;
  const f16* base = in + (size_t)b * ih * iw * C + c0;
  const f16x8 a = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * iw + x0) * C);
  const f16x8 bb = *reinterpret_cast<const f16x8*>(base + ((size_t)y0 * iw + x1) * C);
  const f16x8 c = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * iw + x0) * C);
  const f16x8 d = *reinterpret_cast<const f16x8*>(base + ((size_t)y1 * iw + x1) * C);
  const f16x2u wx1 = {(f16)lx1, (f16)lx1}, wy1 = {(f16)ly1, (f16)ly1};
  f16x8 v;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f16x2u a2 = {a[j], a[j + 1]}, b2 = {bb[j], bb[j + 1]}, c2 = {c[j], c[j + 1]}, d2 = {d[j], d[j + 1]};
    const f16x2u t0 = a2 + (b2 - a2) * wx1, t1 = c2 + (d2 - c2) * wx1;
    const f16x2u r = t0 + (t1 - t0) * wy1;
    v[j] = r[0];
    v[j + 1] = r[1];
  }
  return v;
}

// Storage position of key t in a V^T row: bits 2 and 3 of t swapped.  The
// attention's P.V MFMA (32x32x16, P^T straight from the score accumulator)
// takes, in lane half h of k-step g, the keys {16g + 4h + 0..3, 16g + 8 + 4h +
// 0..3}; stored at 16g + 8h + 0..7 they are one contiguous 16-byte read.
MDE_DEV int vt_pos(int t) { return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1); }

// XCD-aware workgroup order (bijective for any grid): workgroups are dealt
// round-robin over the 8 XCDs (bid % 8 shares an L2), so renumber them to
// give each XCD a contiguous run -- neighbouring work items that share
// source lines then fetch them into one L2 instead of several.
MDE_DEV int xcd_remap(int bid, int nwg) {
  const int q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
  return (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
}

// Tile (tm, tn) of the linear workgroup index `bid` (after the XCD remap,
// which hands each XCD a contiguous run of bids).  gm <= 1: row-major, N
// fastest -- the N tiles of a row block share A in one L2.  gm > 1: row
// blocks in groups of gm, tm fastest inside a group, so the ~32 workgroups an
// XCD runs together cover gm row blocks x a few N tiles and BOTH operands
// stay L2-resident (W larger than an XCD's 4 MB L2 is otherwise re-streamed
// once per row block).  Bijective for any ntm, ntn.
MDE_DEV void tile_of(int bid, int ntm, int ntn, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = bid / ntn;
    tn = bid - tm * ntn;
    return;
  }
  const int per = gm * ntn;
  const int g = bid / per, r = bid - g * per;
  const int mb = g * gm;
  const int gs = ntm - mb < gm ? ntm - mb : gm;
  tn = r / gs;
  tm = mb + (r - tn * gs);
}

// Row-block group of tile_of for a weight operand of n x k halves and bm-row
// tiles: group when W would not stay resident in an XCD's L2 next to the A
// blocks, with at most ~2 MB of A rows per group.  Measured on VGGT-1B
// (profiles/r01_v1[2-4]_vggt_traffic_*): qkv (K 1024, W 6 MB) 477 -> 222 MB
// per launch with groups of 8; fc2 (K 4096, 1 MB of A per row block) best
// row-major: 328 MB vs 344 (groups of 2) and 372 (groups of 8).
MDE_DEV int tile_group_m(int n, int k, int bm) {
  if ((long long)n * k * 2 <= (2ll << 20)) return 1;
  const long long per = (long long)bm * k * 2;
  if (per >= (1ll << 20)) return 1;
  const int g = (int)((2ll << 20) / per);
  return g < 1 ? 1 : (g > 8 ? 8 : g);
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
