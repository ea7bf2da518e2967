// Fused scaled-dot-product attention, head dim 64, for the DINOv2 blocks
// (reference = TensorRT `_gemm_mha_v2`, restating
// upstream `Attention.forward`: softmax(q*dh^-0.5 @ k^T) @ v).
//
// Layouts (written by the qkv GEMM epilogue, E_QKV):
//   q, k : [B*H][Tpad][64] f16, q already multiplied by dh^-0.5 = 1/8 (exact)
//   vt   : [B*H][64][Tpad] f16 (v transposed), pad columns t >= T are zero
//   o    : [B*T][ldo] f16, head h in columns h*64 .. h*64+63
//
// One workgroup = 4 waves = 64 queries of one (batch, head); each wave owns 16
// queries.  The score tile is computed TRANSPOSED, S^T = K Q^T, so the MFMA
// accumulator holds a key x query block whose query sits on the lane: the
// online-softmax max/sum over keys is a reduction over registers plus two
// lane shuffles (xor 16, 32), and P^T feeds the P.V MFMA as the B operand
// straight from the accumulator (O^T = V^T P^T) with no LDS round trip.
// K and V^T key tiles (64 keys) are register-staged into a double-buffered
// LDS image with conflict-free swizzles (K: chunk ^ (row&7) for ds_read_b128;
// V^T: chunk ^ ((row>>1)&7) for ds_read_b64).  Softmax statistics are fp32.
#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

constexpr int KT = 64;  // keys per tile
constexpr float LOG2E = 1.4426950408889634f;

typedef f16 f16x4v __attribute__((ext_vector_type(4)));

MDE_DEV int kswz(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }
MDE_DEV int vswz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }

__global__ void __launch_bounds__(256) attn_fwd_kernel(const f16* __restrict__ q, const f16* __restrict__ k,
                                                        const f16* __restrict__ vt, f16* __restrict__ o,
                                                        int H, int T, int Tpad, int ldo) {
  __shared__ __attribute__((aligned(16))) f16 sK[2][KT * 64];
  __shared__ __attribute__((aligned(16))) f16 sV[2][64 * KT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int qbase = blockIdx.x * 64 + wave * 16;
  const int l15 = lane & 15, hq = lane >> 4;

  const f16* qb = q + (size_t)bh * Tpad * 64;
  const f16* kb = k + (size_t)bh * Tpad * 64;
  const f16* vb = vt + (size_t)bh * 64 * Tpad;

  // Q^T fragments (B operand): lane holds Q[q = qbase + l15][32s + 8hq + j]
  f16x8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    qf[s] = *reinterpret_cast<const f16x8*>(qb + (size_t)(qbase + l15) * 64 + 32 * s + 8 * hq);

  // staging: 512 chunks of 16B per tile for K and for V^T; 2 + 2 per thread
  f16x8 rk[2], rv[2];
  auto fetch = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256;
      const int row = c >> 3, ch = c & 7;
      rk[i] = *reinterpret_cast<const f16x8*>(kb + (size_t)(kt * KT + row) * 64 + ch * 8);
      rv[i] = *reinterpret_cast<const f16x8*>(vb + (size_t)row * Tpad + kt * KT + ch * 8);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256;
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<f16x8*>(&sK[buf][kswz(row, ch)]) = rk[i];
      *reinterpret_cast<f16x8*>(&sV[buf][vswz(row, ch)]) = rv[i];
    }
  };

  float m_run = -INFINITY;  // running max (log2 domain) of this lane's query
  float l_run = 0.f;        // this lane's partial row sum (its 16 key rows per tile)
  f32x4 acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (T + KT - 1) / KT;
  fetch(0);
  stash(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) fetch(kt + 1);
    const f16* K_ = sK[cur];
    const f16* V_ = sV[cur];

    // S^T[key][query] for 4 key sub-tiles of 16
    f32x4 s[4];
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      s[t4] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = t4 * 16 + l15;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(K_ + kswz(row, 4 * ss + hq));
        s[t4] = mfma16x16x32(kf, qf[ss], s[t4]);
      }
    }
    // mask keys beyond T, scale to log2 domain, tile max
    const int key0 = kt * KT + hq * 4;
    float mx = -INFINITY;
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + t4 * 16 + r;
        const float z = key < T ? s[t4][r] * LOG2E : -INFINITY;
        s[t4][r] = z;
        mx = fmaxf(mx, z);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float ls = 0.f;
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = exp2f(s[t4][r] - m_new);
        s[t4][r] = pv;
        ls += pv;
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] *= alpha;

    // P^T as B operand: k-index j<4 -> key sub-tile 2ks, j>=4 -> 2ks+1 (rows 4hq+r)
    f16x8 pb[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb[ks][r] = (f16)s[2 * ks][r];
        pb[ks][4 + r] = (f16)s[2 * ks + 1][r];
      }
    // O^T[dh][q] += V^T[dh][key] P^T[key][q]
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int row = d * 16 + l15;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ka = 32 * ks + 4 * hq;  // keys ka..ka+3 and ka+16..ka+19
        const int kb2 = ka + 16;
        const f16x4v lo = *reinterpret_cast<const f16x4v*>(V_ + vswz(row, ka >> 3) + (ka & 7));
        const f16x4v hi = *reinterpret_cast<const f16x4v*>(V_ + vswz(row, kb2 >> 3) + (kb2 & 7));
        f16x8 af;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          af[r] = lo[r];
          af[4 + r] = hi[r];
        }
        acc[d] = mfma16x16x32(af, pb[ks], acc[d]);
      }
    }
    if (kt + 1 < nkt) stash(cur ^ 1);
    __syncthreads();
  }

  float lt = l_run;
  lt += __shfl_xor(lt, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float inv = 1.f / lt;
  const int qi = qbase + l15;
  if (qi < T) {
    f16* orow = o + ((size_t)b * T + qi) * ldo + h * 64;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      f16x4v v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (f16)(acc[d][r] * inv);
      *reinterpret_cast<f16x4v*>(orow + d * 16 + hq * 4) = v;
    }
  }
}

}  // namespace

hipError_t launch_attention(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T,
                            int Tpad, int ldo, hipStream_t st) {
  if (B <= 0 || T <= 0) return hipSuccess;
  if (Tpad % KT || Tpad < ((T + KT - 1) / KT) * KT) return hipErrorInvalidValue;
  dim3 grid((T + 63) / 64, B * H);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, st, reinterpret_cast<const f16*>(q),
                     reinterpret_cast<const f16*>(k), reinterpret_cast<const f16*>(vt),
                     reinterpret_cast<f16*>(o), H, T, Tpad, ldo);
  return hipGetLastError();
}

}  // namespace mde
