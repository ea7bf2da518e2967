// Fused scaled-dot-product attention, head dim 64, for the DINOv2 blocks
// (reference = TensorRT `_gemm_mha_v2`, restating
// upstream `Attention.forward`: softmax(q*dh^-0.5 @ k^T) @ v).
//
// Layouts (written by the qkv GEMM epilogue, E_QKV):
//   q, k : [B*H][Tpad][64] f16, q pre-multiplied by dh^-0.5 * log2(e), so the
//          scores come out in log2 units and exp() is one v_exp_f32 (exp2)
//   vt   : [B*H][64][Tpad] f16 (v transposed; key t stored at vt_pos(t), a
//          permutation inside each 32-key group), pad columns t >= T zero
//   o    : [B*T][ldo] f16, head h in columns h*64 .. h*64+63
//
// Structure.  A workgroup = NW waves; a wave owns QW (16 or 32) queries as
// 16-query column blocks.  The score tile is computed TRANSPOSED, S^T = K Q^T,
// so the query sits on the MFMA lane: the online-softmax max / sum over keys
// is a reduction over the lane's registers plus two lane shuffles (xor 16,
// 32), and P^T feeds the P.V MFMA as the B operand straight from the
// accumulators (O^T = V^T P^T), no LDS round trip.  K and V^T key tiles (64
// keys) stream global -> LDS by global_load_lds through a 3-slot ring, two
// tiles in flight, counted `s_waitcnt vmcnt` + raw s_barrier (a
// __syncthreads() would drain the DMA).  LDS images are lane-linear with the
// swizzle chunk ^ (row & 7) applied on the source address (conflict-free
// ds_read_b128 for both).  The running max rides in the score MFMA's C
// operand (S' = QK^T - m), so the softmax is max-check + exp2 + sum per
// element; O and l are rescaled only when a max grows.  Softmax statistics in
// fp32; keys >= T are masked on the last tile only.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

namespace {

constexpr int KT = 64;        // keys per tile
constexpr int TILE_B = KT * 128;  // bytes of one K (or V^T) tile image: 64 rows x 128 B

typedef f16 f16x4v __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Deferred rescale (cdna_hip_programming.md 5.5 T13): the running max moves
// only when a tile's max exceeds it by more than RESCALE_T (log2 units), so
// p = exp2(S - m_run) <= 2^RESCALE_T = 256 -- exact in f16's range, and the
// rescale branch (O, l *= 2^-delta) is taken a few times per row, not per tile.
constexpr float RESCALE_T = 8.f;

// byte offset of 16-B chunk `chunk` of a 128-B row: conflict-free ds_read_b128
MDE_DEV int kswz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// max / sum over the 4 lanes {l, l^16, l^32, l^48} with VALU lane swaps
// (v_permlane16/32_swap) instead of LDS-routed shuffles
MDE_DEV float xmax4(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r2[0]), __uint_as_float(r2[1]));
}
MDE_DEV float xsum4(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

template <int N>
MDE_DEV void wait_vm_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier that leaves LDS-DMA in flight: own LDS reads retired,
// raw s_barrier, and compiler fences so no LDS access moves across it.
MDE_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int QW, int NW>
__global__ void __launch_bounds__(NW * 64) attn_fwd_kernel(const f16* __restrict__ q, const f16* __restrict__ k,
                                                           const f16* __restrict__ vt, f16* __restrict__ o, int H,
                                                           int T, int Tpad, int ldo) {
  constexpr int NQ = QW / 16;            // 16-query blocks per wave
  constexpr int BQ = QW * NW;            // queries per workgroup
  constexpr int INS = 8 / NW;            // glds instructions per wave per image (8 per 64-row image)
  constexpr int PER_TILE = 2 * INS;      // K + V^T
  constexpr int SLOT = 2 * TILE_B;
  static_assert(8 % NW == 0, "waves must divide the 8 glds instructions of a tile");
  __shared__ __attribute__((aligned(16))) char smem[3 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs
  // (linear id % 8 shares an L2); remap so each XCD takes a contiguous run
  // of (head, query block) pairs and a head's K/V^T is fetched into one L2,
  // not eight (PMC: 4.5x the algorithmic bytes without it).  Bijective.
  const int nqb = gridDim.x, nwg = gridDim.x * gridDim.y;
  int lin = blockIdx.y * nqb + blockIdx.x;
  {
    const int q8 = nwg / 8, r8 = nwg % 8, x = lin % 8;
    lin = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lin / 8;
  }
  const int bh = lin / nqb;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int qbase = (lin - bh * nqb) * BQ + wave * QW;
  const int l15 = lane & 15, hq = lane >> 4;

  const f16* qb = q + (size_t)bh * Tpad * 64;
  const f16* kb = k + (size_t)bh * Tpad * 64;
  const f16* vb = vt + (size_t)bh * 64 * Tpad;

  // Q^T fragments (B operand): lane holds Q[q][32s + 8hq + j] of its query column
  f16x8 qf[NQ][2];
#pragma unroll
  for (int c = 0; c < NQ; ++c)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qi = qbase + c * 16 + l15;
      qf[c][s] = qi < Tpad ? *reinterpret_cast<const f16x8*>(qb + (size_t)qi * 64 + 32 * s + 8 * hq) : zero8();
    }

  // glds geometry: lane -> row lrow of an 8-row group, physical chunk lane & 7
  const int lrow = lane >> 3, pc = lane & 7;
  auto issue = [&](int kt, int slot) {
    char* sK = smem + slot * SLOT;
    char* sV = sK + TILE_B;
#pragma unroll
    for (int i = 0; i < INS; ++i) {
      const int g = wave * INS + i;  // 8-row group 0..7
      const int row = g * 8 + lrow;
      const int kch = pc ^ (row & 7);
      __builtin_amdgcn_global_load_lds(kb + (size_t)(kt * KT + row) * 64 + kch * 8, sK + g * 8 * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(vb + (size_t)row * Tpad + kt * KT + kch * 8, sV + g * 8 * 128, 16, 0, 0);
    }
  };

  // running max per query (log2 units) as an MFMA C operand: every tile after
  // the first computes S' = S - m_run directly in the accumulator, so
  // p = exp2(S') needs no subtraction unless some max grew (rare branch)
  float m_run[NQ], l_run[NQ];
  f32x4 negm[NQ];
  f32x4 acc[NQ][4];
#pragma unroll
  for (int c = 0; c < NQ; ++c) {
    m_run[c] = 0.f;
    l_run[c] = 0.f;
    negm[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[c][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int nkt = (T + KT - 1) / KT;
  issue(0, 0);
  if (nkt > 1) {
    issue(1, 1);
    wait_vm_n<PER_TILE>();
  } else {
    wait_vm_n<0>();
  }
  lds_barrier();

  auto tile = [&](int kt, auto slot_tag, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    constexpr int slot = decltype(slot_tag)::value;  // compile-time: LDS offsets fold into ds_read immediates
    const char* K_ = smem + slot * SLOT;
    const char* V_ = K_ + TILE_B;
    // S'^T[key][query] = K Q^T - m_run: 4 key sub-tiles x NQ query blocks
    f32x4 s[NQ][4];
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      const int row = t4 * 16 + l15;
      const f16x8 k0 = *reinterpret_cast<const f16x8*>(K_ + kswz(row, hq));
      const f16x8 k1 = *reinterpret_cast<const f16x8*>(K_ + kswz(row, 4 + hq));
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        s[c][t4] = mfma16x16x32(k0, qf[c][0], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : negm[c]);
        s[c][t4] = mfma16x16x32(k1, qf[c][1], s[c][t4]);
      }
    }
    if (kt * KT + KT > T) {  // last, partial tile: keys >= T -> -inf
      const int key0 = kt * KT + hq * 4;
#pragma unroll
      for (int c = 0; c < NQ; ++c)
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (key0 + t4 * 16 + r >= T) s[c][t4][r] = -INFINITY;
    }
    f16x8 pb[NQ][2];
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      // max over the lane's 16 scores as a chain of v_max3 (8 ops)
      float mx = fmaxf(fmaxf(s[c][0][0], s[c][0][1]), s[c][0][2]);
      mx = fmaxf(fmaxf(mx, s[c][0][3]), s[c][1][0]);
      mx = fmaxf(fmaxf(mx, s[c][1][1]), s[c][1][2]);
      mx = fmaxf(fmaxf(mx, s[c][1][3]), s[c][2][0]);
      mx = fmaxf(fmaxf(mx, s[c][2][1]), s[c][2][2]);
      mx = fmaxf(fmaxf(mx, s[c][2][3]), s[c][3][0]);
      mx = fmaxf(fmaxf(mx, s[c][3][1]), s[c][3][2]);
      mx = fmaxf(mx, s[c][3][3]);
      mx = xmax4(mx);  // max of S' over the tile (relative to m_run)
      if (FIRST || __any(mx > RESCALE_T)) {
        // the running max grows by delta >= 0: shift S', rescale O and l
        const float delta = FIRST ? mx : fmaxf(mx, 0.f);
        m_run[c] += delta;
        negm[c] = f32x4{-m_run[c], -m_run[c], -m_run[c], -m_run[c]};
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) s[c][t4] -= delta;
        if (!FIRST) {
          const float alpha = __builtin_amdgcn_exp2f(-delta);
          l_run[c] *= alpha;
#pragma unroll
          for (int d = 0; d < 4; ++d) acc[c][d] *= alpha;
        }
      }
      f32x2 ls2 = {0.f, 0.f};  // packed row sums (v_pk_add_f32)
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 pv = {__builtin_amdgcn_exp2f(s[c][t4][r]), __builtin_amdgcn_exp2f(s[c][t4][r + 1])};
          s[c][t4][r] = pv[0];
          s[c][t4][r + 1] = pv[1];
          ls2 += pv;
        }
      l_run[c] += ls2[0] + ls2[1];
      // P^T as B operand: k index j<4 -> key sub-tile 2ks, j>=4 -> 2ks+1 (rows 4hq+r)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pb[c][ks][r] = (f16)s[c][2 * ks][r];
          pb[c][ks][4 + r] = (f16)s[c][2 * ks + 1][r];
        }
    }
    // O^T[dh][q] += V^T[dh][key] P^T[key][q]; V^T keys are stored vt_pos-
    // permuted, so the 8 keys of k-step ks for lane slot hq are one 16-B chunk
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int row = d * 16 + l15;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 af = *reinterpret_cast<const f16x8*>(V_ + kswz(row, 4 * ks + hq));
#pragma unroll
        for (int c = 0; c < NQ; ++c) acc[c][d] = mfma16x16x32(af, pb[c][ks], acc[c][d]);
      }
    }
  };

  // tile kt lives in ring slot kt % 3; the loop is unrolled over the three
  // slots so every LDS address is lane base + immediate
  auto step = [&](int kt, auto slot_tag, auto first_tag) {
    constexpr int SL = decltype(slot_tag)::value;
    if (kt + 2 < nkt) issue(kt + 2, (SL + 2) % 3);
    tile(kt, slot_tag, first_tag);
    // tile kt+1 must have landed before anyone reads it; its slot's previous
    // contents (tile kt-2) were released at the previous barrier
    if (kt + 2 < nkt) wait_vm_n<PER_TILE>();
    else wait_vm_n<0>();
    lds_barrier();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  step(0, S0{}, std::true_type{});
  int kt = 1;
  for (; kt + 3 <= nkt; kt += 3) {
    step(kt, S1{}, std::false_type{});
    step(kt + 1, S2{}, std::false_type{});
    step(kt + 2, S0{}, std::false_type{});
  }
  if (kt < nkt) step(kt++, S1{}, std::false_type{});
  if (kt < nkt) step(kt++, S2{}, std::false_type{});

#pragma unroll
  for (int c = 0; c < NQ; ++c) {
    const float lt = xsum4(l_run[c]);
    const float inv = 1.f / lt;
    const int qi = qbase + c * 16 + l15;
    if (qi < T) {
      f16* orow = o + ((size_t)b * T + qi) * ldo + h * 64;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        f16x4v v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (f16)(acc[c][d][r] * inv);
        *reinterpret_cast<f16x4v*>(orow + d * 16 + hq * 4) = v;
      }
    }
  }
}

template <int QW, int NW>
hipError_t run_attn(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad, int ldo,
                    hipStream_t st) {
  constexpr int BQ = QW * NW;
  dim3 grid((T + BQ - 1) / BQ, B * H);
  hipLaunchKernelGGL((attn_fwd_kernel<QW, NW>), grid, dim3(NW * 64), 0, st, reinterpret_cast<const f16*>(q),
                     reinterpret_cast<const f16*>(k), reinterpret_cast<const f16*>(vt), reinterpret_cast<f16*>(o), H,
                     T, Tpad, ldo);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_attention(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad,
                            int ldo, hipStream_t st) {
  if (B <= 0 || T <= 0) return hipSuccess;
  if (Tpad % KT || Tpad < ((T + KT - 1) / KT) * KT || (ldo & 3)) return hipErrorInvalidValue;
  // tuning override: MDE_ATTN_CFG = 32x4 | 16x8 | 16x4 | 16x2 (queries/wave x waves)
  static const int forced = [] {
    const char* e = getenv("MDE_ATTN_CFG");
    if (!e) return 0;
    if (!strcmp(e, "32x4")) return 1;
    if (!strcmp(e, "16x8")) return 2;
    if (!strcmp(e, "16x4")) return 3;
    if (!strcmp(e, "16x2")) return 4;
    return 0;
  }();
  switch (forced) {
    case 1: return run_attn<32, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    case 2: return run_attn<16, 8>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    case 3: return run_attn<16, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    case 4: return run_attn<16, 2>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    default: break;
  }
  // measured on MI355X (tools/bench_kernels.py, T 1370, H 6): 128-query
  // workgroups of 8 waves win once they fill the chip (B 32: 181 us vs 230 us
  // for 64-query groups); at B 1 the 64-query groups fill more CUs (21 vs 23 us)
  const long long g128 = (long long)((T + 127) / 128) * B * H;
  if (g128 >= 256) return run_attn<16, 8>(q, k, vt, o, B, H, T, Tpad, ldo, st);
  return run_attn<16, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
}

}  // namespace mde
