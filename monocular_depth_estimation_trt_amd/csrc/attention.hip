// Fused scaled-dot-product attention, head dim 64, for the DINOv2 blocks
// (reference = TensorRT `_gemm_mha_v2`, restating
// upstream `Attention.forward`: softmax(q*dh^-0.5 @ k^T) @ v).
//
// Layouts (written by the qkv GEMM epilogue, E_QKV):
//   q, k : [B*H][Tpad][64] f16, q pre-multiplied by dh^-0.5 * log2(e), so the
//          scores come out in log2 units and exp() is one v_exp_f32 (exp2)
//   vt   : [B*H][64][Tpad] f16 (v transposed; key t stored at vt_pos(t) = t
//          with bits 2 and 3 swapped, see below), pad columns t >= T zero
//   o    : [B*T][ldo] f16, head h in columns h*64 .. h*64+63
//
// Structure.  A workgroup = NW waves, a wave owns 32 queries, and both
// products run on v_mfma_f32_32x32x16_f16: every K / V^T fragment read from
// LDS feeds 32 queries.  The score tile is computed TRANSPOSED, S^T = K Q^T
// (A = K, 32 keys x 16 dims; B = Q^T), so the query sits on the lane: a lane
// holds 16 keys of one query per 32-key block, lanes l and l+32 the other 16
// -- the row max / sum is a register reduction plus ONE v_permlane32_swap.
// S^T's accumulator is directly the B operand of O^T = V^T P^T: registers
// 8s..8s+7 of a key block are k-step s, whose element j of lane half h is key
// 16s + 8(j>>2) + 4h + (j&3); V^T stores key t at vt_pos(t) (bits 2,3 of t
// swapped) so those 8 keys are one contiguous 16-B read.  K and V^T tiles (64
// keys) stream global -> LDS by global_load_lds through a 2-slot ring (tile
// kt+1 in flight while kt is computed), counted `s_waitcnt vmcnt` + raw
// s_barrier; LDS rows are 128 B with chunk swizzle c ^ ((row >> 1) & 7)
// applied on the source address (conflict-free ds_read_b128 for the 32-row x
// 2-chunk operand reads; SQ_LDS_BANK_CONFLICT = 0 measured).  A 64-key tile
// is two 32-key blocks, each run start to finish (scores, softmax, P.V) so
// one 16-register score accumulator is live.  The running max rides in the
// score MFMA's C operand (S' = QK^T - m), O and l are rescaled only when a
// max grows past a threshold (deferred rescale).  Softmax statistics in fp32;
// keys >= T masked on the last block only.  The epilogue pairs lane halves
// with v_permlane32_swap so each lane stores 16 B of one output row.
//
// Small grids (batch 1: 6 or 16 heads x a few query blocks) split the key
// range.  Default: inside the workgroup -- NS key groups of NW / NS query
// waves, each group streaming its own slice of the key tiles through its own
// ring slots, the groups' (O, m, l) merged through LDS after the loop (ViT-L
// B=1: 2 groups of 128 queries; ViT-S B=1: 4 groups of 64).  Fallback (grids
// too large for that, cfg "4s<n>"): over gridDim.z, each split
// writing its unnormalised fp32 O with its running max and sum for
// attn_combine_kernel to merge.
//
// Large grids (B = 48: 8 waves, unsplit) run attn16_fwd_kernel by default
// (switch "attn16", round 6): the same loop on v_mfma_f32_16x16x32_f16, see
// its comment -- 158 vs 167 us standalone at B = 48, step +0.5-0.9 % in four
// same-box pairs.
//
// Measured alternatives (MI355X, B = 28): two 32-query
// sub-blocks per wave (256 VGPRs), 128-key tiles, one-block software
// pipelining, an 8-wave ping-pong of MFMA / softmax segments and a lagged
// second half (waves 4-7 half a tile behind, carrying the scores across the
// barrier: 155 vs 113 us at 226 VGPRs / one workgroup per CU, and 117-120 vs
// 112-114 us with one loop per wave role at 128 VGPRs / two per CU) were all
// slower than this form; 3- and 4-deep K/V rings (cfg "8r3" / "8r4") measure
// the same as 2 (SQ counters: the waits are issue/dependency stalls, not
// load latency).
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "mde_device.h"
#include "mde_ops.h"
#include "tuning.h"

namespace mde {

namespace {

constexpr int KT = 64;            // keys per tile (and Tpad granularity)
constexpr int TILE_B = KT * 128;  // bytes of one K (or V^T) tile image: 64 rows x 128 B
constexpr int SLOT = 2 * TILE_B;  // K + V^T
constexpr int QW = 32;            // queries per wave (one 32-column MFMA block)
#ifndef ATTN_RING
#define ATTN_RING 2               // K/V^T ring depth (tiles; R-1 in flight while one is computed)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));

MDE_DEV f32x16 mfma32(const f16x8& a, const f16x8& b, const f32x16& c) {
  // D[32x32] += A[32x16] B[16x32]; lane l: A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31];
  // D col l&31, row (r&3) + 8(r>>2) + 4(l>>5) for register r
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Deferred rescale (cdna_hip_programming.md 5.5 T13): the running max moves
// only when a block's max exceeds it by more than RESCALE_T (log2 units), so
// p = exp2(S - m_run) <= 2^RESCALE_T = 256 -- exact in f16's range, and the
// rescale branch (O, l *= 2^-delta) is taken a few times per row, not per block.
constexpr float RESCALE_T = 8.f;

// byte offset of 16-B chunk `chunk` of a 128-B row.  The 32x32x16 operand
// read takes rows r0..r0+31 (lanes 0-31) at chunk c and the same rows at
// chunk c+1 (lanes 32-63); a ds_read_b128 lane group covers rows of both
// parities, and (row >> 1) & 7 spreads each parity's 8 rows over 8 chunks:
// every 16-lane group touches 64 distinct banks
MDE_DEV int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

MDE_DEV float swap_max(float x) {  // max over lanes l and l ^ 32
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MDE_DEV float swap_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
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

MDE_DEV unsigned pack2(float a, float b) {
  typedef f16 f16x2 __attribute__((ext_vector_type(2)));
  const f16x2 h = {(f16)a, (f16)b};
  return __builtin_bit_cast(unsigned, h);
}

// Split-KV partials: per (split, sequence*head, padded query) the
// unnormalised O row (fp32 x 64) and (m, l) in log2 units.
struct SplitWs {
  float* o = nullptr;   // [S][BH][Tq][64]
  float* ml = nullptr;  // [S][BH][Tq][2]
  int Tq = 0;           // padded queries per (b, h): gridDim.x * BQ
  int tiles = 0;        // key tiles per split
};

// Per-lane bytes one wave of a key group > 0 parks for the in-workgroup merge:
// O^T (32 fp32) + (m, l)
constexpr int MERGE_WAVE_B = 64 * 34 * 4;

template <int NW, bool SPLIT, int R, int QS = 1, int NS = 1>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(QS == 2 ? 2 : 4, 8)))
attn_fwd_kernel(const f16* __restrict__ q, const f16* __restrict__ k, const f16* __restrict__ vt,
                f16* __restrict__ o, int H, int T, int Tpad, int ldo, SplitWs ws) {
  // QS = 2: each wave owns two 32-query sub-tiles; every K / V^T fragment
  // read feeds both, and one sub-tile's softmax overlaps the other's MFMAs.
  // NS > 1 (small grids): the workgroup's waves form NS key GROUPS of NW / NS
  // query waves; group g walks the g-th slice of the key tiles for the same
  // queries, each with its own K / V^T ring slots, and the groups' (O, m, l)
  // merge through LDS after the loop -- the split-KV parallelism without the
  // fp32 workspace round trip or a second kernel.
  static_assert(QS == 1 || (QS == 2 && !SPLIT && NS == 1), "query sub-tiles per wave");
  static_assert(NS == 1 || (!SPLIT && R == 2), "key groups");
  constexpr int NWQ = NW / NS;       // query waves per key group
  constexpr int BQ = QW * NWQ * QS;  // queries per workgroup
  constexpr int INS = 8 / NWQ;       // glds instructions per wave per image (8 per 64-row image)
  constexpr int PER_TILE = 2 * INS;  // vmcnt entries one tile adds per wave (K + V^T)
  static_assert(NWQ * NS == NW && (NWQ == 1 || NWQ == 2 || NWQ == 4 || NWQ == 8 || (NWQ == 3 && R == 2)),
                "waves per key group");
  static_assert(NW == 4 || NW == 8 || (NS > 1 && (NW == 6 || NW == 12 || NW == 16)), "waves per workgroup");
  static_assert(R >= 2 && R <= 4, "ring depth");
  constexpr int DIST = R - 1;  // tiles in flight ahead of the one computed
  constexpr int RING_B = R * NS * SLOT, MERGE_B = (NS - 1) * NWQ * MERGE_WAVE_B;
  __shared__ __attribute__((aligned(16))) char smem[RING_B > MERGE_B ? RING_B : MERGE_B];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = NS > 1 ? wave_all / NWQ : 0;   // key group
  const int wave = wave_all - grp * NWQ;         // query wave within the group
  // static priority for the second-dispatched half of the 8-wave workgroup
  // (MI355X_MICROARCH.md "Two waves per SIMD" item 4): round 6, B = 48 graph
  // step +0.5-0.6 % in two same-box pairs (5730 -> 5758 / 5767 img/s,
  // gpurun_out r6s7; round 3 had measured no gain on the older kernel)
  if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);
  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs
  // (linear id % 8 shares an L2); remap so each XCD takes a contiguous run
  // of (head, query block) pairs and a head's K/V^T is fetched into one L2,
  // not eight (PMC: 4.5x the algorithmic bytes without it).  Bijective.
  const int nqb = gridDim.x, nwg = gridDim.x * gridDim.y;
  int lin = blockIdx.y * nqb + blockIdx.x;
  lin = xcd_remap(lin, nwg);
  const int bh = lin / nqb;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int qbase = (lin - bh * nqb) * BQ + wave * QW * QS;
  const bool active = qbase < T;  // wave-uniform: a wave past the last query only helps load
  const int l31 = lane & 31, hh = lane >> 5;

  // key tiles [kt0, kt1) of this workgroup / key group (all of them unless
  // split); every group steps ktl - kt0 times (uniform barrier count)
  const int nkt_all = (T + KT - 1) / KT;
  const int gper = (nkt_all + NS - 1) / NS;  // tiles per key group
  const int kt0 = SPLIT ? (int)blockIdx.z * ws.tiles : grp * gper;
  const int kt1 = SPLIT ? min(nkt_all, kt0 + ws.tiles) : min(nkt_all, kt0 + gper);
  const int ktl = NS > 1 ? kt0 + gper : kt1;

  const f16* qb = q + (size_t)bh * Tpad * 64;
  const f16* kb = k + (size_t)bh * Tpad * 64;
  const f16* vb = vt + (size_t)bh * 64 * Tpad;

  // Q^T fragments (B operand), k-step s = dims 16s..16s+15: lane holds
  // Q[query][16s + 8hh + j] of its query column
  const int qi = qbase + l31;  // sub-tile s: query qi + 32 s
  f16x8 qf[QS][4];
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int st = 0; st < 4; ++st)
      qf[s][st] = qi + 32 * s < Tpad ? *reinterpret_cast<const f16x8*>(qb + (size_t)(qi + 32 * s) * 64 + 16 * st + 8 * hh)
                                     : zero8();

  // glds geometry: lane -> row lrow of an 8-row group, physical chunk lane & 7
  const int lrow = lane >> 3, pc = lane & 7;
  char* const gsm = smem + grp * SLOT;  // this key group's share of each ring slot
  auto issue = [&](int kt, int slot) {
    char* sK = gsm + slot * NS * SLOT;
    char* sV = sK + TILE_B;
#pragma unroll
    for (int i = 0; i < (8 + NWQ - 1) / NWQ; ++i) {
      // 8-row group 0..7: wave w takes w, w + NWQ, ... (3 query waves: 3 / 3 / 2;
      // an uneven count is fine here -- the rings that allow NWQ = 3 wait vmcnt(0))
      const int g = wave + i * NWQ;
      if (8 % NWQ && g >= 8) break;
      const int row = g * 8 + lrow;
      const int lc = pc ^ ((row >> 1) & 7);
      __builtin_amdgcn_global_load_lds(kb + (size_t)(kt * KT + row) * 64 + lc * 8, sK + g * 8 * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(vb + (size_t)row * Tpad + kt * KT + lc * 8, sV + g * 8 * 128, 16, 0, 0);
    }
  };

  // running max (log2 units) as an MFMA C operand: after the first block the
  // score MFMA computes S' = S - m_run directly in the accumulator
  float m_run[QS], l_run[QS];
  f32x16 negm[QS], acc[QS][2];
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    m_run[s] = 0.f;
    l_run[s] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      negm[s][r] = 0.f;
      acc[s][0][r] = 0.f;
      acc[s][1][r] = 0.f;
    }
  }

  // wait until tile `kt` has landed, given the tiles issued after it: at
  // most `after` more tiles (0 .. DIST-1) may stay in flight
  auto wait_tiles = [&](int after) {
    if (DIST > 2 && after >= 2) wait_vm_n<(DIST > 2 ? 2 : 0) * PER_TILE>();
    else if (DIST > 1 && after >= 1) wait_vm_n<(DIST > 1 ? 1 : 0) * PER_TILE>();
    else wait_vm_n<0>();
  };
  // prologue: DIST tiles in flight, then tile kt0 landed
#pragma unroll
  for (int i = 0; i < DIST; ++i)
    if (kt0 + i < kt1) issue(kt0 + i, i);
  wait_tiles(min(kt1, kt0 + DIST) - 1 - kt0);
  lds_barrier();

  // S'^T[key][query] = K Q^T - m_run over the 32 keys of block kb2 of tile
  // kt (4 dim k-steps), for every query sub-tile (each K fragment read once);
  // keys >= T -> -inf
  struct Scores {
    f32x16 v[QS];
  };
  auto scores = [&](const char* K_, int kt, int kb2, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    Scores sc;
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      if constexpr (FIRST) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc.v[s][r] = 0.f;
      } else {
        sc.v[s] = negm[s];
      }
    }
    const int krow = kb2 * 32 + l31;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const f16x8 kf = *reinterpret_cast<const f16x8*>(K_ + swz(krow, 2 * st + hh));
#pragma unroll
      for (int s = 0; s < QS; ++s) sc.v[s] = mfma32(kf, qf[s][st], sc.v[s]);
    }
    if (kt * KT + kb2 * 32 + 32 > T) {  // last, partial block
      const int key0 = kt * KT + kb2 * 32 + 4 * hh;
#pragma unroll
      for (int s = 0; s < QS; ++s)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (key0 + (r & 3) + 8 * (r >> 2) >= T) sc.v[s][r] = -INFINITY;
    }
    return sc;
  };
  // online-softmax update and P.V of sub-tile S whose scores are sc (V_ =
  // the V^T image of the block's tile)
  auto softmax_pv = [&](auto s_tag, f32x16 sc, const char* V_, int kb2, auto first_tag) {
    constexpr int S = decltype(s_tag)::value;
    constexpr bool FIRST = decltype(first_tag)::value;
    // the lane's max over its 16 scores (v_max3 chain); the row max (partner
    // lane l ^ 32) only when some row rescales
    float mx = fmaxf(sc[0], sc[1]);
#pragma unroll
    for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, sc[r]), sc[r + 1]);
    if (FIRST || __any(mx > RESCALE_T)) {
      mx = swap_max(mx);  // max of S' over the block (relative to m_run)
      // the running max grows by delta >= 0: shift S', rescale O and l
      const float delta = FIRST ? mx : fmaxf(mx, 0.f);
      m_run[S] += delta;
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[S][r] = -m_run[S];
      sc -= delta;
      if (!FIRST) {
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        l_run[S] *= alpha;
        acc[S][0] *= alpha;
        acc[S][1] *= alpha;
      }
    }
    // P = exp2(S'), row sums, and P^T as the PV B operand: registers
    // 8s..8s+7 are k-step s (keys 16s + 8(j>>2) + 4hh + (j&3))
    f16x8 pb[2];
    float ls0, ls1;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const float p0 = __builtin_amdgcn_exp2f(sc[r]), p1 = __builtin_amdgcn_exp2f(sc[r + 1]);
      ls0 = r ? ls0 + p0 : p0;
      ls1 = r ? ls1 + p1 : p1;
      pb[r >> 3][r & 7] = (f16)p0;
      pb[r >> 3][(r & 7) + 1] = (f16)p1;
    }
    l_run[S] += ls0 + ls1;
    // O^T[dh][q] += V^T[dh][key] P^T[key][q]: two 32-row dh blocks x 2 key k-steps
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int vrow = db * 32 + l31;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const f16x8 vf = *reinterpret_cast<const f16x8*>(V_ + swz(vrow, 2 * (2 * kb2 + g) + hh));
        acc[S][db] = mfma32(vf, pb[g], acc[S][db]);
      }
    }
  };
  using NF = std::false_type;
  // the two blocks of tile kt, in order
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, QS - 1>;
  auto tile = [&](int kt, auto slot_tag, auto first_tag) {
    constexpr int slot = decltype(slot_tag)::value;  // compile-time: LDS offsets fold into ds_read immediates
    const char* K_ = gsm + slot * NS * SLOT;
    {
      const Scores sc = scores(K_, kt, 0, first_tag);
      softmax_pv(Q0{}, sc.v[0], K_ + TILE_B, 0, first_tag);
      if constexpr (QS == 2) softmax_pv(Q1{}, sc.v[QS - 1], K_ + TILE_B, 0, first_tag);
    }
    {
      const Scores sc = scores(K_, kt, 1, NF{});
      softmax_pv(Q0{}, sc.v[0], K_ + TILE_B, 1, NF{});
      if constexpr (QS == 2) softmax_pv(Q1{}, sc.v[QS - 1], K_ + TILE_B, 1, NF{});
    }
  };

  // tile kt lives in ring slot (kt - kt0) % R; the loop is unrolled over the
  // R slots so every LDS address is lane base + immediate.  Step kt issues
  // tile kt+DIST into the slot of tile kt-1 (released by the previous
  // barrier), computes tile kt, and waits -- counted, leaving the newer
  // tiles in flight -- for tile kt+1 before the barrier that ends the step.
  auto step = [&](int kt, auto slot_tag, auto first_tag) {
    constexpr int SL = decltype(slot_tag)::value;
    if (kt + DIST < kt1) issue(kt + DIST, (SL + DIST) % R);
    if (active && (NS == 1 || kt < kt1)) tile(kt, slot_tag, first_tag);
    wait_tiles(min(kt1 - 1, kt + DIST) - (kt + 1));
    lds_barrier();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1 % R>;
  using S2 = std::integral_constant<int, 2 % R>;
  using S3 = std::integral_constant<int, 3 % R>;
  step(kt0, S0{}, std::true_type{});
  int kt = kt0 + 1;
  for (; kt + R <= ktl; kt += R) {
    step(kt, S1{}, NF{});
    step(kt + 1, S2{}, NF{});
    if constexpr (R > 2) step(kt + 2, S3{}, NF{});
    if constexpr (R > 3) step(kt + 3, S0{}, NF{});
  }
  if (kt < ktl) step(kt, S1{}, NF{});
  if (R > 2 && kt + 1 < ktl) step(kt + 1, S2{}, NF{});
  if (R > 3 && kt + 2 < ktl) step(kt + 2, S3{}, NF{});

  if constexpr (NS > 1) {
    // merge the key groups: groups 1.. park (O^T, m, l) in LDS (the ring is
    // free: every wave's last LDS read came before the last step's barrier,
    // and that step waited out every load), group 0 rescales to the common
    // max and sums.  Lane layout is identical across groups (same queries).
    // An empty group (kt0 >= nkt_all: tiny T) is skipped.
    float* mb = reinterpret_cast<float*>(smem);
    if (grp > 0) {
      float* w = mb + ((grp - 1) * NWQ + wave) * (MERGE_WAVE_B / 4);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const f32x16& a = acc[0][c >> 2];
        *reinterpret_cast<float4*>(w + (c * 64 + lane) * 4) =
            make_float4(a[4 * (c & 3)], a[4 * (c & 3) + 1], a[4 * (c & 3) + 2], a[4 * (c & 3) + 3]);
      }
      *reinterpret_cast<float2*>(w + 8 * 64 * 4 + lane * 2) = make_float2(m_run[0], l_run[0]);
    }
    __syncthreads();
    if (grp > 0) return;
    float mg[NS];
    mg[0] = m_run[0];
    float mmax = m_run[0];
#pragma unroll
    for (int g = 1; g < NS; ++g) {
      const float* w = mb + ((g - 1) * NWQ + wave) * (MERGE_WAVE_B / 4);
      mg[g] = w[8 * 64 * 4 + lane * 2];
      if (g * gper < nkt_all) mmax = fmaxf(mmax, mg[g]);
    }
    const float a0 = __builtin_amdgcn_exp2f(m_run[0] - mmax);
    l_run[0] *= a0;
    acc[0][0] *= a0;
    acc[0][1] *= a0;
#pragma unroll
    for (int g = 1; g < NS; ++g) {
      if (g * gper >= nkt_all) continue;  // wave-uniform
      const float* w = mb + ((g - 1) * NWQ + wave) * (MERGE_WAVE_B / 4);
      const float ag = __builtin_amdgcn_exp2f(mg[g] - mmax);
      l_run[0] += ag * w[8 * 64 * 4 + lane * 2 + 1];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(w + (c * 64 + lane) * 4);
        acc[0][c >> 2][4 * (c & 3)] += ag * v.x;
        acc[0][c >> 2][4 * (c & 3) + 1] += ag * v.y;
        acc[0][c >> 2][4 * (c & 3) + 2] += ag * v.z;
        acc[0][c >> 2][4 * (c & 3) + 3] += ag * v.w;
      }
    }
  }
  if (!active) return;

  if constexpr (SPLIT) {
    // unnormalised O^T (relative to m_run) and (m, l) of this key range
    const float lt = swap_sum(l_run[0]);
    const size_t row = ((size_t)blockIdx.z * gridDim.y + bh) * ws.Tq + qi;
    float* orow = ws.o + row * 64;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<float4*>(orow + 32 * db + 8 * g4 + 4 * hh) =
            make_float4(acc[0][db][4 * g4], acc[0][db][4 * g4 + 1], acc[0][db][4 * g4 + 2], acc[0][db][4 * g4 + 3]);
    if (hh == 0) *reinterpret_cast<float2*>(ws.ml + row * 2) = make_float2(m_run[0], lt);
    return;
  }

  // epilogue: lane holds O^T[dh = 32 db + (r&3) + 8(r>>2) + 4hh][qi]; pair
  // register groups (r>>2) = 2pr, 2pr+1 across the lane halves
  // (v_permlane32_swap) so each lane stores dh 16pr + 8hh .. +7 as one 16-B write
#pragma unroll
  for (int sq = 0; sq < QS; ++sq) {
    const float inv = 1.f / swap_sum(l_run[sq]);
    uint4 out[2][2];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int r0 = 8 * pr;  // group 2pr: registers r0..r0+3, group 2pr+1: r0+4..r0+7
        const f32x16& a = acc[sq][db];
        const unsigned ax = pack2(a[r0] * inv, a[r0 + 1] * inv);
        const unsigned ay = pack2(a[r0 + 2] * inv, a[r0 + 3] * inv);
        const unsigned bx = pack2(a[r0 + 4] * inv, a[r0 + 5] * inv);
        const unsigned by = pack2(a[r0 + 6] * inv, a[r0 + 7] * inv);
        auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
        auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
        out[db][pr] = make_uint4(sx[0], sy[0], sx[1], sy[1]);
      }
    const int qs = qi + 32 * sq;
    if (qs < T) {
      f16* orow = o + ((size_t)b * T + qs) * ldo + h * 64 + 8 * hh;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) *reinterpret_cast<uint4*>(orow + db * 32 + 16 * pr) = out[db][pr];
    }
  }
}

// ---- The same loop on v_mfma_f32_16x16x32_f16 (switch "attn16", cfg "<NW>m") ----
//
// Per 32-key block and 32-query wave the work is that of attn_fwd_kernel --
// 256 cycles of matrix pipe, 16 v_exp per lane, the same LDS reads -- but
// the products are 8 + 8 MFMAs of 16 cycles with at most two dependent ones
// per accumulator (the 32x32x16 form chains four 32-cycle MFMAs per score
// tile): the score -> softmax -> P.V chain of a block is shorter, and the
// smaller shape is the one MI355X_MICROARCH.md (DVFS item 7) measured
// holding a higher clock under load.  Layout per wave: two query sub-tiles of
// 16 (s), two key sub-tiles of 16 per block (t); lane l holds query
// 16 s + (l & 15) and, of key sub-tile t, keys 8 t + 16 (g >> 1) + 4 (g & 1)
// + r (g = l >> 4, r = 0..3) -- the K rows are fed to the score MFMA's A
// operand in that order, so the accumulators of t = 0, 1 are directly the
// P^T B operand of the P.V MFMA against the unchanged V^T layout (vt_pos).
// The running max rides in the score C operand (one 4-register copy per
// query sub-tile serves both key sub-tiles); a query's keys sit in four lane
// groups, so the rare rescale's row max reduces with v_permlane32_swap +
// v_permlane16_swap; the row sums come from two more MFMAs with an all-ones
// A operand (below).
MDE_DEV int swz16(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

MDE_DEV float grp4_max(float x) {  // max over lanes (l & 15) + 16 g, g = 0..3
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto c = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(c[0]), __uint_as_float(c[1]));
}

// Per-lane floats one wave of a key group > 0 parks for the merge: O^T (32), m (2), l (2)
constexpr int MERGE16_WAVE_B = 64 * 36 * 4;

// LDS of the body below: the K / V^T ring, or (key groups) the merge area
template <int NW, int NS>
constexpr int attn16_smem() {
  constexpr int NWQ = NW / NS;
  constexpr int RING_B = 2 * NS * SLOT, MERGE_B = (NS - 1) * NWQ * MERGE16_WAVE_B;
  return RING_B > MERGE_B ? RING_B : MERGE_B;
}

// One workgroup's queries [qblk * BQ, +BQ) of sequence x head bh (the
// kernel below picks bh / qblk).
// NS > 1 (batch-1 grids, and the partial blocks of attn_tail = 2): NS key
// groups of NW / NS query waves, as in attn_fwd_kernel -- each group streams
// its slice of the key tiles through its own ring slots, (O, m, l) merged
// through LDS after the loop
template <int NW, int NS>
MDE_DEV void attn16_body(const f16* __restrict__ q, const f16* __restrict__ k, const f16* __restrict__ vt,
                         f16* __restrict__ o, int H, int T, int Tpad, int ldo, char* smem, int bh, int qblk) {
  constexpr int NWQ = NW / NS;  // query waves per key group
  static_assert(NWQ * NS == NW && (NWQ == 2 || NWQ == 4 || NWQ == 8) && (NW == 4 || NW == 8), "waves");
  constexpr int BQ = QW * NWQ;
  constexpr int INS = 8 / NWQ;  // glds row groups per wave per 64-row image

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = NS > 1 ? wave_all / NWQ : 0;
  const int wave = wave_all - grp * NWQ;
  if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);
  const int b = bh / H, h = bh - (bh / H) * H;
  const int qbase = qblk * BQ + wave * QW;
  const bool active = qbase < T;
  const int l15 = lane & 15, g = lane >> 4;
  const int nkt_all = (T + KT - 1) / KT;
  const int gper = (nkt_all + NS - 1) / NS;  // key tiles per group
  const int kt0 = grp * gper, kt1 = min(nkt_all, kt0 + gper), ktl = kt0 + gper;

  const f16* qb = q + (size_t)bh * Tpad * 64;
  const f16* kb = k + (size_t)bh * Tpad * 64;
  const f16* vb = vt + (size_t)bh * 64 * Tpad;

  // Q^T (B operand) of sub-tile s, dim step d: lane holds Q[16 s + l15][32 d + 8 g + j]
  f16x8 qf[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int qi = qbase + 16 * s + l15;
#pragma unroll
    for (int d = 0; d < 2; ++d)
      qf[s][d] = qi < Tpad ? *reinterpret_cast<const f16x8*>(qb + (size_t)qi * 64 + 32 * d + 8 * g) : zero8();
  }

  const int lrow = lane >> 3, pc = lane & 7;
  char* const gsm = smem + grp * SLOT;  // this key group's share of each ring slot
  auto issue = [&](int kt, int slot) {
    char* sK = gsm + slot * NS * SLOT;
    char* sV = sK + TILE_B;
#pragma unroll
    for (int i = 0; i < INS; ++i) {
      const int gg = wave + i * NWQ;  // 8-row group
      const int row = gg * 8 + lrow;
      const int lc = pc ^ lrow;      // swz16: row & 7 == lrow
      __builtin_amdgcn_global_load_lds(kb + (size_t)(kt * KT + row) * 64 + lc * 8, sK + gg * 8 * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(vb + (size_t)row * Tpad + kt * KT + lc * 8, sV + gg * 8 * 128, 16, 0, 0);
    }
  };

  float m_run[2] = {0.f, 0.f};
  f32x4 negm[2], acc[4][2], lacc[2];  // lacc: the row sums, of the f16 P, by MFMA
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    negm[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    lacc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // K row (within the 64-key tile) that A-operand row l15 of key sub-tile t of block kb2 reads
  const int krow0 = ((l15 >> 3) << 4) + (l15 & 7);

  struct Sc16 {
    f32x4 v[2][2];  // [t][s]: S'^T = K Q^T - m_run
  };
  auto scores = [&](const char* K_, int kt, int kb2, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    Sc16 sc;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) sc.v[t][s] = FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : negm[s];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(K_ + swz16(kb2 * 32 + 8 * t + krow0, 4 * d + g));
#pragma unroll
        for (int s = 0; s < 2; ++s) sc.v[t][s] = mfma16x16x32(kf, qf[s][d], sc.v[t][s]);
      }
    return sc;
  };
  // keys >= T -> -inf (last, partial block; a separate step so the branch
  // does not cut the score MFMAs off the code they are scheduled with)
  auto mask = [&](Sc16& sc, int kt, int kb2) {
    if (kt * KT + kb2 * 32 + 32 > T) {
      const int key0 = kt * KT + kb2 * 32 + 16 * (g >> 1) + 4 * (g & 1);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (key0 + 8 * t + r >= T) {
            sc.v[t][0][r] = -INFINITY;
            sc.v[t][1][r] = -INFINITY;
          }
    }
  };
  // online softmax of one block's scores: the running max (rescale when it
  // grows past RESCALE_T), then P = exp2(S') as the P.V B operand and the row sums
  struct Pb16 {
    f16x8 v[2];
  };
  // pend: probabilities computed against the old max whose P.V is still to
  // come (block 0's, issued under block 1's exp2 chain) -- scaled with O
  auto rescale = [&](Sc16& sc, auto first_tag, Pb16* pend) {
    constexpr bool FIRST = decltype(first_tag)::value;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float mx = fmaxf(fmaxf(sc.v[0][s][0], sc.v[0][s][1]), sc.v[0][s][2]);
      mx = fmaxf(fmaxf(mx, sc.v[0][s][3]), sc.v[1][s][0]);
      mx = fmaxf(fmaxf(mx, sc.v[1][s][1]), sc.v[1][s][2]);
      mx = fmaxf(mx, sc.v[1][s][3]);
      if (FIRST || __any(mx > RESCALE_T)) {
        mx = grp4_max(mx);  // the query's block max (relative to m_run)
        const float delta = FIRST ? mx : fmaxf(mx, 0.f);
        m_run[s] += delta;
        negm[s] = f32x4{-m_run[s], -m_run[s], -m_run[s], -m_run[s]};
        sc.v[0][s] -= delta;
        sc.v[1][s] -= delta;
        if (!FIRST) {
          const float alpha = __builtin_amdgcn_exp2f(-delta);
          lacc[s] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) acc[dt][s] *= alpha;
          if (pend) {
            const f16 ah = (f16)alpha;
#pragma unroll
            for (int j = 0; j < 8; ++j) pend->v[s][j] *= ah;
          }
        }
      }
    }
  };
  auto probs = [&](const Sc16& sc) {
    Pb16 pb;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb.v[s][r] = (f16)__builtin_amdgcn_exp2f(sc.v[0][s][r]);
        pb.v[s][4 + r] = (f16)__builtin_amdgcn_exp2f(sc.v[1][s][r]);
      }
    }
    return pb;
  };
  // O^T[16 dt + 4 g + r][query] += V^T[16 dt + l15][key slot 32 kb2 + 8 g + j] P^T
  auto pv = [&](const Pb16& pb, const char* V_, int kb2) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f16x8 vf = *reinterpret_cast<const f16x8*>(V_ + swz16(16 * dt + l15, 4 * kb2 + g));
#pragma unroll
      for (int s = 0; s < 2; ++s) acc[dt][s] = mfma16x16x32(vf, pb.v[s], acc[dt][s]);
    }
    // row sums: an all-ones A operand makes every row of D the query's sum of
    // its 32 f16 probabilities -- the same P the numerator used -- in place of
    // 16 fp32 adds per lane and the final cross-lane sum (2 MFMAs, 16 cycles each)
    f16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (f16)1.0f;
#pragma unroll
    for (int s = 0; s < 2; ++s) lacc[s] = mfma16x16x32(ones, pb.v[s], lacc[s]);
  };
  using NF = std::false_type;
  auto step = [&](int kt, auto slot_tag, auto first_tag) {
    constexpr int SL = decltype(slot_tag)::value;
    if (kt + 1 < kt1) issue(kt + 1, SL ^ 1);  // into the slot of tile kt - 1 (released by the last barrier)
    // two overlapped phases per tile: block 1's score MFMAs (against the
    // updated max) beside block 0's exp2 chain, then block 0's P.V MFMAs
    // beside block 1's exp2 chain (a rescale in between scales block 0's
    // pending P with O).  (A copy of the tile body without the masking
    // branches for the full tiles measured no faster, r6s25.)
    if (active && kt < kt1) {
      const char* K_ = gsm + SL * NS * SLOT;
      Sc16 s0 = scores(K_, kt, 0, first_tag);
      mask(s0, kt, 0);
      rescale(s0, first_tag, nullptr);
      Sc16 s1 = scores(K_, kt, 1, NF{});
      mask(s1, kt, 1);
      Pb16 p0 = probs(s0);
      rescale(s1, NF{}, &p0);
      pv(p0, K_ + TILE_B, 0);
      const Pb16 p1 = probs(s1);
      pv(p1, K_ + TILE_B, 1);
    }
    wait_vm_n<0>();
    lds_barrier();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (kt0 < kt1) issue(kt0, 0);
  wait_vm_n<0>();
  lds_barrier();
  step(kt0, S0{}, std::true_type{});
  int kt = kt0 + 1;
  for (; kt + 2 <= ktl; kt += 2) {
    step(kt, S1{}, NF{});
    step(kt + 1, S0{}, NF{});
  }
  if (kt < ktl) step(kt, S1{}, NF{});

  if constexpr (NS > 1) {
    // merge: groups 1.. park (O^T, m, l) in LDS (the ring is free: the last
    // step waited out every load and its barrier every read), group 0
    // rescales to the common max and sums; lane layouts match across groups
    float* mb = reinterpret_cast<float*>(smem);
    if (grp > 0) {
      float* w = mb + ((grp - 1) * NWQ + wave) * (MERGE16_WAVE_B / 4);
#pragma unroll
      for (int c = 0; c < 8; ++c) *reinterpret_cast<f32x4*>(w + (c * 64 + lane) * 4) = acc[c >> 1][c & 1];
      *reinterpret_cast<f32x4*>(w + 8 * 64 * 4 + lane * 4) = f32x4{m_run[0], m_run[1], lacc[0][0], lacc[1][0]};
    }
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float mmax = m_run[s];
#pragma unroll
      for (int gr = 1; gr < NS; ++gr)
        if (gr * gper < nkt_all)
          mmax = fmaxf(mmax, mb[((gr - 1) * NWQ + wave) * (MERGE16_WAVE_B / 4) + 8 * 64 * 4 + lane * 4 + s]);
      const float a0 = __builtin_amdgcn_exp2f(m_run[s] - mmax);
      lacc[s] *= a0;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt][s] *= a0;
#pragma unroll
      for (int gr = 1; gr < NS; ++gr) {
        if (gr * gper >= nkt_all) continue;  // an empty group (tiny T)
        const float* w = mb + ((gr - 1) * NWQ + wave) * (MERGE16_WAVE_B / 4);
        const f32x4 ml = *reinterpret_cast<const f32x4*>(w + 8 * 64 * 4 + lane * 4);
        const float ag = __builtin_amdgcn_exp2f(ml[s] - mmax);
        lacc[s][0] += ag * ml[2 + s];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) acc[dt][s] += ag * *reinterpret_cast<const f32x4*>(w + ((2 * dt + s) * 64 + lane) * 4);
      }
    }
  }
  if (!active) return;

  // epilogue: lane holds O^T[16 dt + 4 g + r][16 s + l15]; lane groups g, g ^ 1
  // exchange (v_permlane16_swap) so each lane stores 8 consecutive dh (16 B)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float inv = 1.f / lacc[s][0];
    const int qs = qbase + 16 * s + l15;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const f32x4 a = acc[2 * p][s], c = acc[2 * p + 1][s];
      const unsigned ax = pack2(a[0] * inv, a[1] * inv), ay = pack2(a[2] * inv, a[3] * inv);
      const unsigned cx = pack2(c[0] * inv, c[1] * inv), cy = pack2(c[2] * inv, c[3] * inv);
      auto sx = __builtin_amdgcn_permlane16_swap(ax, cx, false, false);
      auto sy = __builtin_amdgcn_permlane16_swap(ay, cy, false, false);
      if (qs < T)
        *reinterpret_cast<uint4*>(o + ((size_t)b * T + qs) * ldo + h * 64 + 32 * p + 16 * (g & 1) + 8 * (g >> 1)) =
            make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
  }
}

template <int NW, int NS>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4, 8)))
attn16_fwd_kernel(const f16* __restrict__ q, const f16* __restrict__ k, const f16* __restrict__ vt,
                  f16* __restrict__ o, int H, int T, int Tpad, int ldo, int tail_last) {
  // attn_tail = 2 (8 waves, unsplit): a partial last block of at most 128
  // queries runs as two key groups of 4 query waves (the <8, 2> body) instead
  // of 3 active waves of 8 over all keys
  constexpr bool KTAIL = NW == 8 && NS == 1;
  constexpr int SM0 = attn16_smem<NW, NS>(), SM1 = KTAIL ? attn16_smem<8, 2>() : 0;
  __shared__ __attribute__((aligned(16))) char smem[SM0 > SM1 ? SM0 : SM1];
  constexpr int BQ = QW * (NW / NS);
  const int nqb = gridDim.x;
  // work order: XCD-remapped (bh, query block), or (tail_last, switch
  // "attn_tail") every sequence's partial last query block dispatched after
  // all full ones -- the grid's last, partly filled round then holds the
  // blocks with idle query waves, which run shorter
  const int id = blockIdx.y * nqb + blockIdx.x;
  const int full = (nqb - 1) * (int)gridDim.y;
  int bh, qblk;
  if (NS == 1 && tail_last && nqb > 1 && T % BQ != 0) {
    if (id < full) {
      const int l = xcd_remap(id, full);
      bh = l / (nqb - 1);
      qblk = l - bh * (nqb - 1);
    } else {
      // each XCD's partial blocks in reverse head order: the heads whose
      // full blocks it ran last come first, their K / V^T tiles still in its L2
      const int u = id - full, nh = (int)gridDim.y, x = u & 7, q8 = nh >> 3, r8 = nh & 7;
      const int size = q8 + (x < r8 ? 1 : 0);
      const int start = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
      bh = start + size - 1 - (u >> 3);
      qblk = nqb - 1;
    }
  } else {
    const int lin = xcd_remap(id, nqb * gridDim.y);
    bh = lin / nqb;
    qblk = lin - bh * nqb;
  }
  if constexpr (KTAIL) {
    if (tail_last == 2 && qblk == nqb - 1 && T - qblk * BQ <= BQ / 2 && (T + KT - 1) / KT >= 2) {
      attn16_body<8, 2>(q, k, vt, o, H, T, Tpad, ldo, smem, bh, qblk * 2);
      return;
    }
  }
  attn16_body<NW, NS>(q, k, vt, o, H, T, Tpad, ldo, smem, bh, qblk);
}

// Merge S split-KV partials: one thread per (sequence*head, query, 8 dims).
// O = sum_s 2^(m_s - m) O_s / sum_s 2^(m_s - m) l_s, m = max_s m_s.
__global__ void __launch_bounds__(256) attn_combine_kernel(SplitWs ws, int S, int BH, int H, int T, int ldo,
                                                           f16* __restrict__ o) {
  const int id = blockIdx.x * 256 + threadIdx.x;
  const int d8 = id & 7, rest = id >> 3;
  const int qi = rest % T, bh = rest / T;
  if (bh >= BH) return;
  float m = -INFINITY;
  for (int s = 0; s < S; ++s) m = fmaxf(m, ws.ml[(((size_t)s * BH + bh) * ws.Tq + qi) * 2]);
  float lsum = 0.f, acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int s = 0; s < S; ++s) {
    const size_t row = ((size_t)s * BH + bh) * ws.Tq + qi;
    const float2 ml = *reinterpret_cast<const float2*>(ws.ml + row * 2);
    const float w = __builtin_amdgcn_exp2f(ml.x - m);
    lsum += w * ml.y;
    const float4 a = *reinterpret_cast<const float4*>(ws.o + row * 64 + 8 * d8);
    const float4 c = *reinterpret_cast<const float4*>(ws.o + row * 64 + 8 * d8 + 4);
    acc[0] += w * a.x;
    acc[1] += w * a.y;
    acc[2] += w * a.z;
    acc[3] += w * a.w;
    acc[4] += w * c.x;
    acc[5] += w * c.y;
    acc[6] += w * c.z;
    acc[7] += w * c.w;
  }
  const float inv = 1.f / lsum;
  f16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (f16)(acc[j] * inv);
  const int b = bh / H, h = bh - b * H;
  *reinterpret_cast<f16x8*>(o + ((size_t)b * T + qi) * ldo + h * 64 + 8 * d8) = v;
}

template <int NW, int R, int QS = 1>
hipError_t run_attn(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad, int ldo,
                    float* ws, size_t ws_bytes, int split, hipStream_t st) {
  constexpr int BQ = QW * NW * QS;
  const int nqb = (T + BQ - 1) / BQ, nkt = (T + KT - 1) / KT;
  const auto cq = reinterpret_cast<const f16*>(q);
  const auto ck = reinterpret_cast<const f16*>(k);
  const auto cv = reinterpret_cast<const f16*>(vt);
  const auto co = reinterpret_cast<f16*>(o);
  if (QS == 1 && split > 1 && ws) {
    SplitWs w;
    w.Tq = nqb * BQ;
    w.tiles = (nkt + split - 1) / split;
    const int S = (nkt + w.tiles - 1) / w.tiles;  // every split non-empty
    const size_t rows = (size_t)S * B * H * w.Tq;
    if (S > 1 && rows * 66 * sizeof(float) <= ws_bytes) {
      w.o = ws;
      w.ml = ws + rows * 64;
      hipLaunchKernelGGL((attn_fwd_kernel<NW, true, R, 1>), dim3(nqb, B * H, S), dim3(NW * 64), 0, st, cq, ck, cv, co, H, T,
                         Tpad, ldo, w);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      const long long n = (long long)B * H * T * 8;
      hipLaunchKernelGGL(attn_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, S, B * H, H, T,
                         ldo, co);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((attn_fwd_kernel<NW, false, R, QS>), dim3(nqb, B * H), dim3(NW * 64), 0, st, cq, ck, cv, co, H, T, Tpad,
                     ldo, SplitWs{});
  return hipGetLastError();
}

// NS key groups of NW / NS query waves in each workgroup (in-workgroup split-KV)
template <int NW, int NS>
hipError_t run_attn_grp(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad, int ldo,
                        hipStream_t st) {
  constexpr int BQ = QW * (NW / NS);
  const int nqb = (T + BQ - 1) / BQ;
  hipLaunchKernelGGL((attn_fwd_kernel<NW, false, 2, 1, NS>), dim3(nqb, B * H), dim3(NW * 64), 0, st,
                     reinterpret_cast<const f16*>(q), reinterpret_cast<const f16*>(k), reinterpret_cast<const f16*>(vt),
                     reinterpret_cast<f16*>(o), H, T, Tpad, ldo, SplitWs{});
  return hipGetLastError();
}

template <int NW, int NS = 1>
hipError_t run_attn16(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad, int ldo,
                      hipStream_t st) {
  constexpr int BQ = QW * (NW / NS);
  const int nqb = (T + BQ - 1) / BQ;
  hipLaunchKernelGGL((attn16_fwd_kernel<NW, NS>), dim3(nqb, B * H), dim3(NW * 64), 0, st, reinterpret_cast<const f16*>(q),
                     reinterpret_cast<const f16*>(k), reinterpret_cast<const f16*>(vt), reinterpret_cast<f16*>(o), H, T,
                     Tpad, ldo, knob(KNOB_ATTN_TAIL));
  return hipGetLastError();
}

}  // namespace

size_t attention_split_ws_bytes(int B, int H, int T) {
  // the largest split the launcher picks: 8 ways over 128-query workgroups
  const size_t tq = (size_t)(T + 127) / 128 * 128;
  return (size_t)8 * B * H * tq * 66 * sizeof(float);
}

hipError_t launch_attention(const h16* q, const h16* k, const h16* vt, h16* o, int B, int H, int T, int Tpad,
                            int ldo, hipStream_t st, float* ws, size_t ws_bytes, const char* cfg) {
  if (B <= 0 || T <= 0) return hipSuccess;
  // the 16-B output stores need ldo % 8 == 0 (and a 16-B aligned o)
  if (Tpad % KT || Tpad < ((T + KT - 1) / KT) * KT || (ldo & 7) || ((uintptr_t)o & 15)) return hipErrorInvalidValue;
  const int nkt = (T + KT - 1) / KT;
  // cfg = <waves>[s<split>][g<groups>][r<ring>][q2] ("8", "4", "4s8", "8r3", ...):
  // a forced launch shape (mde_op_attention_cfg: tests, tuning)
  const char* forced = cfg && cfg[0] ? cfg : nullptr;
  int nw = 0, split = 1, ring = ATTN_RING, qs2 = 0, groups = 1, m16 = 0;
  if (forced) {
    nw = atoi(forced);
    m16 = strchr(forced, 'm') != nullptr;  // "<waves>m": the 16x16x32 kernel (attn16_fwd_kernel)
    const char* sp = strchr(forced, 's');
    split = sp ? atoi(sp + 1) : 1;
    const char* rp = strchr(forced, 'r');
    if (rp) ring = atoi(rp + 1);
    qs2 = strstr(forced, "q2") != nullptr;
    const char* gp = strchr(forced, 'g');  // "<waves>g<groups>": in-workgroup key groups
    if (gp) groups = atoi(gp + 1);
  }
  if (nw != 4 && nw != 8 && !(groups > 1 && (nw == 6 || nw == 12 || nw == 16))) {
    // 256-query workgroups share each K/V^T tile over 8 waves once the grid
    // fills the chip (2 per CU); smaller grids take 128-query groups and,
    // below one group per CU, split the keys -- at least 7 key tiles per
    // split and at most ~400 workgroups (batch 1: ViT-S 3 splits, 0.932 ->
    // 0.923 ms per forward vs 4; ViT-L 2, vs 4: 3.70 -> 3.67 ms)
    const long long g256 = (long long)((T + 255) / 256) * B * H;
    const long long g128 = (long long)((T + 127) / 128) * B * H;
    nw = g256 >= 512 ? 8 : 4;
    split = 1;
    if (nw == 4 && g128 < 256)
      while (split < 8 && nkt >= 7 * (split + 1) && g128 * (split + 1) <= 400) ++split;
    // the split runs as key groups inside 8-wave workgroups, merged through
    // LDS (no fp32 partials, no combine launch): two groups of 128 queries
    // (64 KB LDS, two workgroups per CU) for a two-way split -- ViT-L 518^2
    // B=1 3.52 -> 3.38 ms per forward --, four groups of 64 queries (128 KB,
    // one per CU) when that grid fits the CUs -- ViT-S B=1 0.890 -> 0.859 ms
    // (same box, profiles/r03_v5_*)
    const long long g64 = (long long)((T + 63) / 64) * B * H;
    if (nw == 4 && split >= 3 && g64 <= 256 && nkt >= 4) {
      nw = 8;
      split = 1;
      groups = 4;
    } else if (nw == 4 && split == 2) {
      nw = 8;
      split = 1;
      groups = 2;
    }
  }
  // (the key-group form, cfg "8g2m" / "8g4m", measured 3 % slower than the
  // 32x32x16 one at batch 1: ViT-L 17.4-17.9 vs 16.9-17.4 us, ViT-S 12.4-12.7
  // vs 12.1-12.4, gpurun_out r6s24 -- the switch covers the unsplit shape only)
  if (!forced && nw == 8 && groups == 1 && split <= 1) m16 = knob(KNOB_ATTN16);
  if (m16 && groups > 1 && nkt >= groups && nw == 8 && split <= 1 && !qs2) {
    if (groups == 2) return run_attn16<8, 2>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (groups == 4) return run_attn16<8, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
  }
  if (m16 && groups == 1 && split <= 1 && !qs2) {
    if (nw == 8) return run_attn16<8>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 4) return run_attn16<4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
  }
  if (groups > 1 && nkt >= groups) {
    if (nw == 4 && groups == 2) return run_attn_grp<4, 2>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 4 && groups == 4) return run_attn_grp<4, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 8 && groups == 2) return run_attn_grp<8, 2>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 8 && groups == 4) return run_attn_grp<8, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 12 && groups == 3) return run_attn_grp<12, 3>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 6 && groups == 2) return run_attn_grp<6, 2>(q, k, vt, o, B, H, T, Tpad, ldo, st);
    if (nw == 16 && groups == 4) return run_attn_grp<16, 4>(q, k, vt, o, B, H, T, Tpad, ldo, st);
  }
  if (nw == 8 && qs2 && split <= 1) return run_attn<8, 2, 2>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, 1, st);
  if (nw == 4 && qs2 && split <= 1) return run_attn<4, 2, 2>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, 1, st);
  if (nw == 8) {
    if (ring == 4) return run_attn<8, 4>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
    if (ring == 3) return run_attn<8, 3>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
    return run_attn<8, 2>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
  }
  if (ring == 4) return run_attn<4, 4>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
  if (ring == 3) return run_attn<4, 3>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
  return run_attn<4, 2>(q, k, vt, o, B, H, T, Tpad, ldo, ws, ws_bytes, split, st);
}

}  // namespace mde
