// Shared MFMA-tile epilogue of the GEMM and the direct-conv kernels.
//
// acc[i][j] holds C^T of the 16x16 block (row block i, column block j): the
// MFMA is issued with the weights as its A operand, so lane l owns output row
// mrow[i] (= -1 when outside the problem) and the four consecutive columns
// ncol + 16 j .. +3 -- every store is 8 B (f16) or 16 B (f32) per lane.
// The epilogue fuses what follows the contraction in the reference graph.
#pragma once
#include <type_traits>
#include "mde_device.h"
#include "mde_ops.h"

namespace mde {

// E_STORE residual element offset of output element o = m*ldo + n: the row
// of a repeated table (res0_rows > 0) or the output's own offset.
MDE_DEV size_t res0_offset(const GemmParams& p, int m, int n, size_t o) {
  return p.res0_rows > 0 ? (size_t)(m % p.res0_rows) * p.ldo + n : o;
}

// res1 of output row m, channels [n, n + 8), through GemmParams::res1_up
MDE_DEV f16x8 res1_up8(const GemmParams& p, int m, int n) {
  const int hw = p.oh * p.ow, b = m / hw, r = m - b * hw, oy = r / p.ow, ox = r - (r / p.ow) * p.ow;
  return upsample8(reinterpret_cast<const f16*>(p.res1_up), b, p.res1_uh, p.res1_uw, p.N, p.oh, p.ow, oy, ox, n);
}

// NaN (sum, M2) for the 32-column slice of column n in row `row` of the
// folded-LayerNorm partials (GemmParams::lnst_out)
MDE_DEV void poison_ln_partials(const GemmParams& p, int row, int n) {
  *reinterpret_cast<float2*>(p.lnst_out + ((size_t)(n >> 5) * p.lnst_rows + row) * 2) =
      make_float2(__builtin_nanf(""), __builtin_nanf(""));
}

// slice: the split-K slice of an E_PARTIAL tile (its fp32 slab in x32)
// RUP: E_STORE may read res1 through GemmParams::res1_up (the direct conv)
template <int EM, int TM, int TN, bool RUP = false>
MDE_DEV void store_tile(const GemmParams& p, f32x4 (&acc)[TM][TN], const int (&mrow)[TM], int ncol, int lane,
                        int slice = 0) {
  if constexpr (EM == E_HEAD) {
    static_assert(TN == 2, "head epilogue needs the full 32-channel row in one wave (BN 32, WN 1)");
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = mrow[i];
      const f16* pe = (p.hpe && m >= 0) ? reinterpret_cast<const f16*>(p.hpe) + (size_t)(m % p.hpe_pix) * 32 : nullptr;
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n0 = j * 16 + (lane >> 4) * 4;
        f16x4 pv = {(f16)0.0f, (f16)0.0f, (f16)0.0f, (f16)0.0f};
        if (pe) pv = *reinterpret_cast<const f16x4*>(pe + n0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r] + p.bias[n0 + r] + (float)pv[r];
          part += (v > 0.f ? v : 0.f) * p.w2[n0 + r];
        }
      }
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      if ((lane >> 4) == 0 && m >= 0) {
        const float z = part + p.b2;
        p.out32[m] = p.head_metric == 2 ? __expf(z)
                     : p.head_metric ? p.max_depth / (1.f + __expf(-z)) : (z > 0.f ? z : 0.f);
      }
    }
    return;
  } else if constexpr (EM == E_PARTIAL) {
    float* dst = p.x32 + (size_t)slice * p.M * p.ldo;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        if (mrow[i] >= 0) *reinterpret_cast<f32x4*>(dst + (size_t)mrow[i] * p.ldo + n) = acc[i][j];
    }
    return;
  } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
      float4 bn = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EM == E_CONVT) {
        if (p.bias) bn = *reinterpret_cast<const float4*>(p.bias + (n % p.cout));
      } else {
        if (p.bias) bn = *reinterpret_cast<const float4*>(p.bias + n);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mrow[i];
        if (m < 0) continue;
        float v[4] = {acc[i][j][0] + bn.x, acc[i][j][1] + bn.y, acc[i][j][2] + bn.z, acc[i][j][3] + bn.w};
        if constexpr (EM == E_STORE) {
          if (p.act == ACT_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
          } else if (p.act == ACT_GELU) {
            const f32x2 lo = gelu_erf2(f32x2{v[0], v[1]}), hi = gelu_erf2(f32x2{v[2], v[3]});
            v[0] = lo[0], v[1] = lo[1], v[2] = hi[0], v[3] = hi[1];
          }
          const size_t o = (size_t)m * p.ldo + n;
          if (p.res0) {
            const f16x4 r0 =
                *reinterpret_cast<const f16x4*>(reinterpret_cast<const f16*>(p.res0) + res0_offset(p, m, n, o));
            if (p.res0_relu) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += fmaxf((float)r0[r], 0.f);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += (float)r0[r];
            }
          }
          if (p.res1) {
            const f16x4 r1 = *reinterpret_cast<const f16x4*>(reinterpret_cast<const f16*>(p.res1) + o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (float)r1[r];
          }
          if constexpr (RUP) {
            if (p.res1_up) {
              const f16x8 u = res1_up8(p, m, n & ~7);
              const int hq = n & 4;
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += (float)u[hq + r];
            }
          }
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = (f16)v[r];
          *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.out16) + o) = h;
        } else if constexpr (EM == E_QKV) {
          const int D = p.heads * 64;
          const int which = n / D, w = n - which * D;
          const int b = m / p.T, t = m - (m / p.T) * p.T;
          const size_t bh = (size_t)b * p.heads + (w >> 6);
          if (which == 2) {
            f16* dst = reinterpret_cast<f16*>(p.vt) + (bh * 64 + (w & 63)) * p.Tpad + vt_pos(t);
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)r * p.Tpad] = (f16)v[r];
          } else {
            const float sc = which == 0 ? p.qscale : 1.f;
            f16x4 h;
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = (f16)(v[r] * sc);
            f16* dst = (which == 0 ? reinterpret_cast<f16*>(p.q) : reinterpret_cast<f16*>(p.k)) +
                       (bh * p.Tpad + t) * 64 + (w & 63);
            *reinterpret_cast<f16x4*>(dst) = h;
          }
        } else if constexpr (EM == E_RESID) {
          // the folded-LayerNorm partials are written by the LDS-staged
          // epilogue only (whole 32-column slices per wave): a tile that
          // reaches this direct path poisons them, so the next qkv / fc1
          // produces NaN instead of silently normalising with stale stats
          if (p.lnst_out) poison_ln_partials(p, m, n);
          const float4 l = *reinterpret_cast<const float4*>(p.ls + n);
          if (p.xh) {  // f16 residual stream: fp32 update, one rounding
            f16x4* x = reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.xh) + (size_t)m * p.ldo + n);
            f16x4 xv = *x;
            xv[0] = (f16)((float)xv[0] + l.x * v[0]);
            xv[1] = (f16)((float)xv[1] + l.y * v[1]);
            xv[2] = (f16)((float)xv[2] + l.z * v[2]);
            xv[3] = (f16)((float)xv[3] + l.w * v[3]);
            *x = xv;
          } else {
            float4* x = reinterpret_cast<float4*>(p.x32 + (size_t)m * p.ldo + n);
            float4 xv = *x;
            xv.x += l.x * v[0];
            xv.y += l.y * v[1];
            xv.z += l.z * v[2];
            xv.w += l.w * v[3];
            *x = xv;
          }
        } else if constexpr (EM == E_PATCH) {
          const int b = m / p.npatch, pi = m - (m / p.npatch) * p.npatch;
          const float4 ps = *reinterpret_cast<const float4*>(p.pos + (size_t)pi * p.ldo + n);
          const size_t xo = ((size_t)b * p.T + p.tok0 + pi) * p.ldo + n;
          if (p.lnst_out) poison_ln_partials(p, (int)((size_t)b * p.T + p.tok0 + pi), n);
          if (p.xh) {
            f16x4 h = {(f16)(v[0] + ps.x), (f16)(v[1] + ps.y), (f16)(v[2] + ps.z), (f16)(v[3] + ps.w)};
            *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.xh) + xo) = h;
          } else {
            *reinterpret_cast<float4*>(p.x32 + xo) = float4{v[0] + ps.x, v[1] + ps.y, v[2] + ps.z, v[3] + ps.w};
          }
        } else if constexpr (EM == E_CONVT) {
          const int q = n / p.cout, co = n - q * p.cout;
          const int dy = q / p.s, dx = q - (q / p.s) * p.s;
          const int hw = p.ih * p.iw;
          const int b = m / hw, rem = m - (m / hw) * hw;
          const int y = rem / p.iw, x = rem - (rem / p.iw) * p.iw;
          const int OH = p.ih * p.s, OW = p.iw * p.s;
          const size_t o = (((size_t)b * OH + y * p.s + dy) * OW + x * p.s + dx) * p.ldo + co;  // ldo = channel stride
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = (f16)v[r];
          *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.out16) + o) = h;
        }
      }
    }
  }
}

// LDS-staged epilogue for the row-major outputs (E_STORE, E_RESID and the
// q/k thirds of E_QKV): the wave parks its (16 TM) x (16 TN) tile in its own
// LDS slice (bias/activation applied, residuals not yet), then re-reads it
// row-wise so that each lane owns 8 consecutive columns and every store
// instruction writes whole 128-B lines (the direct path touches 16 partial
// lines per instruction).  One rounding to f16, as the direct path.
// `lds` = this wave's slice: 16 TM * 16 TN * 4 bytes, or with HALF only half
// of that -- then the tile is parked as f16 when nothing is added after the
// activation (E_QKV, E_CONVT, E_STORE without residuals: the f16 value IS the
// output, so still one rounding), otherwise as fp32 in two row passes.
// mof(row) = output row of wave-tile row `row` (or -1), n0w = the wave's
// first output column; the caller has retired every LDS read of the main
// loop (barrier) before the call.  Returns false (nothing written) for modes
// it does not stage -- the caller then runs store_tile.
template <int EM, int TM, int TN, int HALF = 0, bool PRES = false, class RowMap>
MDE_DEV bool store_tile_lds(const GemmParams& p, f32x4 (&acc)[TM][TN], RowMap mof, int n0w, int lane, char* lds) {
  constexpr int R = TM * 16, C = TN * 16;  // wave tile
  constexpr int CHR = C / 4;               // 16-B fp32 chunks per staged row
  constexpr int CPR = C / 8;               // lanes per row in the read-back (8 columns each)
  constexpr int RPI = 64 / CPR;            // rows per read-back instruction
  static_assert(TN >= 1 && C % 8 == 0, "tile");
  if constexpr (EM != E_STORE && EM != E_RESID && EM != E_QKV && EM != E_CONVT && EM != E_PATCH) {
    return false;
  } else if constexpr ((CPR & (CPR - 1)) != 0 || (CHR & (CHR - 1)) != 0) {
    // the row swizzles and the read-back geometry need power-of-two chunk
    // counts per row (a 48-column wave tile, TN = 3, takes the direct path)
    return false;
  } else {
    if constexpr (EM == E_RESID || EM == E_PATCH) {
      if (p.lnst_out && (C % 32)) return false;  // LN partials need whole 32-column slices per wave
    }
    // E_CONVT: 8 consecutive columns stay inside one sub-pixel when cout % 8 == 0,
    // so each lane writes 16 B of one output pixel (the direct path writes 8 B)
    if constexpr (EM == E_CONVT) {
      if (p.cout & 7) return false;
    }
    int which = 0;
    if constexpr (EM == E_QKV) {
      which = n0w / (p.heads * 64);
      if ((n0w & 63) + C > 64) return false;
      // V^T staging: one whole head, 64 token rows crossing at most one image
      if (which == 2 && (C != 64 || R != 64 || p.T < R)) return false;
    }
    bool f16stage = false;  // HALF: f16 rows (else fp32 in two passes)
    if constexpr (HALF) {
      bool exact = EM == E_QKV || EM == E_CONVT;
      if constexpr (EM == E_STORE) exact = !p.res0 && !p.res1 && !(PRES && p.res1_up);
      f16stage = exact;
      if (!exact && (TM % 2)) return false;
    }
    // fp32 rows: C*4 bytes, 16-B chunks swizzled by row
    auto phys = [&](int row, int ch) { return row * (C * 4) + ((ch ^ (row & (CHR >= 8 ? 7 : CHR - 1))) << 4); };
    // f16 rows: C*2 bytes; c8 = 8-B column quad, the 16-B chunk c8/2 swizzled by row
    auto phys8 = [&](int row, int c8) {
      return row * (C * 2) + ((((c8 >> 1) ^ (row & (CPR >= 8 ? 7 : CPR - 1))) << 4) | ((c8 & 1) << 3));
    };
    // bias for all TN column groups in one batch of unpredicated loads (a
    // predicated load per group costs one serialised round trip each)
    float4 bias[TN];
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0w + j * 16 + (lane >> 4) * 4;
        const int nc = n < p.N ? n : 0;
        bias[j] = *reinterpret_cast<const float4*>(p.bias + (EM == E_CONVT ? nc % p.cout : nc));
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) bias[j] = float4{0.f, 0.f, 0.f, 0.f};
    }
    float4 ls0 = {0.f, 0.f, 0.f, 0.f}, ls1 = ls0;
    const int rr = lane / CPR, cc = lane - (lane / CPR) * CPR;
    const int n = n0w + cc * 8;
    if constexpr (EM == E_RESID) {
      const int nc = n < p.N ? n : 0;
      ls0 = *reinterpret_cast<const float4*>(p.ls + nc);
      ls1 = *reinterpret_cast<const float4*>(p.ls + nc + 4);
    }

    // ---- phase 1: accumulator rows [PS*R/NP, (PS+1)*R/NP) (+bias, activation) -> LDS ----
    // (the activation is a template tag: one uniform branch per tile, not
    // per fragment -- a runtime switch inside the unrolled loop costs every
    // fragment its moves, branches and re-materialised constants)
    auto park_act = [&](auto ps_tag, auto np_tag, auto f16_tag, auto act_tag) {
      constexpr int PS = decltype(ps_tag)::value, NP = decltype(np_tag)::value;
      constexpr bool F16 = decltype(f16_tag)::value;
      constexpr int ACT = decltype(act_tag)::value;
      const float sc = (EM == E_QKV && F16 && which == 0) ? p.qscale : 1.f;  // f16 rows carry the q scale
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float4 bn = bias[j];  // columns n >= N are computed but never stored
#pragma unroll
        for (int i = PS * (TM / NP); i < (PS + 1) * (TM / NP); ++i) {
          f32x4 v = acc[i][j];
          v[0] += bn.x; v[1] += bn.y; v[2] += bn.z; v[3] += bn.w;
          if constexpr (ACT == ACT_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
          } else if constexpr (ACT == ACT_GELU) {
            const f32x2 lo = gelu_erf2(f32x2{v[0], v[1]}), hi = gelu_erf2(f32x2{v[2], v[3]});
            v = f32x4{lo[0], lo[1], hi[0], hi[1]};
          }
          const int row = (i - PS * (TM / NP)) * 16 + (lane & 15);
          if constexpr (F16) {
            f16x4 h = {(f16)(v[0] * sc), (f16)(v[1] * sc), (f16)(v[2] * sc), (f16)(v[3] * sc)};
            *reinterpret_cast<f16x4*>(lds + phys8(row, j * 4 + (lane >> 4))) = h;
          } else {
            *reinterpret_cast<f32x4*>(lds + phys(row, j * 4 + (lane >> 4))) = v;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    };
    auto park = [&](auto ps_tag, auto np_tag, auto f16_tag) {
      if constexpr (EM == E_STORE) {
        if (p.act == ACT_GELU) return park_act(ps_tag, np_tag, f16_tag, std::integral_constant<int, ACT_GELU>{});
        if (p.act == ACT_RELU) return park_act(ps_tag, np_tag, f16_tag, std::integral_constant<int, ACT_RELU>{});
      }
      park_act(ps_tag, np_tag, f16_tag, std::integral_constant<int, ACT_NONE>{});
    };
    // 4 staged values of row `row`, 16-B fp32 chunk / 8-B f16 quad `ch`
    auto rd4 = [&](auto f16_tag, int row, int ch) -> f32x4 {
      if constexpr (decltype(f16_tag)::value) {
        const f16x4 h = *reinterpret_cast<const f16x4*>(lds + phys8(row, ch));
        return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
      } else {
        return *reinterpret_cast<const f32x4*>(lds + phys(row, ch));
      }
    };

    // ---- phase 2 for V^T [bh][64 dh][Tpad] (one pass): a lane takes a quad
    // of 4 consecutive token rows x 4 dh columns (4 conflict-free LDS reads:
    // the 16 lanes of an LDS phase read 16 different chunks of the same
    // rows), transposes it in registers and stores 4 token quads (8 B each;
    // vt_pos keeps 4-aligned quads contiguous) -- 16 8-B stores per lane
    // instead of 64 2-byte column stores.  Quads are aligned in token space
    // (t % 4 == 0, one image); a quad cut by the tile edge or an image
    // boundary stores element-wise, as do rows [0, shift).  (GEMM rows are
    // contiguous: m = m0 + r.  The tile's 64 rows cross at most one image
    // boundary, at row rb: one division per lane.)
    auto vt_out = [&](auto f16_tag) {
      const int w = n0w - 2 * p.heads * 64;
      const int m0 = mof(0);
      const int b0 = m0 >= 0 ? m0 / p.T : 0;
      const int t00 = m0 - b0 * p.T, rb = p.T - t00;  // row rb starts image b0 + 1
      const int shift = m0 >= 0 ? (4 - t00 % 4) % 4 : 0;
      f16* vt0 = reinterpret_cast<f16*>(p.vt) + (size_t)(w >> 6) * 64 * p.Tpad;
      const int dc = lane & 15;  // dh 4dc .. 4dc+3
      const size_t hs = (size_t)p.heads * 64 * p.Tpad;  // one image's V^T
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int r0 = shift + 4 * (it * 4 + (lane >> 4));
        int mm[4], be[4], te[4];
        f16x4 rows[4];  // the staged values are f16 outputs either way: 8 VGPRs, not 16
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = r0 + e < R;
          mm[e] = in ? mof(r0 + e) : -1;
          be[e] = b0 + (r0 + e >= rb ? 1 : 0);
          te[e] = t00 + r0 + e - (r0 + e >= rb ? p.T : 0);
          if constexpr (decltype(f16_tag)::value) {
            rows[e] = in ? *reinterpret_cast<const f16x4*>(lds + phys8(r0 + e, dc)) : f16x4{};
          } else {
            const f32x4 v = in ? rd4(f16_tag, r0 + e, dc) : f32x4{0.f, 0.f, 0.f, 0.f};
            rows[e] = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
          }
        }
        const bool quad = mm[0] >= 0 && mm[3] >= 0 && (te[0] & 3) == 0 && be[3] == be[0];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f16* col = vt0 + (size_t)(4 * dc + k) * p.Tpad;
          if (quad) {
            f16x4 h = {rows[0][k], rows[1][k], rows[2][k], rows[3][k]};
            *reinterpret_cast<f16x4*>(col + be[0] * hs + vt_pos(te[0])) = h;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (mm[e] >= 0) col[be[e] * hs + vt_pos(te[e])] = rows[e][k];
          }
        }
      }
      if (shift > 0) {  // rows [0, shift): lane -> (row lane >> 4, dh 16 it + lane & 15)
        const int r = lane >> 4;
        const int m = r < shift ? mof(r) : -1;
        if (m >= 0) {
          const int be = b0 + (r >= rb ? 1 : 0), te = t00 + r - (r >= rb ? p.T : 0);
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int d = it * 16 + (lane & 15);
            const float v = rd4(f16_tag, r, d >> 2)[d & 3];
            vt0[(size_t)d * p.Tpad + be * hs + vt_pos(te)] = (f16)v;
          }
        }
      }
    };

    // folded-LN partials of the f16 residual rows written here: 4 lanes (32
    // columns) per slice, (sum, sum of squared deviations from the slice
    // mean) -> lnst_out[n / 32][m]
    auto ln_partials = [&](int m, const f16x8& xv) {
      float s1 = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) s1 += (float)xv[r];
      s1 += __shfl_xor(s1, 1);
      s1 += __shfl_xor(s1, 2);
      const float ms = s1 * (1.f / 32.f);
      float s2 = 0.f;  // M2 about the slice mean (Chan et al.'s pairwise merge downstream)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float d = (float)xv[r] - ms;
        s2 += d * d;
      }
      s2 += __shfl_xor(s2, 1);
      s2 += __shfl_xor(s2, 2);
      if ((n & 31) == 0)
        *reinterpret_cast<float2*>(p.lnst_out + ((size_t)(n >> 5) * p.lnst_rows + m) * 2) = make_float2(s1, s2);
    };
    // ---- phase 2: whole rows of pass PS out ----
    auto rows_out = [&](auto ps_tag, auto np_tag, auto f16_tag) {
      constexpr int PS = decltype(ps_tag)::value, NP = decltype(np_tag)::value;
      constexpr bool F16 = decltype(f16_tag)::value;
      constexpr int RP = R / NP;  // rows staged per pass
      // f16 staging of a mode whose staged value IS the output (E_STORE without
      // residuals -- f16stage -- E_QKV with the q scale applied in park, E_CONVT):
      // the row leaves as the staged 16 bytes, no f16 -> f32 -> f16 round trip
      constexpr bool RAW = F16 && (EM == E_STORE || EM == E_QKV || EM == E_CONVT);
      if (n >= p.N) return;
      // E_QKV: (image, token) of this lane's rows, advanced by RPI rows per
      // iteration instead of a 32-bit division per row (GEMM row maps are
      // linear: m = m0 + row)
      int qb = 0, qt = 0;
      if constexpr (EM == E_QKV) {
        const int m0r = mof(PS * RP + rr);
        if (m0r < 0) return;
        qb = m0r / p.T;
        qt = m0r - qb * p.T;
      }
      // E_RESID: the pass's f16 residual rows are loaded before its first
      // store -- the compiler cannot move a load above a store it cannot
      // disambiguate, so interleaved each row iteration paid a full round
      // trip (load -> vmcnt(0) -> store).  A lane reads and writes only its
      // own elements, so loading ahead is safe in place.
      constexpr int IT = (RP + RPI - 1) / RPI;
      // (E_STORE's residuals only where the caller asks, PRES: the direct
      // convs -- on the fc1 GEMM tile the arrays cost 22 VGPRs)
      constexpr bool PRE = EM == E_RESID || (EM == E_STORE && PRES && !RAW);
      f16x8 pre0[PRE ? IT : 1], pre1[EM == E_STORE && PRE ? IT : 1];
      if constexpr (PRE) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int row = it * RPI + rr;
          if (RP % RPI != 0 && row >= RP) break;
          const int m = mof(PS * RP + row);
          if (m < 0) continue;
          const size_t o = (size_t)m * p.ldo + n;
          if constexpr (EM == E_STORE) {
            if (p.res0) pre0[it] = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res0) + res0_offset(p, m, n, o));
            if (p.res1) pre1[it] = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res1) + o);
            if constexpr (PRES) {
              if (p.res1_up) pre1[it] = res1_up8(p, m, n);  // (res1 itself is null then)
            }
          } else {
            if (p.xh) pre0[it] = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.xh) + o);
          }
        }
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int row = it * RPI + rr;
        if (RP % RPI != 0 && row >= RP) break;
        if constexpr (EM == E_QKV) {
          if (it > 0) {
            qt += RPI;
            while (qt >= p.T) {
              qt -= p.T;
              ++qb;
            }
          }
        }
        const int m = mof(PS * RP + row);
        if (m < 0) continue;
        f16x8 raw{};
        float v[8];
        if constexpr (RAW) {
          raw = *reinterpret_cast<const f16x8*>(lds + phys8(row, 2 * cc));
        } else {
          const f32x4 a = rd4(f16_tag, row, 2 * cc);
          const f32x4 b = rd4(f16_tag, row, 2 * cc + 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = a[r];
            v[4 + r] = b[r];
          }
        }
        if constexpr (EM == E_STORE) {
          const size_t o = (size_t)m * p.ldo + n;
          if constexpr (RAW) {
            *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.out16) + o) = raw;
            continue;
          }
          if (p.res0) {
            f16x8 r0;
            if constexpr (PRE) r0 = pre0[it];
            else r0 = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res0) + res0_offset(p, m, n, o));
            if (p.res0_relu) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] += fmaxf((float)r0[r], 0.f);
            } else {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] += (float)r0[r];
            }
          }
          if (p.res1 || (PRE && PRES && p.res1_up)) {
            f16x8 r1;
            if constexpr (PRE) r1 = pre1[it];
            else r1 = *reinterpret_cast<const f16x8*>(reinterpret_cast<const f16*>(p.res1) + o);
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] += (float)r1[r];
          }
          f16x8 h;
#pragma unroll
          for (int r = 0; r < 8; ++r) h[r] = (f16)v[r];
          *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.out16) + o) = h;
        } else if constexpr (EM == E_RESID) {
          if (p.xh) {  // f16 residual stream: fp32 update, one rounding, 16-B RMW
            f16x8* x = reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.xh) + (size_t)m * p.ldo + n);
            f16x8 xv = pre0[it];
            const float l8[8] = {ls0.x, ls0.y, ls0.z, ls0.w, ls1.x, ls1.y, ls1.z, ls1.w};
#pragma unroll
            for (int r = 0; r < 8; ++r) xv[r] = (f16)((float)xv[r] + l8[r] * v[r]);
            *x = xv;
            if (p.lnst_out) ln_partials(m, xv);
          } else {
            float4* x = reinterpret_cast<float4*>(p.x32 + (size_t)m * p.ldo + n);
            float4 x0 = x[0], x1 = x[1];
            x0.x += ls0.x * v[0]; x0.y += ls0.y * v[1]; x0.z += ls0.z * v[2]; x0.w += ls0.w * v[3];
            x1.x += ls1.x * v[4]; x1.y += ls1.y * v[5]; x1.z += ls1.z * v[6]; x1.w += ls1.w * v[7];
            x[0] = x0;
            x[1] = x1;
          }
        } else if constexpr (EM == E_PATCH) {
          // patch row m = (image, patch) -> token row b*T + tok0 + patch, + pos
          const int b = m / p.npatch, pi = m - (m / p.npatch) * p.npatch;
          const float4 p0 = *reinterpret_cast<const float4*>(p.pos + (size_t)pi * p.ldo + n);
          const float4 p1 = *reinterpret_cast<const float4*>(p.pos + (size_t)pi * p.ldo + n + 4);
          const float pp[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
          const size_t row = (size_t)b * p.T + p.tok0 + pi;
          if (p.xh) {
            f16x8 h;
#pragma unroll
            for (int r = 0; r < 8; ++r) h[r] = (f16)(v[r] + pp[r]);
            *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.xh) + row * p.ldo + n) = h;
            if (p.lnst_out) ln_partials((int)row, h);
          } else {
            float4* x = reinterpret_cast<float4*>(p.x32 + row * p.ldo + n);
            x[0] = float4{v[0] + pp[0], v[1] + pp[1], v[2] + pp[2], v[3] + pp[3]};
            x[1] = float4{v[4] + pp[4], v[5] + pp[5], v[6] + pp[6], v[7] + pp[7]};
          }
        } else if constexpr (EM == E_CONVT) {
          const int q = n / p.cout, co = n - q * p.cout;
          const int dy = q / p.s, dx = q - (q / p.s) * p.s;
          const int hw = p.ih * p.iw;
          const int b = m / hw, rem = m - (m / hw) * hw;
          const int y = rem / p.iw, x = rem - (rem / p.iw) * p.iw;
          const int OH = p.ih * p.s, OW = p.iw * p.s;
          const size_t o = (((size_t)b * OH + y * p.s + dy) * OW + x * p.s + dx) * p.ldo + co;
          f16x8 h = raw;
          if constexpr (!RAW) {
#pragma unroll
            for (int r = 0; r < 8; ++r) h[r] = (f16)v[r];
          }
          *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.out16) + o) = h;
        } else {  // E_QKV, q or k third
          const int D = p.heads * 64, w = n - which * D;
          const int bh = qb * p.heads + (w >> 6);
          f16x8 h = raw;
          if constexpr (!RAW) {
            const float sc = which == 0 ? p.qscale : 1.f;
#pragma unroll
            for (int r = 0; r < 8; ++r) h[r] = (f16)(v[r] * sc);
          }
          // 32-bit element offset: q / k hold B * heads * Tpad * 64 < 2^31 halves
          f16* dst = (which == 0 ? reinterpret_cast<f16*>(p.q) : reinterpret_cast<f16*>(p.k)) +
                     (unsigned)((bh * p.Tpad + qt) * 64 + (w & 63));
          *reinterpret_cast<f16x8*>(dst) = h;
        }
      }
    };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using T_ = std::true_type;
    using F_ = std::false_type;
    auto one_pass = [&](auto f16_tag) {
      park(I0{}, I1{}, f16_tag);
      if constexpr (EM == E_QKV) {
        if (which == 2) {
          vt_out(f16_tag);
          return;
        }
      }
      rows_out(I0{}, I1{}, f16_tag);
    };
    if constexpr (HALF) {
      if (f16stage) {
        one_pass(T_{});
      } else if constexpr (TM % 2 == 0) {
        park(I0{}, I2{}, F_{});
        rows_out(I0{}, I2{}, F_{});
        __builtin_amdgcn_wave_barrier();  // pass 0's reads before pass 1 overwrites the slice
        park(I1{}, I2{}, F_{});
        rows_out(I1{}, I2{}, F_{});
      }
    } else {
      one_pass(F_{});
    }
    return true;
  }
}

}  // namespace mde
