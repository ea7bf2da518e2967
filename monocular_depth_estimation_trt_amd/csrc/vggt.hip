// VGGT depth-path forward schedule: the reference's
// `models/vggt` TensorRT engine (onnx_export.py:38-131, `VGGTDepthOnlyWrapper`:
// input "images" [B, S, 3, 518, 518] fp32 in [0, 1], output "depth"
// [B, S, 518, 518, 1]), restated on the gfx950 kernels of this library.
// Graph (upstream facebookresearch/vggt, restated in oracle/vggt_ref.py):
//
//   images (ImageNet normalisation folded into the patch-embed weights)
//   -> DINOv2-L/14 with 4 registers: [cls, 4 reg, 1369 patches] x 24 blocks,
//      final norm over the patch tokens
//   -> aggregator: [camera, 4 reg (set 0 for frame 0, set 1 else), patches];
//      24 x (frame block over each frame's 1374 tokens, global block over the
//      S * 1374 tokens of a batch item); blocks carry per-head q/k LayerNorm
//      and 2D RoPE (q_norm/k_norm + rope: one kernel between QKV and attention)
//   -> at blocks 4/11/17/23: LayerNorm(2048) over cat(frame_out, global_out)
//      of the patch tokens, 1x1 projection + UV embedding (one epilogue)
//   -> the DA-V2 DPT decoder (ConvT4 / ConvT2 / id / conv s2, layerN_rn,
//      refinenets whose residual units add relu(x): nn.ReLU(inplace=True))
//   -> output_conv1, bilinear x2 and to 518 (fused into the conv loaders),
//      output_conv2 with the folded UV-embedding conv added before its ReLU,
//      1x1 -> depth channel, exp (one epilogue).
//
// Layout: residual stream X fp32 [B*S][T][D] (frame-major inside a batch
// item, so the global view [B][S*T][D] is the same memory); q / k / v^T
// head-major f16 with a zero pad to Tpad (frame) or Tgpad = roundup(S*T, 64)
// (global, separate buffers when S > 1); maps NHWC f16 over the B*S frames.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "engine_internal.h"

namespace mde {

namespace {

constexpr float kQScale = 0.125f * 1.4426950408889634f;  // dh^-0.5 * log2(e): scores in log2 units

bool dims_are(const DevTensor* t, std::initializer_list<int> d) {
  if (!t || t->ndim != (int)d.size()) return false;
  int i = 0;
  for (int v : d)
    if (t->dims[i++] != v) return false;
  return true;
}

}  // namespace

std::string setup_vggt(mde_engine* e) {
  const PackConfig& c = e->cfg;
  const int D = c.embed_dim;
  if (c.patch != 14 || D % 64 || c.num_heads * 64 != D || c.img_h != c.img_w || c.img_h % 14 || c.img_h <= 0 ||
      c.features % 32 || c.head_hidden != 32 || c.metric != 2 || c.input_u8 != 0 || c.mlp_hidden != 4 * D)
    return "unsupported VGGT geometry in packed config";
  if (D != 128 && D != 256 && D != 384 && D != 768 && D != 1024) return "VGGT embed dim must be 128/256/384/768/1024";
  if (c.frames < 1 || c.npre != 5 || c.aa_depth < 1 || !(c.agg_eps > 0.f) || c.depth < 1)
    return "bad VGGT aggregator fields in packed config";
  for (int i = 0; i < 4; ++i)
    if (c.taps[i] < 0 || c.taps[i] >= c.aa_depth || (i && c.taps[i] <= c.taps[i - 1]))
      return "VGGT taps must be increasing aggregator block indices";
  e->D = D;
  e->H = c.num_heads;
  e->F = c.features;
  e->ph = c.img_h / 14;
  e->pw = c.img_w / 14;
  e->np = e->ph * e->pw;
  e->npre = c.npre;
  e->S = c.frames;
  e->T = e->np + e->npre;
  e->Tpad = (e->T + 63) / 64 * 64;
  e->Tg = e->S * e->T;
  e->Tgpad = (e->Tg + 63) / 64 * 64;
  e->h4 = (e->ph + 1) / 2;
  e->w4 = (e->pw + 1) / 2;
  e->c1p = (c.out_channels[0] + 31) / 32 * 32;
  std::vector<std::string> need = {"patch.w", "patch.b", "pos.patch", "pre.dino", "norm.g", "norm.b", "pre.agg",
                                   "rope.cos", "rope.sin", "dh.norm.g", "dh.norm.b", "rs0.w", "rs0.b", "rs1.w",
                                   "rs1.b", "rs3.w", "rs3.b", "head.c1.w", "head.c1.b", "head.c2.w", "head.c2.b",
                                   "head.pe", "head.c3.w", "head.c3.b"};
  const char* blk[] = {"ln1.g", "ln1.b", "qkv.w", "qkv.b", "proj.w", "proj.b", "ls1",
                       "ln2.g", "ln2.b", "fc1.w", "fc1.b", "fc2.w", "fc2.b", "ls2"};
  for (int i = 0; i < c.depth; ++i)
    for (const char* s : blk) need.push_back("db" + std::to_string(i) + "." + s);
  for (int i = 0; i < c.aa_depth; ++i)
    for (const char* pfx : {"fb", "gb"}) {
      const std::string p = pfx + std::to_string(i) + ".";
      for (const char* s : blk) need.push_back(p + s);
      for (const char* s : {"qn.g", "qn.b", "kn.g", "kn.b"}) need.push_back(p + s);
    }
  for (int i = 0; i < 4; ++i) {
    need.push_back("proj" + std::to_string(i) + ".w");
    need.push_back("proj" + std::to_string(i) + ".b");
    need.push_back("pe" + std::to_string(i));
    need.push_back("rn" + std::to_string(i + 1) + ".w");
  }
  for (int r = 1; r <= 4; ++r) {
    const std::string p = "rf" + std::to_string(r) + ".";
    need.push_back(p + "out.w");
    need.push_back(p + "out.b");
    for (int u = (r == 4 ? 2 : 1); u <= 2; ++u)
      for (int cc = 1; cc <= 2; ++cc) {
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + ".w");
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + ".b");
      }
  }
  for (auto& s : need)
    if (!e->get(s)) return "packed VGGT engine lacks tensor '" + s + "'";
  // tables the kernels index without bounds checks
  const DevTensor* rc = e->get("rope.cos");
  const DevTensor* rs = e->get("rope.sin");
  const int gmax = std::max(e->ph, e->pw) + 1;
  if (rc->ndim != 2 || rc->dims[1] != 16 || rc->dims[0] < gmax || rs->ndim != 2 || rs->dims[1] != 16 ||
      rs->dims[0] < gmax)
    return "VGGT RoPE tables too small for the packed grid";
  if (!dims_are(e->get("pre.dino"), {5, D}) || !dims_are(e->get("pre.agg"), {2, 5, D}) ||
      !dims_are(e->get("pos.patch"), {e->np, D}) || !dims_are(e->get("head.pe"), {c.img_h * c.img_w, 32}) ||
      !dims_are(e->get("head.c3.w"), {32}) || e->get("head.pe")->dtype != 1)
    return "VGGT token / embedding tables do not match the packed geometry";
  for (int i = 0; i < 4; ++i) {
    const DevTensor* pe = e->get("pe" + std::to_string(i));
    if (!dims_are(pe, {e->np, c.out_channels[i]}) || pe->dtype != 1)
      return "VGGT projection embedding table pe" + std::to_string(i) + " does not match the packed geometry";
  }
  return "";
}

size_t plan_arena_vggt(const mde_engine& e, int B, VGBuf* b, uint8_t* base) {
  ArenaPlan a(base);
  const size_t n = (size_t)B * e.S;  // frames in the batch
  const size_t T = e.T, D = e.D, F = e.F, np = e.np;
  const int* oc = e.cfg.out_channels;
  const size_t s1 = (size_t)(4 * e.ph) * (4 * e.pw), s2 = (size_t)(2 * e.ph) * (2 * e.pw), s3 = np,
               s4 = (size_t)e.h4 * e.w4;
  const size_t s0 = (size_t)(8 * e.ph) * (8 * e.pw);
  VGBuf t{};
  t.P = a.h(n * np * 672);
  t.X = a.f(n * T * D);
  t.Xf = a.f(n * T * D);
  t.Hn = a.h(n * T * D);
  t.O = a.h(n * T * D);
  t.Mh = a.h(n * T * e.cfg.mlp_hidden);
  t.Q = a.h(n * e.H * e.Tpad * 64);
  t.K = a.h(n * e.H * e.Tpad * 64);
  t.Vt = a.h(n * e.H * e.Tpad * 64);
  if (e.S > 1) {
    t.Qg = a.h((size_t)B * e.H * e.Tgpad * 64);
    t.Kg = a.h((size_t)B * e.H * e.Tgpad * 64);
    t.Vg = a.h((size_t)B * e.H * e.Tgpad * 64);
  } else {  // one frame: the global sequence is the frame sequence
    t.Qg = t.Q;
    t.Kg = t.K;
    t.Vg = t.Vt;
  }
  t.tap = a.h(n * np * 2 * D);
  for (int i = 0; i < 4; ++i) t.pj[i] = a.h(n * np * oc[i]);
  t.l1 = a.h(n * s1 * e.c1p);
  t.l2 = a.h(n * s2 * oc[1]);
  t.l4 = a.h(n * s4 * oc[3]);
  const size_t ss[4] = {s1, s2, s3, s4};
  for (int i = 0; i < 4; ++i) t.rn[i] = a.h(n * ss[i] * F);
  t.tb = a.h(n * s1 * F);
  t.sb = a.h(n * s1 * F);
  t.ub = a.h(n * s1 * F);
  t.vb = a.h(n * s1 * F);
  t.p4 = a.h(n * s3 * F);
  t.p3 = a.h(n * s2 * F);
  t.p2 = a.h(n * s1 * F);
  t.c1 = a.h(n * s0 * (F / 2));
  t.ws_rows = n * T <= 4096 ? n * T : 0;
  t.ws = t.ws_rows ? a.f(fc2_ws_floats(t.ws_rows, D)) : nullptr;
  t.sws = a.f(kSplitWsAlloc);
  if (b) *b = t;
  return a.off;
}

// One transformer block over `seqs` sequences of T tokens (the residual
// stream c.v.X, seqs * T rows).  qk: aggregator block (q/k LayerNorm + RoPE,
// the q scale applied after them); else a DINOv2 block (q pre-scaled by the
// QKV epilogue).
void Runner::vggt_block(const std::string& p, float eps, bool qk, int seqs, int T, int Tpad, h16* Q, h16* K, h16* Vt) {
  mde_engine& e = *c.e;
  VGBuf& v = c.v;
  const int D = e.D, rows = seqs * T, mlp = e.cfg.mlp_hidden;
  step((p + "norm1").c_str(), [&] {
    return launch_layernorm(v.X, v.Hn, w32(p + "ln1.g"), w32(p + "ln1.b"), rows, D, eps, T, 0, st);
  });
  {
    GemmParams g = dense(v.Hn, D, p + "qkv.w", rows, 3 * D, D);
    g.emode = E_QKV;
    g.bias = w32(p + "qkv.b");
    g.q = Q;
    g.k = K;
    g.vt = Vt;
    g.T = T;
    g.Tpad = Tpad;
    g.heads = e.H;
    g.qscale = qk ? 1.f : kQScale;
    gemm((p + "qkv").c_str(), g);
  }
  if (qk) {
    RopeGeom geo;
    geo.T = T;
    geo.Tpad = Tpad;
    geo.P = e.T;
    geo.npre = e.npre;
    geo.gw = e.pw;
    geo.qscale = kQScale;
    geo.eps = eps;
    step((p + "qk_rope").c_str(), [&] {
      return launch_qk_norm_rope(Q, K, w32(p + "qn.g"), w32(p + "qn.b"), w32(p + "kn.g"), w32(p + "kn.b"),
                                 w32("rope.cos"), w32("rope.sin"), seqs * e.H, geo, st);
    });
  }
  step((p + "attn").c_str(), [&] { return launch_attention(Q, K, Vt, v.O, seqs, e.H, T, Tpad, D, st); });
  {
    GemmParams g = dense(v.O, D, p + "proj.w", rows, D, D);
    g.emode = E_RESID;
    g.bias = w32(p + "proj.b");
    g.ls = w32(p + "ls1");
    g.x32 = v.X;
    g.ldo = D;
    gemm((p + "proj").c_str(), g);
  }
  step((p + "norm2").c_str(), [&] {
    return launch_layernorm(v.X, v.Hn, w32(p + "ln2.g"), w32(p + "ln2.b"), rows, D, eps, T, 0, st);
  });
  {
    GemmParams g = dense(v.Hn, D, p + "fc1.w", rows, mlp, D);
    g.emode = E_STORE;
    g.bias = w32(p + "fc1.b");
    g.act = ACT_GELU;
    g.out16 = v.Mh;
    g.ldo = mlp;
    gemm((p + "fc1").c_str(), g);
  }
  {
    GemmParams g = dense(v.Mh, mlp, p + "fc2.w", rows, D, mlp);
    g.emode = E_RESID;
    g.bias = w32(p + "fc2.b");
    g.ls = w32(p + "ls2");
    g.x32 = v.X;
    g.ldo = D;
    // small batch: split fc2's K = 4D loop (as the DA-V2 fc2, engine.hip);
    // B = 1, S = 1: 352 64^2 tiles x 2 slices
    const long long t64 = (long long)((rows + 63) / 64) * ((D + 63) / 64);
    if (v.ws && (size_t)rows <= v.ws_rows && t64 < 512 && mlp >= 1024 && knob(KNOB_SPLITK)) {
      g.partial = v.ws;
      g.splitk = t64 < 256 ? 4 : 2;
      g.slot_cap = fc2_ws_floats(rows, D);
      g.tile_cnt = split_counters(v.sws);
      g.tile_cnt_cap = kTileCnt;
    }
    gemm((p + "fc2").c_str(), g);
  }
}

// FeatureFusionBlock with in-place-ReLU residual units (the skips add
// relu(x)); out_conv (1x1) before the resize, as dav2_fusion.
void Runner::vggt_fusion(int r, const h16* x0, const h16* x1, int n, int h, int w, h16* dst, int oh, int ow) {
  const std::string p = "rf" + std::to_string(r);
  const int F = c.e->F;
  VGBuf& v = c.v;
  const h16* s = x0;
  if (x1) {
    rcu(p + ".rcu1", x1, x0, v.sb, v.tb, n, h, w, F, true);
    s = v.sb;
  }
  rcu(p + ".rcu2", s, nullptr, v.ub, v.tb, n, h, w, F, true);
  GemmParams g = dense(v.ub, F, p + ".out.w", n * h * w, F, F);
  g.emode = E_STORE;
  g.bias = w32(p + ".out.b");
  g.out16 = v.vb;
  g.ldo = F;
  gemm((p + ".out").c_str(), g);
  if (dst) step((p + ".resize").c_str(), [&] { return launch_resize(v.vb, dst, n, h, w, F, oh, ow, st); });
}

hipError_t Runner::forward_vggt(int B, const float* img, float* out) {
  mde_engine& e = *c.e;
  const PackConfig& cf = e.cfg;
  VGBuf& v = c.v;
  const int n = B * e.S;  // frames
  const int D = e.D, T = e.T, np = e.np, F = e.F;
  const int* oc = cf.out_channels;
  char nm[64];
  split_ws = v.sws;

  // ---- DINOv2-L/14-reg patch embedding over all frames ----
  step("patch_prep", [&] {
    return launch_patch_prep(img, v.P, v.X, w32("pre.dino"), n, cf.img_h, cf.img_w, e.ph, e.pw, T, D, st);
  });
  step("dino.prefix", [&] { return launch_prefix_rows(v.X, w32("pre.dino"), n, T, e.npre, D, 1, 1, st); });
  {
    GemmParams g = dense(v.P, 672, "patch.w", n * np, D, 672);
    g.emode = E_PATCH;
    g.bias = w32("patch.b");
    g.x32 = v.X;
    g.ldo = D;
    g.T = T;
    g.tok0 = e.npre;
    g.pos = w32("pos.patch");
    g.npatch = np;
    gemm("patch_embed", g);
  }
  for (int i = 0; i < cf.depth; ++i)
    vggt_block("db" + std::to_string(i) + ".", cf.ln_eps, false, n, T, e.Tpad, v.Q, v.K, v.Vt);
  step("dino.norm", [&] {
    return launch_rows_layernorm(v.X, w32("norm.g"), w32("norm.b"), n, T, e.npre, D, cf.ln_eps, st);
  });
  // ---- aggregator ----
  step("agg.prefix", [&] { return launch_prefix_rows(v.X, w32("pre.agg"), n, T, e.npre, D, e.S, 2, st); });
  int tap = 0;
  for (int i = 0; i < cf.aa_depth; ++i) {
    vggt_block("fb" + std::to_string(i) + ".", cf.agg_eps, true, n, T, e.Tpad, v.Q, v.K, v.Vt);
    const bool tapped = tap < 4 && cf.taps[tap] == i;
    if (tapped) {
      snprintf(nm, sizeof nm, "tap%d.frame_copy", tap);
      step(nm, [&] {
        return hipMemcpyAsync(v.Xf, v.X, (size_t)n * T * D * sizeof(float), hipMemcpyDeviceToDevice, st);
      });
    }
    vggt_block("gb" + std::to_string(i) + ".", cf.agg_eps, true, B, e.Tg, e.Tgpad, v.Qg, v.Kg, v.Vg);
    if (!tapped) continue;
    // depth-head tap: LN over cat(frame, global) patch tokens -> 1x1 projection + UV embedding
    snprintf(nm, sizeof nm, "tap%d.norm", tap);
    step(nm, [&] {
      return launch_tap_concat_ln(v.Xf, v.X, v.tap, w32("dh.norm.g"), w32("dh.norm.b"), n, T, e.npre, D, cf.agg_eps,
                                  st);
    });
    GemmParams g = dense(v.tap, 2 * D, "proj" + std::to_string(tap) + ".w", n * np, oc[tap], 2 * D);
    g.emode = E_STORE;
    g.bias = w32("proj" + std::to_string(tap) + ".b");
    g.out16 = v.pj[tap];
    g.ldo = oc[tap];
    g.res0 = w16("pe" + std::to_string(tap));
    g.res0_rows = np;
    snprintf(nm, sizeof nm, "reassemble%d.project", tap);
    gemm(nm, g);
    ++tap;
  }
  if (tap != 4) return hipErrorInvalidValue;

  // ---- DPT decoder (as forward_dav2, over the n frames) ----
  {
    GemmParams g = dense(v.pj[0], oc[0], "rs0.w", n * np, 16 * oc[0], oc[0]);
    g.emode = E_CONVT;
    g.bias = w32("rs0.b");
    g.out16 = v.l1;
    g.s = 4;
    g.cout = oc[0];
    g.ldo = e.c1p;
    g.ih = e.ph;
    g.iw = e.pw;
    gemm("reassemble0.convT4", g);
  }
  {
    GemmParams g = dense(v.pj[1], oc[1], "rs1.w", n * np, 4 * oc[1], oc[1]);
    g.emode = E_CONVT;
    g.bias = w32("rs1.b");
    g.out16 = v.l2;
    g.s = 2;
    g.cout = oc[1];
    g.ldo = oc[1];
    g.ih = e.ph;
    g.iw = e.pw;
    gemm("reassemble1.convT2", g);
  }
  {
    GemmParams g = conv(v.pj[3], n, e.ph, e.pw, oc[3], "rs3.w", oc[3], 2);
    g.bias = w32("rs3.b");
    g.out16 = v.l4;
    gemm("reassemble3.conv_s2", g);
  }
  const int hs[4] = {4 * e.ph, 2 * e.ph, e.ph, e.h4};
  const int ws[4] = {4 * e.pw, 2 * e.pw, e.pw, e.w4};
  const h16* lay[4] = {v.l1, v.l2, v.pj[2], v.l4};
  const int cin[4] = {e.c1p, oc[1], oc[2], oc[3]};
  for (int i = 0; i < 4; ++i) {
    GemmParams g = conv(lay[i], n, hs[i], ws[i], cin[i], "rn" + std::to_string(i + 1) + ".w", F, 1);
    g.out16 = v.rn[i];
    snprintf(nm, sizeof nm, "layer%d_rn", i + 1);
    gemm(nm, g);
  }
  vggt_fusion(4, v.rn[3], nullptr, n, hs[3], ws[3], v.p4, hs[2], ws[2]);
  vggt_fusion(3, v.p4, v.rn[2], n, hs[2], ws[2], v.p3, hs[1], ws[1]);
  vggt_fusion(2, v.p3, v.rn[1], n, hs[1], ws[1], v.p2, hs[0], ws[0]);
  vggt_fusion(1, v.p2, v.rn[0], n, hs[0], ws[0], nullptr, 0, 0);  // 1x1 result in vb at hs[0] x ws[0]
  // ---- head ----
  const int H1 = 2 * hs[0], W1 = 2 * ws[0];
  {
    GemmParams g;
    g.amode = A_CONV3_UP;
    g.emode = E_STORE;
    g.A = v.vb;
    g.cb = n;
    g.ch = hs[0];
    g.cw = ws[0];
    g.cc = F;
    g.uh = H1;
    g.uw = W1;
    g.oh = H1;
    g.ow = W1;
    g.stride = 1;
    g.W = w16("head.c1.w");
    g.ldw = ldw("head.c1.w");
    g.M = n * H1 * W1;
    g.N = F / 2;
    g.K = 9 * F;
    g.bias = w32("head.c1.b");
    g.out16 = v.c1;
    g.ldo = F / 2;
    gemm("head.output_conv1", g);
  }
  {
    const int OH = cf.img_h, OW = cf.img_w;
    GemmParams g;
    g.amode = A_CONV3_UP;
    g.emode = E_HEAD;
    g.A = v.c1;
    g.cb = n;
    g.ch = H1;
    g.cw = W1;
    g.cc = F / 2;
    g.uh = OH;
    g.uw = OW;
    g.oh = OH;
    g.ow = OW;
    g.stride = 1;
    g.W = w16("head.c2.w");
    g.ldw = ldw("head.c2.w");
    g.M = n * OH * OW;
    g.N = cf.head_hidden;
    g.K = 9 * (F / 2);
    g.bias = w32("head.c2.b");
    g.hpe = w16("head.pe");
    g.hpe_pix = OH * OW;
    g.w2 = w32("head.c3.w");
    g.b2 = e.head_b2;
    g.head_metric = 2;  // depth = exp(channel 0) (upstream activate_head "exp")
    g.out32 = out;
    gemm("head.output_conv2", g);
  }
  return err;
}

}  // namespace mde
