// Depth Pro forward schedule: the reference's
// `models/depth_pro` TensorRT engine (onnx_export.py:13-60 -> inputs
// "input" [B,3,1536,1536] fp32 normalised to [-1,1]; outputs
// "canonical_inverse_depth" [B,1,1536,1536] and "fov_deg" [B]), restated on
// the gfx950 kernels of this library.  Graph (upstream apple/ml-depth-pro,
// line-by-line in HF:models/depth_pro/modeling_depth_pro.py):
//
//   pyramid x1/x0.5/x0.25 -> 35 patches of 384^2 -> patch encoder (DINOv2-L/16,
//   hooks after blocks 5 and 11 of the 25 high-res patches); x0.25 image ->
//   image encoder and fov encoder (two more DINOv2-L/16)
//   -> merge patches per level (final LayerNorm fused into the gather)
//   -> neck: 1x1 projections + ConvT(2,2) stacks, image ConvT, cat + 1x1 fuse,
//      3x3 projections to 256 channels at 48, 96, 192, 384, 768
//   -> fusion stage: residual conv units, deconv + 1x1 (folded into one
//      ConvT GEMM at pack time), 48 -> 768
//   -> head: 3x3 -> ConvT(2,2) -> 3x3 + ReLU + 1x1 + ReLU (one fused
//      epilogue) -> canonical inverse depth at 1536^2
//   -> fov: Linear neck on the fov tokens + ReLU(3x3 s2 of the 48^2 global
//      features), 2 x (3x3 s2 + ReLU), 6x6 valid conv -> degrees.
//
// Layout: token rows are sequence-major (sequence s = patch * B + image, the
// upstream unfold order), maps NHWC f16, residual streams fp32.
#include <cmath>
#include <cstdio>

#include "engine_internal.h"

namespace mde {

namespace {

int ilog2_exact(int v) {
  int e = 0;
  while ((1 << e) < v) ++e;
  return (1 << e) == v ? e : -1;
}

}  // namespace

std::string setup_depth_pro(mde_engine* e) {
  const PackConfig& c = e->cfg;
  const int S = c.img_h;
  if (c.img_h != c.img_w || c.patch != 16 || c.vit_size <= 0 || c.vit_size % 16 || c.embed_dim % 64 ||
      c.num_heads * 64 != c.embed_dim || c.input_u8 != 0 || c.head_hidden != 32 || c.features % 32)
    return "unsupported Depth Pro geometry in packed config";
  const int G = c.vit_size / 16;
  // the fixed upstream geometry: S = 4 * vit_size (pyramid x0.25 = one patch),
  // levels x0.5 (overlap 0.5) and x1 (overlap 0.25); every merged map must
  // come out at its target size so HF's bilinear resize is the identity
  if (S != 4 * c.vit_size || G % 4 || ilog2_exact(S / G) != 6)
    return "Depth Pro engine supports only the upstream 1536 = 4 x 384 geometry (G = 24 tokens per side)";
  const int fs[3] = {1, 2, 4};  // level i: high, med, low (HF ratios 1, 0.5, 0.25)
  const int strides[3] = {c.vit_size * 3 / 4, c.vit_size / 2, c.vit_size};
  int first = 0;
  for (int i = 0; i < 3; ++i) {
    const int s = S / fs[i];
    int n = 1, stride = c.vit_size;
    if (s != c.vit_size) {
      stride = strides[i];
      n = (s - c.vit_size) / stride + 1;
      if ((n - 1) * stride + c.vit_size != s) return "pyramid level does not tile exactly";
    }
    int pad = n > 1 ? c.merge_pad * fs[i] : 0;  // int(merge_pad / ratio)
    if (n * n < 4) pad = 0;
    pad = std::min(G / 4, pad);
    const int merged = n * G - 2 * (n - 1) * pad;
    const int want = G * (4 / fs[i]);  // base (G) * 2^level_from_low
    if (merged != want) return "merged level map is not the target size (non-identity resize unsupported)";
    e->lev_n[i] = n;
    e->lev_pad[i] = pad;
    e->lev_stride[i] = stride;
    e->lev_f[i] = fs[i];
    e->lev_base[i] = first;
    first += n * n;
  }
  e->G = G;
  e->nseq = first;
  e->D = c.embed_dim;
  e->H = c.num_heads;
  e->F = c.features;
  e->T = G * G + 1;
  e->Tpad = (e->T + 63) / 64 * 64;
  for (int i = 0; i < 2; ++i)
    if (c.hooks[i] < 0 || c.hooks[i] >= c.depth) return "hook block out of range";
  if (c.use_fov) {
    const int k = (int)((G - 1) / (float)(1 << c.fov_layers) + 1);
    if (c.fov_layers != 2 || k != c.fov_k || (G >> c.fov_layers) != k) return "unsupported FOV head geometry";
  }
  // every tensor the forward uses must be present
  std::vector<std::string> need;
  const char* encs[3] = {"pe.", "ie.", "fe."};
  for (int x = 0; x < (c.use_fov ? 3 : 2); ++x) {
    const std::string p = encs[x];
    for (const char* s : {"patch.w", "patch.b", "pos.patch", "pos.cls", "norm.g", "norm.b"}) need.push_back(p + s);
    for (int i = 0; i < c.depth; ++i)
      for (const char* s : {"ln1.g", "ln1.b", "qkv.w", "qkv.b", "proj.w", "proj.b", "ls1", "ln2.g", "ln2.b",
                            "fc1.w", "fc1.b", "fc2.w", "fc2.b", "ls2"})
        need.push_back(p + "b" + std::to_string(i) + "." + s);
  }
  for (const char* s : {"img.up.w", "img.up.b", "fuse.w", "fuse.b", "s0.proj.w", "s0.up.w", "s1.proj.w", "s1.up.w",
                        "s2.proj.w", "s2.up.w", "h0.proj.w", "h0.up0.w", "h0.up1.w", "h1.proj.w", "h1.up0.w",
                        "h1.up1.w", "h1.up2.w", "prj0.w", "prj1.w", "prj2.w", "prj3.w", "fs4.out.w", "fs4.out.b",
                        "head.c1.w", "head.c1.b", "head.up.w", "head.up.b", "head.c2.w", "head.c2.b", "head.c3.w",
                        "head.c3.b"})
    need.push_back(s);
  if (c.inter_dims[1] != c.features) need.push_back("prj4.w");
  for (int l = 0; l < 5; ++l) {
    const std::string p = "fs" + std::to_string(l) + ".";
    for (int u = 1; u <= 2; ++u)
      for (int cc = 1; cc <= 2; ++cc) {
        if (l == 0 && u == 1) continue;  // the first layer has no residual input
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + ".w");
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + ".b");
      }
    if (l < 4) {
      need.push_back(p + "up.w");
      need.push_back(p + "up.b");
    }
  }
  if (c.use_fov)
    for (const char* s : {"fov.neck.w", "fov.neck.b", "fov.conv.w", "fov.conv.b", "fov.h0.w", "fov.h0.b",
                          "fov.h1.w", "fov.h1.b", "fov.final.w", "fov.final.b"})
      need.push_back(s);
  for (auto& s : need)
    if (!e->get(s)) return "packed Depth Pro engine lacks tensor '" + s + "'";
  return "";
}

size_t plan_arena_dp(const mde_engine& e, int B, DPBuf* b, uint8_t* base) {
  ArenaPlan a(base);
  const PackConfig& c = e.cfg;
  const size_t bb = (size_t)B, G = (size_t)e.G, GG = G * G, D = (size_t)e.D, F = (size_t)e.F;
  const size_t ns = bb * e.nseq, T = (size_t)e.T;
  const size_t sd0 = c.scaled_dims[0], sd1 = c.scaled_dims[1], sd2 = c.scaled_dims[2];
  const size_t id0 = c.inter_dims[0], id1 = c.inter_dims[1];
  auto sq = [&](size_t k) { return k * k * GG; };  // pixels of a (k G)^2 map
  DPBuf t{};
  t.P = a.h(ns * GG * 768);
  t.Xp = a.f(ns * T * D);
  t.Xi = a.f(bb * T * D);
  t.Xf = c.use_fov ? a.f(bb * T * D) : nullptr;
  t.Hn = a.h(ns * T * D);
  t.O = a.h(ns * T * D);
  t.Q = a.h(ns * e.H * e.Tpad * 64);
  t.K = a.h(ns * e.H * e.Tpad * 64);
  t.Vt = a.h(ns * e.H * e.Tpad * 64);
  t.Mh = a.h(ns * T * c.mlp_hidden);
  for (int i = 0; i < 2; ++i) t.hook[i] = a.h(bb * sq(4) * D);
  t.lev[0] = a.h(bb * sq(4) * D);  // high (4G)
  t.lev[1] = a.h(bb * sq(2) * D);  // med (2G)
  t.lev[2] = a.h(bb * sq(1) * D);  // low (G)
  t.im = a.h(bb * GG * D);
  t.fm = c.use_fov ? a.h(bb * GG * D) : nullptr;
  t.fovf = c.use_fov ? a.h(bb * GG * (F / 2)) : nullptr;
  const size_t tmp = std::max({sq(1) * sd0, sq(2) * sd1, sq(4) * std::max({sd2, F, id1}), sq(16) * id1});
  t.tmp = a.h(bb * tmp);
  t.tmp2 = a.h(bb * sq(8) * std::max(id0, id1));
  t.gcat = a.h(bb * sq(2) * 2 * sd0);
  t.glob = a.h(bb * sq(2) * sd0);
  t.f1 = a.h(bb * sq(4) * sd1);
  t.f2 = a.h(bb * sq(8) * sd2);
  t.i0 = a.h(bb * sq(16) * id0);
  t.i1 = a.h(bb * sq(32) * id1);
  const size_t k[5] = {2, 4, 8, 16, 32};
  for (int i = 0; i < 4; ++i) t.pr[i] = a.h(bb * sq(k[i]) * F);
  t.pr[4] = (id1 == F) ? t.i1 : a.h(bb * sq(32) * F);
  t.h0 = a.h(bb * sq(32) * F);
  t.h1 = a.h(bb * sq(32) * F);
  t.tb = a.h(bb * sq(32) * F);
  t.sb = a.h(bb * sq(32) * F);
  t.ub = a.h(bb * sq(32) * F);
  t.c1 = a.h(bb * sq(32) * (F / 2));
  t.ct = a.h(bb * sq(64) * (F / 2));
  if (c.use_fov) {
    t.fv1 = a.h(bb * GG * (F / 2));
    t.fv2 = a.h(bb * (GG / 4) * (F / 4));
    t.fv3 = a.h(bb * (GG / 16) * (F / 8));
  }
  t.sws = a.f(kSplitWsAlloc);
  if (b) *b = t;
  return a.off;
}

// One DINOv2 encoder over nseq sequences of T tokens whose patch rows are P
// (nseq * G^2 rows of 768).  Hooks (patch encoder only): after block
// hooks[k], the raw residual stream of the first hook_seqs sequences (the
// high-res level) is merged into d.hook[k].
void Runner::dp_encoder(const std::string& pfx, float* X, const h16* P, int nseq, int hook_seqs) {
  mde_engine& e = *c.e;
  const PackConfig& cf = e.cfg;
  DPBuf& d = c.d;
  const int D = e.D, T = e.T, G = e.G, GG = G * G;
  char nm[96];
  snprintf(nm, sizeof nm, "%scls", pfx.c_str());
  step(nm, [&] { return launch_cls_rows(X, w32(pfx + "pos.cls"), nseq, T, D, st); });
  {
    GemmParams g = dense(P, 768, pfx + "patch.w", nseq * GG, D, 768);
    g.emode = E_PATCH;
    g.bias = w32(pfx + "patch.b");
    g.x32 = X;
    g.ldo = D;
    g.T = T;
    g.pos = w32(pfx + "pos.patch");
    g.npatch = GG;
    snprintf(nm, sizeof nm, "%spatch_embed", pfx.c_str());
    gemm(nm, g);
  }
  for (int i = 0; i < cf.depth; ++i) {
    const std::string p = pfx + "b" + std::to_string(i) + ".";
    snprintf(nm, sizeof nm, "%sblock%d.norm1", pfx.c_str(), i);
    step(nm, [&] {
      return launch_layernorm(X, d.Hn, w32(p + "ln1.g"), w32(p + "ln1.b"), nseq * T, D, cf.ln_eps, T, 0, st);
    });
    {
      GemmParams g = dense(d.Hn, D, p + "qkv.w", nseq * T, 3 * D, D);
      g.emode = E_QKV;
      g.bias = w32(p + "qkv.b");
      g.q = d.Q;
      g.k = d.K;
      g.vt = d.Vt;
      g.T = T;
      g.Tpad = e.Tpad;
      g.heads = e.H;
      g.qscale = 0.125f * 1.4426950408889634f;  // dh^-0.5 * log2(e)
      snprintf(nm, sizeof nm, "%sblock%d.qkv", pfx.c_str(), i);
      gemm(nm, g);
    }
    snprintf(nm, sizeof nm, "%sblock%d.attn", pfx.c_str(), i);
    step(nm, [&] { return launch_attention(d.Q, d.K, d.Vt, d.O, nseq, e.H, T, e.Tpad, D, st); });
    {
      GemmParams g = dense(d.O, D, p + "proj.w", nseq * T, D, D);
      g.emode = E_RESID;
      g.bias = w32(p + "proj.b");
      g.ls = w32(p + "ls1");
      g.x32 = X;
      g.ldo = D;
      snprintf(nm, sizeof nm, "%sblock%d.proj", pfx.c_str(), i);
      gemm(nm, g);
    }
    snprintf(nm, sizeof nm, "%sblock%d.norm2", pfx.c_str(), i);
    step(nm, [&] {
      return launch_layernorm(X, d.Hn, w32(p + "ln2.g"), w32(p + "ln2.b"), nseq * T, D, cf.ln_eps, T, 0, st);
    });
    {
      GemmParams g = dense(d.Hn, D, p + "fc1.w", nseq * T, cf.mlp_hidden, D);
      g.emode = E_STORE;
      g.bias = w32(p + "fc1.b");
      g.act = ACT_GELU;
      g.out16 = d.Mh;
      g.ldo = cf.mlp_hidden;
      snprintf(nm, sizeof nm, "%sblock%d.fc1", pfx.c_str(), i);
      gemm(nm, g);
    }
    {
      GemmParams g = dense(d.Mh, cf.mlp_hidden, p + "fc2.w", nseq * T, D, cf.mlp_hidden);
      g.emode = E_RESID;
      g.bias = w32(p + "fc2.b");
      g.ls = w32(p + "ls2");
      g.x32 = X;
      g.ldo = D;
      snprintf(nm, sizeof nm, "%sblock%d.fc2", pfx.c_str(), i);
      gemm(nm, g);
    }
    for (int k = 0; k < 2 && hook_seqs > 0; ++k) {
      if (cf.hooks[k] != i) continue;
      DpMerge m;
      m.B = nseq / e.nseq;
      m.n = e.lev_n[0];
      m.G = G;
      m.pad = e.lev_pad[0];
      m.base = e.lev_base[0];
      m.T = T;
      h16* dst = d.hook[k];
      snprintf(nm, sizeof nm, "%shook%d.merge", pfx.c_str(), k);
      step(nm, [&] { return launch_merge_tokens(X, dst, nullptr, nullptr, D, m, cf.ln_eps, st); });
    }
  }
}

hipError_t Runner::forward_dp(int B, const float* img, float* out, float* fov) {
  mde_engine& e = *c.e;
  const PackConfig& cf = e.cfg;
  DPBuf& d = c.d;
  const int D = e.D, G = e.G, F = e.F, T = e.T, S = cf.img_h;
  const int sd0 = cf.scaled_dims[0], sd1 = cf.scaled_dims[1], sd2 = cf.scaled_dims[2];
  const int id0 = cf.inter_dims[0], id1 = cf.inter_dims[1];
  const int ns = B * e.nseq;
  split_ws = d.sws;

  // ---- encoders ----
  {
    DpPyramid pyr;
    pyr.nlev = 3;
    pyr.nseq = e.nseq;
    for (int i = 0; i < 3; ++i) {
      pyr.first[i] = e.lev_base[i];
      pyr.n[i] = e.lev_n[i];
      pyr.stride[i] = e.lev_stride[i];
      pyr.f[i] = e.lev_f[i];
    }
    step("pyramid_patches", [&] { return launch_dp_patch_prep(img, d.P, B, S, G, pyr, st); });
  }
  dp_encoder("pe.", d.Xp, d.P, ns, B * e.lev_n[0] * e.lev_n[0]);
  auto merge = [&](const char* name, const float* X, h16* dst, const std::string& enc, int lev, int nb) {
    DpMerge m;
    m.B = nb;
    m.n = e.lev_n[lev];
    m.G = G;
    m.pad = e.lev_pad[lev];
    m.base = e.lev_base[lev];
    m.T = T;
    step(name, [&] {
      return launch_merge_tokens(X, dst, w32(enc + "norm.g"), w32(enc + "norm.b"), D, m, cf.ln_eps, st);
    });
  };
  merge("pe.merge_high", d.Xp, d.lev[0], "pe.", 0, B);
  merge("pe.merge_med", d.Xp, d.lev[1], "pe.", 1, B);
  merge("pe.merge_low", d.Xp, d.lev[2], "pe.", 2, B);
  // image / fov encoders: the x0.25 image IS the low-res level's single patch,
  // whose patch rows are the last B sequences of P
  const h16* Plow = d.P + (size_t)e.lev_base[2] * B * G * G * 768;
  auto single = [&](const char* name, const float* X, h16* dst, const std::string& enc) {
    DpMerge m;
    m.B = B;
    m.n = 1;
    m.G = G;
    m.pad = 0;
    m.base = 0;
    m.T = T;
    step(name, [&] {
      return launch_merge_tokens(X, dst, w32(enc + "norm.g"), w32(enc + "norm.b"), D, m, cf.ln_eps, st);
    });
  };
  dp_encoder("ie.", d.Xi, Plow, B, 0);
  single("ie.merge", d.Xi, d.im, "ie.");
  if (cf.use_fov) {
    dp_encoder("fe.", d.Xf, Plow, B, 0);
    single("fe.merge", d.Xf, d.fm, "fe.");
  }

  // ---- neck: upsample blocks ----
  {
    GemmParams g = convt2(d.im, B, G, G, D, "img.up.w", sd0, d.gcat + sd0, 2 * sd0);
    g.bias = w32("img.up.b");
    gemm("neck.image_block", g);
  }
  auto proj1x1 = [&](const char* name, const h16* in, int npix, int cin, const std::string& wn, int cout,
                     h16* dst) {
    GemmParams g = dense(in, cin, wn, npix, cout, cin);
    g.emode = E_STORE;
    g.out16 = dst;
    g.ldo = cout;
    gemm(name, g);
  };
  proj1x1("neck.scaled0.proj", d.lev[2], B * G * G, D, "s0.proj.w", sd0, d.tmp);
  gemm("neck.scaled0.up", convt2(d.tmp, B, G, G, sd0, "s0.up.w", sd0, d.gcat, 2 * sd0));
  {
    GemmParams g = dense(d.gcat, 2 * sd0, "fuse.w", B * 4 * G * G, sd0, 2 * sd0);
    g.emode = E_STORE;
    g.bias = w32("fuse.b");
    g.out16 = d.glob;
    g.ldo = sd0;
    gemm("neck.fuse_image_with_low_res", g);
  }
  proj1x1("neck.scaled1.proj", d.lev[1], B * 4 * G * G, D, "s1.proj.w", sd1, d.tmp);
  gemm("neck.scaled1.up", convt2(d.tmp, B, 2 * G, 2 * G, sd1, "s1.up.w", sd1, d.f1, sd1));
  proj1x1("neck.scaled2.proj", d.lev[0], B * 16 * G * G, D, "s2.proj.w", sd2, d.tmp);
  gemm("neck.scaled2.up", convt2(d.tmp, B, 4 * G, 4 * G, sd2, "s2.up.w", sd2, d.f2, sd2));
  // intermediate[0] (hook hooks[0]): proj -> 2 ConvT; intermediate[1]: proj -> 3 ConvT
  proj1x1("neck.inter0.proj", d.hook[0], B * 16 * G * G, D, "h0.proj.w", F, d.tmp);
  gemm("neck.inter0.up0", convt2(d.tmp, B, 4 * G, 4 * G, F, "h0.up0.w", id0, d.tmp2, id0));
  gemm("neck.inter0.up1", convt2(d.tmp2, B, 8 * G, 8 * G, id0, "h0.up1.w", id0, d.i0, id0));
  proj1x1("neck.inter1.proj", d.hook[1], B * 16 * G * G, D, "h1.proj.w", id1, d.tmp);
  gemm("neck.inter1.up0", convt2(d.tmp, B, 4 * G, 4 * G, id1, "h1.up0.w", id1, d.tmp2, id1));
  gemm("neck.inter1.up1", convt2(d.tmp2, B, 8 * G, 8 * G, id1, "h1.up1.w", id1, d.tmp, id1));
  gemm("neck.inter1.up2", convt2(d.tmp, B, 16 * G, 16 * G, id1, "h1.up2.w", id1, d.i1, id1));
  // ---- neck: 3x3 projections to F channels ----
  auto prj = [&](int i, const h16* in, int k, int cin) {
    GemmParams g = conv(in, B, k * G, k * G, cin, "prj" + std::to_string(i) + ".w", F, 1);
    g.out16 = d.pr[i];
    char nm[48];
    snprintf(nm, sizeof nm, "neck.projection%d", i);
    gemm(nm, g);
  };
  prj(0, d.glob, 2, sd0);
  prj(1, d.f1, 4, sd1);
  prj(2, d.f2, 8, sd2);
  prj(3, d.i0, 16, id0);
  if (id1 != F) prj(4, d.i1, 32, id1);

  // ---- fusion stage: 2G -> 32G ----
  h16* hin = d.pr[0];
  h16* hbuf[2] = {d.h0, d.h1};
  for (int l = 0; l < 5; ++l) {
    const int k = 2 << l;  // map side / G: 2, 4, 8, 16, 32
    const std::string p = "fs" + std::to_string(l);
    const h16* s = hin;
    if (l > 0) {
      rcu(p + ".rcu1", d.pr[l], hin, d.sb, d.tb, B, k * G, k * G, F);
      s = d.sb;
    }
    rcu(p + ".rcu2", s, nullptr, d.ub, d.tb, B, k * G, k * G, F);
    if (l < 4) {
      // deconv(2,2) + 1x1 projection, folded into one ConvT GEMM (+ projection bias)
      h16* hout = hbuf[l & 1];
      GemmParams g = convt2(d.ub, B, k * G, k * G, F, p + ".up.w", F, hout, F);
      g.bias = w32(p + ".up.b");
      gemm((p + ".up").c_str(), g);
      hin = hout;
    } else {
      GemmParams g = dense(d.ub, F, p + ".out.w", B * k * k * G * G, F, F);
      g.emode = E_STORE;
      g.bias = w32(p + ".out.b");
      g.out16 = hbuf[l & 1];
      g.ldo = F;
      gemm((p + ".out").c_str(), g);
      hin = hbuf[l & 1];
    }
  }

  // ---- head at 32G -> 64G ----
  {
    GemmParams g = conv(hin, B, 32 * G, 32 * G, F, "head.c1.w", F / 2, 1);
    g.bias = w32("head.c1.b");
    g.out16 = d.c1;
    gemm("head.conv1", g);
  }
  {
    GemmParams g = convt2(d.c1, B, 32 * G, 32 * G, F / 2, "head.up.w", F / 2, d.ct, F / 2);
    g.bias = w32("head.up.b");
    gemm("head.deconv", g);
  }
  {
    GemmParams g = conv(d.ct, B, S, S, F / 2, "head.c2.w", cf.head_hidden, 1);
    g.emode = E_HEAD;
    g.bias = w32("head.c2.b");
    g.w2 = w32("head.c3.w");
    g.b2 = e.head_b2;
    g.head_metric = 0;  // ReLU: canonical inverse depth
    g.out32 = out;
    gemm("head.conv2_conv3", g);
  }

  // ---- fov ----
  if (cf.use_fov) {
    {
      GemmParams g = dense(d.fm, D, "fov.neck.w", B * G * G, F / 2, D);
      g.emode = E_STORE;
      g.bias = w32("fov.neck.b");
      g.out16 = d.fovf;
      g.ldo = F / 2;
      gemm("fov.neck", g);
    }
    {
      GemmParams g = conv(d.pr[0], B, 2 * G, 2 * G, F, "fov.conv.w", F / 2, 2);
      g.bias = w32("fov.conv.b");
      g.act = ACT_RELU;
      g.res0 = d.fovf;  // fov_features + relu(conv(global))
      g.out16 = d.fv1;
      gemm("fov.conv", g);
    }
    {
      GemmParams g = conv(d.fv1, B, G, G, F / 2, "fov.h0.w", F / 4, 2);
      g.bias = w32("fov.h0.b");
      g.act = ACT_RELU;
      g.out16 = d.fv2;
      gemm("fov.head0", g);
    }
    {
      GemmParams g = conv(d.fv2, B, G / 2, G / 2, F / 4, "fov.h1.w", F / 8, 2);
      g.bias = w32("fov.h1.b");
      g.act = ACT_RELU;
      g.out16 = d.fv3;
      gemm("fov.head1", g);
    }
    const int K = cf.fov_k * cf.fov_k * (F / 8);
    step("fov.final", [&] { return launch_fov_final(d.fv3, w32("fov.final.w"), e.fov_b, K, B, fov, st); });
  }
  return err;
}

}  // namespace mde
