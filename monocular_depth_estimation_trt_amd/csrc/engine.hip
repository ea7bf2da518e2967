// libmde_hip engine: packed-weight loader, execution context and the DA-V2
// forward schedule, behind the C ABI of include/mde.h.  The Depth Pro
// schedule lives in depth_pro.hip, VGGT's in vggt.hip; all share
// engine_internal.h.
//
// Replaces TensorRT's ICudaEngine / IExecutionContext as used by the
// reference (core/common.py:141-312, core/common_runtime.py:131-275): one
// engine per device owns the packed weights; a context owns the activation
// arena (sized for its max batch) and runs the forward asynchronously on the
// caller's stream, replayed from a captured hipGraph per (batch, addresses).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "engine_internal.h"

using namespace mde;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return MDE_ERR_HIP;
}

#define HIP_OR(call, what)                         \
  do {                                             \
    hipError_t e_ = (call);                        \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

// DA-V2 load-time checks and derived geometry
std::string setup_dav2(mde_engine* e) {
  const PackConfig& c = e->cfg;
  if (c.patch != 14 || c.embed_dim % 64 || c.num_heads * 64 != c.embed_dim || c.img_h % 14 || c.img_w % 14 ||
      c.img_h <= 0 || c.img_w <= 0 || c.features % 16 || c.head_hidden != 32)
    return "unsupported model geometry in packed config";
  if (c.input_u8 != 0 && c.input_u8 != 1) return "bad input format in packed config";
  if (c.resid_f16 != 0 && c.resid_f16 != 1) return "bad residual precision in packed config";
  if (c.input_u8 && (c.in_scale == 0.f || c.in_std[0] == 0.f || c.in_std[1] == 0.f || c.in_std[2] == 0.f))
    return "uint8 input preamble with a zero scale/std";
  e->D = c.embed_dim;
  e->H = c.num_heads;
  e->F = c.features;
  e->ph = c.img_h / 14;
  e->pw = c.img_w / 14;
  e->np = e->ph * e->pw;
  e->T = e->np + 1;
  e->Tpad = (e->T + 63) / 64 * 64;
  e->h4 = (e->ph + 1) / 2;
  e->w4 = (e->pw + 1) / 2;
  e->c1p = (c.out_channels[0] + 31) / 32 * 32;
  // every tensor the forward uses must be present
  std::vector<std::string> need = {"patch.w", "patch.b", "pos.patch", "pos.cls", "norm.g", "norm.b",
                                   "rs0.w", "rs0.b", "rs1.w", "rs1.b", "rs3.w", "rs3.b",
                                   "head.c1.w", "head.c1.b", "head.c2.w", "head.c2.b", "head.c3.w", "head.c3.b"};
  if (c.enc_f32 != 0 && c.enc_f32 != 1) return "bad encoder precision in packed config";
  if (c.enc_f32) need[0] = "patch.w32";
  const char* wsuf = c.enc_f32 ? ".w32" : ".w";  // exact-fp32 encoders carry fp32 linears
  // exact-fp32 DPT head: fp32 head weights packed (round 5; a round-4 fp32
  // pack without them keeps the f16 head)
  e->head_f32 = c.enc_f32 && e->get("head.c1.w32") != nullptr;
  const char* hsuf = e->head_f32 ? ".w32" : ".w";
  if (e->head_f32) {
    if (c.out_channels[0] % 4 || c.out_channels[1] % 4 || c.out_channels[2] % 4 || c.out_channels[3] % 4 ||
        c.features % 8)
      return "unsupported DPT channel counts for the fp32 head";
    for (auto& n : need)
      if (n == "rs0.w" || n == "rs1.w" || n == "rs3.w" || n == "head.c1.w" || n == "head.c2.w") n += "32";
  }
  for (int i = 0; i < c.depth; ++i) {
    for (const char* s : {"ln1.g", "ln1.b", "qkv.b", "proj.b", "ls1", "ln2.g", "ln2.b", "fc1.b", "fc2.b", "ls2"})
      need.push_back("b" + std::to_string(i) + "." + s);
    for (const char* s : {"qkv", "proj", "fc1", "fc2"}) need.push_back("b" + std::to_string(i) + "." + s + wsuf);
  }
  for (int i = 0; i < 4; ++i) {
    need.push_back("proj" + std::to_string(i) + hsuf);
    need.push_back("proj" + std::to_string(i) + ".b");
    need.push_back("rn" + std::to_string(i + 1) + hsuf);
  }
  for (int r = 1; r <= 4; ++r) {
    std::string p = "rf" + std::to_string(r) + ".";
    need.push_back(p + "out" + hsuf);
    need.push_back(p + "out.b");
    for (int u = 1; u <= 2; ++u)
      for (int cc = 1; cc <= 2; ++cc) {
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + hsuf);
        need.push_back(p + "rcu" + std::to_string(u) + ".c" + std::to_string(cc) + ".b");
      }
  }
  for (auto& s : need)
    if (!e->get(s)) return "packed engine lacks tensor '" + s + "'";
  return "";
}

int load_pack(const uint8_t* data, size_t n, int device, mde_engine** out) {
  if (n < sizeof(PackHeader) + sizeof(PackConfig)) return fail(MDE_ERR_FORMAT, "packed engine truncated");
  PackHeader hd;
  memcpy(&hd, data, sizeof hd);
  if (memcmp(hd.magic, "MDEPACK1", 8) != 0) return fail(MDE_ERR_FORMAT, "bad magic (not an mde packed engine)");
  if (hd.version != kPackVersion)
    return fail(MDE_ERR_FORMAT, "packed engine version " + std::to_string(hd.version) + ", expected " +
                                    std::to_string(kPackVersion));
  const size_t tab = sizeof(PackHeader) + sizeof(PackConfig);
  if (tab + (size_t)hd.n_tensors * sizeof(PackTensor) > n || hd.data_offset + hd.data_bytes > n ||
      hd.data_offset < tab + (size_t)hd.n_tensors * sizeof(PackTensor))
    return fail(MDE_ERR_FORMAT, "packed engine tables out of range");
  auto* e = new mde_engine();
  e->device = device;
  memcpy(&e->cfg, data + sizeof(PackHeader), sizeof(PackConfig));
  e->family = e->cfg.family;
  if (e->family != FAMILY_DAV2 && e->family != FAMILY_DEPTH_PRO && e->family != FAMILY_VGGT) {
    delete e;
    return fail(MDE_ERR_FORMAT, "unknown model family in packed config");
  }
  for (uint32_t i = 0; i < hd.n_tensors; ++i) {
    PackTensor pt;
    memcpy(&pt, data + tab + (size_t)i * sizeof(PackTensor), sizeof pt);
    if (pt.offset + pt.nbytes > hd.data_bytes || pt.ndim < 1 || pt.ndim > 4) {
      delete e;
      return fail(MDE_ERR_FORMAT, "tensor record out of range");
    }
    DevTensor dt;
    dt.ptr = (void*)(uintptr_t)pt.offset;  // rebased after the upload
    dt.dtype = pt.dtype;
    dt.ndim = pt.ndim;
    for (int k = 0; k < 4; ++k) dt.dims[k] = pt.dims[k];
    pt.name[sizeof(pt.name) - 1] = 0;
    e->t[pt.name] = dt;
  }
  const std::string bad = e->family == FAMILY_DAV2        ? setup_dav2(e)
                          : e->family == FAMILY_DEPTH_PRO ? setup_depth_pro(e)
                                                          : setup_vggt(e);
  if (!bad.empty()) {
    delete e;
    return fail(MDE_ERR_FORMAT, bad);
  }
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) {
    delete e;
    return hip_fail(he, "hipSetDevice");
  }
  e->wbytes = hd.data_bytes;
  he = hipMalloc(&e->wmem, std::max<size_t>(hd.data_bytes, 256));
  if (he != hipSuccess) {
    delete e;
    return hip_fail(he, "hipMalloc(weights)");
  }
  he = hipMemcpy(e->wmem, data + hd.data_offset, hd.data_bytes, hipMemcpyHostToDevice);
  if (he != hipSuccess) {
    hipFree(e->wmem);
    delete e;
    return hip_fail(he, "hipMemcpy(weights)");
  }
  for (auto& kv : e->t) kv.second.ptr = (uint8_t*)e->wmem + (uintptr_t)kv.second.ptr;
  *out = e;
  return MDE_OK;
}

}  // namespace

namespace mde {

// ---- DA-V2 activation arena ---------------------------------------------------
// switch "lnfold" = 0 (tuning.h): norm1 / norm2 as LayerNorm launches + the
// unfolded linears (A/B, tests); read when a context is created
bool lnfold_off() { return knob(KNOB_LNFOLD) == 0; }

size_t plan_arena_dav2(const mde_engine& e, int B, DAV2Buf* b, uint8_t* base) {
  ArenaPlan a(base);
  const size_t bb = (size_t)B;
  const int D = e.D, F = e.F, np = e.np;
  const int* oc = e.cfg.out_channels;
  const size_t s1 = (size_t)(4 * e.ph) * (4 * e.pw), s2 = (size_t)(2 * e.ph) * (2 * e.pw), s3 = np,
               s4 = (size_t)e.h4 * e.w4;
  const size_t s0 = (size_t)(8 * e.ph) * (8 * e.pw);
  DAV2Buf t{};
  if (e.cfg.enc_f32) {
    // exact-fp32 encoder (fp32.hip): fp32 operands end to end; the f16
    // encoder scratch is not needed, the taps / DPT head below are shared
    const size_t rows = bb * e.T;
    t.X = a.f(rows * D);
    t.P32 = a.f(bb * np * 672);
    t.Hn32 = a.f(rows * D);
    t.Q32 = a.f(bb * e.H * e.Tpad * 64);
    t.K32 = a.f(bb * e.H * e.Tpad * 64);
    t.V32 = a.f(bb * e.H * e.Tpad * 64);
    t.O32 = a.f(rows * D);
    t.Mh32 = a.f(rows * e.cfg.mlp_hidden);
  }
  t.P = e.cfg.enc_f32 ? nullptr : a.h(bb * np * 672);
  // residual stream in f16 (precision "fp16": the fp32 update rounded once
  // per residual add, as an fp16 TensorRT engine computes it -- half the
  // bytes of every residual read-modify-write and LayerNorm read) or fp32
  if (e.cfg.enc_f32) {
    t.Xh = nullptr;
  } else if (e.cfg.resid_f16) {
    t.X = nullptr;
    t.Xh = a.h(bb * e.T * D);
  } else {
    t.X = a.f(bb * e.T * D);
    t.Xh = nullptr;
  }
  const bool h16enc = !e.cfg.enc_f32;  // the f16 encoder's scratch
  t.Hn = h16enc ? a.h(bb * e.T * D) : nullptr;
  // LayerNorm folded into qkv / fc1 (packs with the folded weights): the
  // residual writers leave per-32-column (sum, sum of squares) partials here
  const bool fold = h16enc && e.cfg.resid_f16 && D % 128 == 0 && D <= 1024 && e.get("pos.cls.st") && !lnfold_off();
  t.st = fold ? a.f(bb * e.T * (D / 16)) : nullptr;
  t.Q = h16enc ? a.h(bb * e.H * e.Tpad * 64) : nullptr;
  t.K = h16enc ? a.h(bb * e.H * e.Tpad * 64) : nullptr;
  t.Vt = h16enc ? a.h(bb * e.H * e.Tpad * 64) : nullptr;
  t.O = h16enc ? a.h(bb * e.T * D) : nullptr;
  t.Mh = h16enc ? a.h(bb * e.T * e.cfg.mlp_hidden) : nullptr;
  // tap token maps: only without the tap-LayerNorm fold (the projects read
  // the residual stream directly when proj*.wf is packed)
  const bool fold_taps = fold && e.get("proj0.wf");
  const size_t ss[4] = {s1, s2, s3, s4};
  if (!e.head_f32) {
    for (int i = 0; i < 4; ++i) t.tap[i] = fold_taps ? nullptr : a.h(bb * np * D);
    for (int i = 0; i < 4; ++i) t.pj[i] = a.h(bb * np * oc[i]);
    t.l1 = a.h(bb * s1 * e.c1p);  // channels padded to a multiple of 32 (pad stays 0)
    t.l2 = a.h(bb * s2 * oc[1]);
    t.l4 = a.h(bb * s4 * oc[3]);
    for (int i = 0; i < 4; ++i) t.rn[i] = a.h(bb * ss[i] * F);
    t.tb = a.h(bb * s1 * F);
    t.sb = a.h(bb * s1 * F);
    t.ub = a.h(bb * s1 * F);
    t.vb = a.h(bb * s1 * F);
    t.p4 = a.h(bb * s3 * F);
    t.p3 = a.h(bb * s2 * F);
    t.p2 = a.h(bb * s1 * F);
    t.c1 = a.h(bb * s0 * (F / 2));
  } else {
    // exact-fp32 DPT head: the same maps in fp32 (l1 unpadded: the fp32 conv
    // takes any channel count % 4), plus the upsampled head inputs
    const size_t sout = (size_t)e.cfg.img_h * e.cfg.img_w;
    for (int i = 0; i < 4; ++i) t.tap32[i] = a.f(bb * np * D);
    for (int i = 0; i < 4; ++i) t.pj32[i] = a.f(bb * np * oc[i]);
    t.l1_32 = a.f(bb * s1 * oc[0]);
    t.l2_32 = a.f(bb * s2 * oc[1]);
    t.l4_32 = a.f(bb * s4 * oc[3]);
    for (int i = 0; i < 4; ++i) t.rn32[i] = a.f(bb * ss[i] * F);
    t.tb32 = a.f(bb * s1 * F);
    t.sb32 = a.f(bb * s1 * F);
    t.ub32 = a.f(bb * s1 * F);
    t.vb32 = a.f(bb * s1 * F);
    t.p4_32 = a.f(bb * s3 * F);
    t.p3_32 = a.f(bb * s2 * F);
    t.p2_32 = a.f(bb * s1 * F);
    t.up1_32 = a.f(bb * s0 * F);
    t.c1_32 = a.f(bb * s0 * (F / 2));
    t.up2_32 = a.f(bb * sout * (F / 2));
    t.hid32 = a.f(bb * sout * 32);
  }
  t.ws = h16enc && bb * e.T <= 4096 ? a.f(fc2_ws_floats(bb * e.T, D)) : nullptr;
  // attention split-KV workspace for the batches whose (head, 128-query)
  // grid is under one workgroup per CU (launch_attention splits those)
  const int bsplit = std::min<int>(B, (256 + ((e.T + 127) / 128) * e.H - 1) / (((e.T + 127) / 128) * e.H));
  t.aws_bytes = h16enc && bsplit >= 1 ? attention_split_ws_bytes(bsplit, e.H, e.T) : 0;
  t.aws = t.aws_bytes ? a.f(t.aws_bytes / sizeof(float)) : nullptr;
  t.sws = a.f(kSplitWsAlloc);
  if (b) *b = t;
  return a.off;
}

}  // namespace mde

namespace {

size_t plan_arena(const mde_engine& e, int B, mde_context* c, uint8_t* base) {
  if (e.family == FAMILY_DEPTH_PRO) return plan_arena_dp(e, B, c ? &c->d : nullptr, base);
  if (e.family == FAMILY_VGGT) return plan_arena_vggt(e, B, c ? &c->v : nullptr, base);
  return plan_arena_dav2(e, B, c ? &c->b : nullptr, base);
}

}  // namespace

namespace mde {

// FeatureFusionBlock: [x0 + RCU1(x1)] -> RCU2 -> out_conv(1x1) -> resize.
// The 1x1 out_conv is applied BEFORE the bilinear resize (both are linear
// and bilinear weights sum to 1, so they commute exactly in real
// arithmetic); this runs the 1x1 GEMM on 4x fewer pixels.
// x0_up: x0 is the x2 resize of the previous block's 1x1 output (x0_up, uh x
// uw), not yet written -- read on the fly by rcu1's second conv (switch
// "resize_fold"; GemmParams::res1_up), or written into x0 by that launch when
// its conv route cannot.  Returns true when this block's own resize into dst
// is left to the next block that way.
bool Runner::dav2_fusion(int r, const h16* x0, const h16* x1, int B, int h, int w, h16* dst, int oh, int ow,
                         const h16* x0_up, int uh, int uw) {
  const std::string p = "rf" + std::to_string(r);
  const int F = c.e->F;
  const h16* s = x0;
  if (x1) {
    rcu(p + ".rcu1", x1, x0, c.b.sb, c.b.tb, B, h, w, F, false, x0_up, uh, uw);
    s = c.b.sb;
  }
  rcu(p + ".rcu2", s, nullptr, c.b.ub, c.b.tb, B, h, w, F);
  GemmParams g = dense(c.b.ub, F, p + ".out.w", B * h * w, F, F);
  g.emode = E_STORE;
  g.bias = w32(p + ".out.b");
  g.out16 = c.b.vb;
  g.ldo = F;
  gemm((p + ".out").c_str(), g);
  if (!dst) return false;
  if (knob(KNOB_RESIZE_FOLD)) return true;  // vb stays intact until the next block's rcu1 has read it
  step((p + ".resize").c_str(), [&] { return launch_resize(c.b.vb, dst, B, h, w, F, oh, ow, st); });
  return false;
}

// The exact-fp32 DPT head (precision "fp32" packs with fp32 head weights):
// the f16 head's schedule on fp32 maps and the fp32 GEMM (fp32.hip) --
// projects, resize layers (ConvT pixel shuffle / 3x3 s2), layerN_rn, the
// four fusion blocks (out_conv before the x2 resize, as the f16 head) and
// the depth head with its two bilinear upsamples materialised in fp32.
void Runner::dav2_head32(int B, float* out) {
  mde_engine& e = *c.e;
  const PackConfig& cf = e.cfg;
  const int D = e.D, np = e.np, F = e.F;
  const int* oc = cf.out_channels;
  DAV2Buf& b = c.b;
  const int hs[4] = {4 * e.ph, 2 * e.ph, e.ph, e.h4};
  const int ws[4] = {4 * e.pw, 2 * e.pw, e.pw, e.w4};
  const float* lay[4] = {b.l1_32, b.l2_32, b.pj32[2], b.l4_32};
  char nm[64];
  for (int i = 0; i < 4; ++i) {
    {
      Gemm32Params g = dense32(b.tap32[i], D, "proj" + std::to_string(i) + ".w32", B * np, oc[i], D);
      g.bias = w32("proj" + std::to_string(i) + ".b");
      g.out32 = b.pj32[i];
      g.ldo = oc[i];
      snprintf(nm, sizeof nm, "reassemble%d.project", i);
      gemm32(nm, g);
    }
    if (i == 0 || i == 1) {
      const int sc = i == 0 ? 4 : 2;
      Gemm32Params g = dense32(b.pj32[i], oc[i], i == 0 ? "rs0.w32" : "rs1.w32", B * np, sc * sc * oc[i], oc[i]);
      g.emode = E_CONVT;
      g.bias = w32(i == 0 ? "rs0.b" : "rs1.b");
      g.out32 = i == 0 ? b.l1_32 : b.l2_32;
      g.s = sc;
      g.cout = oc[i];
      g.ldo = oc[i];
      g.cb = B;
      g.ih = e.ph;
      g.iw = e.pw;
      gemm32(i == 0 ? "reassemble0.convT4" : "reassemble1.convT2", g);
    } else if (i == 3) {
      Gemm32Params g = conv32(b.pj32[3], B, e.ph, e.pw, oc[3], "rs3.w32", oc[3], 2);
      g.bias = w32("rs3.b");
      g.out32 = b.l4_32;
      gemm32("reassemble3.conv_s2", g);
    }
    Gemm32Params g = conv32(lay[i], B, hs[i], ws[i], oc[i], "rn" + std::to_string(i + 1) + ".w32", F, 1);
    g.out32 = b.rn32[i];
    snprintf(nm, sizeof nm, "layer%d_rn", i + 1);
    gemm32(nm, g);
  }
  // fusion: [x0 + RCU1(x1)] -> RCU2 -> out_conv (1x1) -> x2 resize
  auto fusion = [&](int r, const float* x0, const float* x1, int h, int w, float* dst, int oh, int ow) {
    const std::string p = "rf" + std::to_string(r);
    const float* s = x0;
    if (x1) {
      rcu32(p + ".rcu1", x1, x0, b.sb32, b.tb32, B, h, w, F);
      s = b.sb32;
    }
    rcu32(p + ".rcu2", s, nullptr, b.ub32, b.tb32, B, h, w, F);
    Gemm32Params g = dense32(b.ub32, F, p + ".out.w32", B * h * w, F, F);
    g.bias = w32(p + ".out.b");
    g.out32 = b.vb32;
    g.ldo = F;
    gemm32((p + ".out").c_str(), g);
    if (dst) step((p + ".resize").c_str(), [&] { return launch_resize32(b.vb32, dst, B, h, w, F, oh, ow, st); });
  };
  fusion(4, b.rn32[3], nullptr, hs[3], ws[3], b.p4_32, hs[2], ws[2]);
  fusion(3, b.p4_32, b.rn32[2], hs[2], ws[2], b.p3_32, hs[1], ws[1]);
  fusion(2, b.p3_32, b.rn32[1], hs[1], ws[1], b.p2_32, hs[0], ws[0]);
  fusion(1, b.p2_32, b.rn32[0], hs[0], ws[0], nullptr, 0, 0);  // 1x1 result in vb32 at hs[0] x ws[0]
  // head: x2 upsample -> output_conv1 -> upsample to the input size ->
  // output_conv2 (3x3 + ReLU, then 1x1 + activation)
  const int H1 = 2 * hs[0], W1 = 2 * ws[0], OH = cf.img_h, OW = cf.img_w;
  step("head.upsample1", [&] { return launch_resize32(b.vb32, b.up1_32, B, hs[0], ws[0], F, H1, W1, st); });
  {
    Gemm32Params g = conv32(b.up1_32, B, H1, W1, F, "head.c1.w32", F / 2, 1);
    g.bias = w32("head.c1.b");
    g.out32 = b.c1_32;
    gemm32("head.output_conv1", g);
  }
  step("head.upsample2", [&] { return launch_resize32(b.c1_32, b.up2_32, B, H1, W1, F / 2, OH, OW, st); });
  {
    Gemm32Params g = conv32(b.up2_32, B, OH, OW, F / 2, "head.c2.w32", cf.head_hidden, 1);
    g.bias = w32("head.c2.b");
    g.act = ACT_RELU;
    g.out32 = b.hid32;
    gemm32("head.output_conv2", g);
  }
  step("head.output_conv3", [&] {
    return launch_head32(b.hid32, w32("head.c3.w"), e.head_b2, B * OH * OW, cf.metric, cf.max_depth, out, st);
  });
}

hipError_t Runner::forward_dav2(int B, const void* img, float* out) {
  mde_engine& e = *c.e;
  const PackConfig& cf = e.cfg;
  const int D = e.D, T = e.T, np = e.np, F = e.F;
  const int* oc = cf.out_channels;
  DAV2Buf& b = c.b;

  const bool fold = b.st != nullptr;
  split_ws = b.sws;
  const float* cls_st = fold ? w32("pos.cls.st") : nullptr;
  if (!cf.enc_f32) {
  step("patch_prep", [&] {
    if (cf.input_u8)
      return launch_patch_prep_u8((const unsigned char*)img, b.P, b.Xh ? nullptr : b.X, w32("pos.cls"), B, cf.img_h,
                                  cf.img_w, e.ph, e.pw, T, D, cf.in_scale, cf.in_mean, cf.in_std, st, b.Xh, b.st,
                                  cls_st);
    return launch_patch_prep((const float*)img, b.P, b.X, w32("pos.cls"), B, cf.img_h, cf.img_w, e.ph, e.pw, T, D,
                             st, b.Xh, b.st, cls_st);
  });
  {
    GemmParams g = dense(b.P, 672, "patch.w", B * np, D, 672);
    g.emode = E_PATCH;
    g.bias = w32("patch.b");
    g.x32 = b.X;
    g.xh = b.Xh;
    g.ldo = D;
    g.T = T;
    g.pos = w32("pos.patch");
    g.npatch = np;
    if (fold) {
      g.lnst_out = b.st;
      g.lnst_ns = D / 32;
      g.lnst_rows = B * T;
    }
    gemm("patch_embed", g);
  }
  }  // !enc_f32
  // ---- DPT head: reassemble (project, resize layer) + layerN_rn of tap i ----
  const int hs[4] = {4 * e.ph, 2 * e.ph, e.ph, e.h4};
  const int ws[4] = {4 * e.pw, 2 * e.pw, e.pw, e.w4};
  const h16* lay[4] = {b.l1, b.l2, b.pj[2], b.l4};
  const int cin[4] = {e.c1p, oc[1], oc[2], oc[3]};
  char nm[64];
  // the taps' final LayerNorm folded into the projects (packs with proj*.wf):
  // each project runs right after its tap block, on the raw f16 residual rows
  // (cls rows skipped by the GEMM's row map) and that block's LN partials --
  // before the next block rewrites both -- with W * gamma, as qkv / fc1 do
  const bool fold_taps = fold && e.get("proj0.wf") != nullptr;
  auto project_folded = [&](int i) {
    const std::string pn = "proj" + std::to_string(i);
    GemmParams g = dense(b.Xh, D, pn + ".wf", B * np, oc[i], D);
    g.emode = E_STORE;
    g.bias = w32(pn + ".c2");
    g.out16 = b.pj[i];
    g.ldo = oc[i];
    g.lnst_in = b.st;
    g.lnc1 = w32(pn + ".c1");
    g.lnst_ns = D / 32;
    g.lnst_rows = B * T;
    g.ln_eps = cf.ln_eps;
    g.a_tok = T;
    snprintf(nm, sizeof nm, "reassemble%d.project", i);
    gemm(nm, g);
  };
  auto reassemble = [&](int i) {
    if (!fold_taps) {
      GemmParams g = dense(b.tap[i], D, "proj" + std::to_string(i) + ".w", B * np, oc[i], D);
      g.emode = E_STORE;
      g.bias = w32("proj" + std::to_string(i) + ".b");
      g.out16 = b.pj[i];
      g.ldo = oc[i];
      snprintf(nm, sizeof nm, "reassemble%d.project", i);
      gemm(nm, g);
    }
    if (i == 0) {
      GemmParams g = dense(b.pj[0], oc[0], "rs0.w", B * np, 16 * oc[0], oc[0]);
      g.emode = E_CONVT;
      g.bias = w32("rs0.b");
      g.out16 = b.l1;
      g.s = 4;
      g.cout = oc[0];
      g.ldo = e.c1p;
      g.ih = e.ph;
      g.iw = e.pw;
      gemm("reassemble0.convT4", g);
    } else if (i == 1) {
      GemmParams g = dense(b.pj[1], oc[1], "rs1.w", B * np, 4 * oc[1], oc[1]);
      g.emode = E_CONVT;
      g.bias = w32("rs1.b");
      g.out16 = b.l2;
      g.s = 2;
      g.cout = oc[1];
      g.ldo = oc[1];
      g.ih = e.ph;
      g.iw = e.pw;
      gemm("reassemble1.convT2", g);
    } else if (i == 3) {
      GemmParams g = conv(b.pj[3], B, e.ph, e.pw, oc[3], "rs3.w", oc[3], 2);
      g.bias = w32("rs3.b");
      g.out16 = b.l4;
      gemm("reassemble3.conv_s2", g);
    }
    GemmParams g = conv(lay[i], B, hs[i], ws[i], cin[i], "rn" + std::to_string(i + 1) + ".w", F, 1);
    g.out16 = b.rn[i];
    snprintf(nm, sizeof nm, "layer%d_rn", i + 1);
    gemm(nm, g);
  };
  int tap = 0;
  if (cf.enc_f32) {
    // ---- exact-fp32 encoder (fp32.hip): every encoder operand fp32, the taps'
    // final LayerNorm writes the f16 NHWC token maps the DPT head reads ----
    step("patch_prep", [&] {
      if (cf.input_u8)
        return launch_patch_prep_u8((const unsigned char*)img, nullptr, b.X, w32("pos.cls"), B, cf.img_h, cf.img_w,
                                    e.ph, e.pw, T, D, cf.in_scale, cf.in_mean, cf.in_std, st, nullptr, nullptr,
                                    nullptr, b.P32);
      return launch_patch_prep((const float*)img, nullptr, b.X, w32("pos.cls"), B, cf.img_h, cf.img_w, e.ph, e.pw, T,
                               D, st, nullptr, nullptr, nullptr, b.P32);
    });
    {
      Gemm32Params g = dense32(b.P32, 672, "patch.w32", B * np, D, 672);
      g.emode = E_PATCH;
      g.bias = w32("patch.b");
      g.x32 = b.X;
      g.ldo = D;
      g.T = T;
      g.pos = w32("pos.patch");
      g.npatch = np;
      gemm32("patch_embed", g);
    }
    for (int i = 0; i < cf.depth; ++i) {
      const std::string p = "b" + std::to_string(i) + ".";
      snprintf(nm, sizeof nm, "block%d.norm1", i);
      step(nm, [&] { return launch_layernorm32(b.X, b.Hn32, w32(p + "ln1.g"), w32(p + "ln1.b"), B * T, D, cf.ln_eps, st); });
      {
        Gemm32Params g = dense32(b.Hn32, D, p + "qkv.w32", B * T, 3 * D, D);
        g.emode = E_QKV;
        g.bias = w32(p + "qkv.b");
        g.q = b.Q32;
        g.k = b.K32;
        g.v = b.V32;
        g.T = T;
        g.Tpad = e.Tpad;
        g.heads = e.H;
        g.qscale = 0.125f * 1.4426950408889634f;  // dh^-0.5 * log2(e): scores in log2 units
        snprintf(nm, sizeof nm, "block%d.qkv", i);
        gemm32(nm, g);
      }
      snprintf(nm, sizeof nm, "block%d.attn", i);
      step(nm, [&] { return launch_attention32(b.Q32, b.K32, b.V32, b.O32, B, e.H, T, e.Tpad, D, st); });
      {
        Gemm32Params g = dense32(b.O32, D, p + "proj.w32", B * T, D, D);
        g.emode = E_RESID;
        g.bias = w32(p + "proj.b");
        g.ls = w32(p + "ls1");
        g.x32 = b.X;
        g.ldo = D;
        snprintf(nm, sizeof nm, "block%d.proj", i);
        gemm32(nm, g);
      }
      snprintf(nm, sizeof nm, "block%d.norm2", i);
      step(nm, [&] { return launch_layernorm32(b.X, b.Hn32, w32(p + "ln2.g"), w32(p + "ln2.b"), B * T, D, cf.ln_eps, st); });
      {
        Gemm32Params g = dense32(b.Hn32, D, p + "fc1.w32", B * T, cf.mlp_hidden, D);
        g.emode = E_STORE;
        g.bias = w32(p + "fc1.b");
        g.act = ACT_GELU;
        g.out32 = b.Mh32;
        g.ldo = cf.mlp_hidden;
        snprintf(nm, sizeof nm, "block%d.fc1", i);
        gemm32(nm, g);
      }
      {
        Gemm32Params g = dense32(b.Mh32, cf.mlp_hidden, p + "fc2.w32", B * T, D, cf.mlp_hidden);
        g.emode = E_RESID;
        g.bias = w32(p + "fc2.b");
        g.ls = w32(p + "ls2");
        g.x32 = b.X;
        g.ldo = D;
        snprintf(nm, sizeof nm, "block%d.fc2", i);
        gemm32(nm, g);
      }
      if (tap < 4 && cf.taps[tap] == i) {
        snprintf(nm, sizeof nm, "tap%d.norm", tap);
        if (e.head_f32) {
          float* dst = b.tap32[tap];
          step(nm, [&] {
            return launch_layernorm32(b.X, dst, w32("norm.g"), w32("norm.b"), B * T, D, cf.ln_eps, st, T, 1);
          });
        } else {
          h16* dst = b.tap[tap];
          step(nm, [&] { return launch_layernorm(b.X, dst, w32("norm.g"), w32("norm.b"), B * T, D, cf.ln_eps, T, 1, st); });
        }
        ++tap;
      }
    }
  } else {
  for (int i = 0; i < cf.depth; ++i) {
    const std::string p = "b" + std::to_string(i) + ".";
    const std::string pn = "b" + std::to_string(i + 1) + ".";
    // small batch: fc2's 64^2 tiles do not fill the chip and each walks a
    // K = 4D loop -- split K (B = 1: ViT-S 132 tiles x 4, ViT-L 352 x 2;
    // ViT-L fc2 1.23 -> 0.88 ms per forward; proj at K = 1024 gained
    // nothing); switch "splitk" = 0 turns it off (A/B, tests)
    auto split_k = [&](GemmParams& g, int K) {
      const long long t64 = (long long)((B * T + 63) / 64) * ((D + 63) / 64);
      if (b.ws && t64 < 512 && K >= 1024 && knob(KNOB_SPLITK)) {
        g.partial = b.ws;
        g.splitk = t64 < 256 ? 4 : 2;
        g.slot_cap = fc2_ws_floats((size_t)B * T, D);
        g.tile_cnt = split_counters(b.sws);
        g.tile_cnt_cap = kTileCnt;
      }
    };
    // LayerNorm folded across the GEMM boundary (packs with folded weights):
    // the consumer reads the raw f16 residual rows with W * gamma and the
    // producers' row partials (GemmParams::lnst_in); otherwise a LayerNorm launch
    auto ln_fold = [&](GemmParams& g, const std::string& w) {
      g.A = b.Xh;
      g.lda = D;
      g.W = w16(p + w + ".wf");
      g.ldw = ldw(p + w + ".wf");
      g.bias = w32(p + w + ".c2");
      g.lnst_in = b.st;
      g.lnc1 = w32(p + w + ".c1");
      g.lnst_ns = D / 32;
      g.lnst_rows = B * T;
      g.ln_eps = cf.ln_eps;
    };
    if (!fold) {
      snprintf(nm, sizeof nm, "block%d.norm1", i);
      step(nm, [&] {
        return launch_layernorm(b.X, b.Hn, w32(p + "ln1.g"), w32(p + "ln1.b"), B * T, D, cf.ln_eps, T, 0, st, b.Xh);
      });
    }
    {
      GemmParams g = dense(b.Hn, D, p + "qkv.w", B * T, 3 * D, D);
      g.emode = E_QKV;
      g.bias = w32(p + "qkv.b");
      g.q = b.Q;
      g.k = b.K;
      g.vt = b.Vt;
      g.T = T;
      g.Tpad = e.Tpad;
      g.heads = e.H;
      g.qscale = 0.125f * 1.4426950408889634f;  // dh^-0.5 * log2(e): scores in log2 units
      if (fold) ln_fold(g, "qkv");
      snprintf(nm, sizeof nm, "block%d.qkv", i);
      gemm(nm, g);
    }
    snprintf(nm, sizeof nm, "block%d.attn", i);
    step(nm, [&] { return launch_attention(b.Q, b.K, b.Vt, b.O, B, e.H, T, e.Tpad, D, st, b.aws, b.aws_bytes); });
    {
      GemmParams g = dense(b.O, D, p + "proj.w", B * T, D, D);
      g.emode = E_RESID;
      g.bias = w32(p + "proj.b");
      g.ls = w32(p + "ls1");
      g.x32 = b.X;
      g.xh = b.Xh;
      g.ldo = D;
      if (fold) {
        g.lnst_out = b.st;
        g.lnst_ns = D / 32;
        g.lnst_rows = B * T;
      }
      snprintf(nm, sizeof nm, "block%d.proj", i);
      gemm(nm, g);
    }
    if (!fold) {
      snprintf(nm, sizeof nm, "block%d.norm2", i);
      step(nm, [&] {
        return launch_layernorm(b.X, b.Hn, w32(p + "ln2.g"), w32(p + "ln2.b"), B * T, D, cf.ln_eps, T, 0, st, b.Xh);
      });
    }
    {
      GemmParams g = dense(b.Hn, D, p + "fc1.w", B * T, cf.mlp_hidden, D);
      g.emode = E_STORE;
      g.bias = w32(p + "fc1.b");
      g.act = ACT_GELU;
      g.out16 = b.Mh;
      g.ldo = cf.mlp_hidden;
      if (fold) ln_fold(g, "fc1");
      snprintf(nm, sizeof nm, "block%d.fc1", i);
      gemm(nm, g);
    }
    {
      GemmParams g = dense(b.Mh, cf.mlp_hidden, p + "fc2.w", B * T, D, cf.mlp_hidden);
      g.emode = E_RESID;
      g.bias = w32(p + "fc2.b");
      g.ls = w32(p + "ls2");
      g.x32 = b.X;
      g.xh = b.Xh;
      g.ldo = D;
      split_k(g, cf.mlp_hidden);
      if (fold) {
        g.lnst_out = b.st;
        g.lnst_ns = D / 32;
        g.lnst_rows = B * T;
      }
      snprintf(nm, sizeof nm, "block%d.fc2", i);
      gemm(nm, g);
    }
    if (tap < 4 && cf.taps[tap] == i) {
      if (fold_taps) {
        project_folded(tap);
      } else {
        snprintf(nm, sizeof nm, "tap%d.norm", tap);
        h16* dst = b.tap[tap];
        step(nm, [&] {
          return launch_layernorm(b.X, dst, w32("norm.g"), w32("norm.b"), B * T, D, cf.ln_eps, T, 1, st, b.Xh);
        });
      }
      ++tap;
    }
  }
  }  // f16 encoder
  if (tap != 4) return hipErrorInvalidValue;
  if (e.head_f32) {
    dav2_head32(B, out);
    return err;
  }
  for (int i = 0; i < 4; ++i) reassemble(i);
  // ---- fusion (refinenet4 .. refinenet1) ----
  bool up = dav2_fusion(4, b.rn[3], nullptr, B, hs[3], ws[3], b.p4, hs[2], ws[2]);
  up = dav2_fusion(3, b.p4, b.rn[2], B, hs[2], ws[2], b.p3, hs[1], ws[1], up ? b.vb : nullptr, hs[3], ws[3]);
  up = dav2_fusion(2, b.p3, b.rn[1], B, hs[1], ws[1], b.p2, hs[0], ws[0], up ? b.vb : nullptr, hs[2], ws[2]);
  dav2_fusion(1, b.p2, b.rn[0], B, hs[0], ws[0], nullptr, 0, 0, up ? b.vb : nullptr, hs[1], ws[1]);  // 1x1 result in vb at hs[0] x ws[0]
  // ---- head ----
  const int H1 = 2 * hs[0], W1 = 2 * ws[0];  // refinenet1 upsample x2 (fused into output_conv1's loader)
  {
    GemmParams g;
    g.amode = A_CONV3_UP;
    g.emode = E_STORE;
    g.A = b.vb;
    g.cb = B;
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
    g.M = B * H1 * W1;
    g.N = F / 2;
    g.K = 9 * F;
    g.bias = w32("head.c1.b");
    g.out16 = b.c1;
    g.ldo = F / 2;
    gemm("head.output_conv1", g);
  }
  {
    const int OH = cf.img_h, OW = cf.img_w;  // (ph*14, pw*14)
    GemmParams g;
    g.amode = A_CONV3_UP;
    g.emode = E_HEAD;
    g.A = b.c1;
    g.cb = B;
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
    g.M = B * OH * OW;
    g.N = cf.head_hidden;
    g.K = 9 * (F / 2);
    g.bias = w32("head.c2.b");
    g.w2 = w32("head.c3.w");
    g.b2 = e.head_b2;
    g.head_metric = cf.metric;
    g.max_depth = cf.max_depth;
    g.out32 = out;
    gemm("head.output_conv2", g);
  }
  return err;
}

}  // namespace mde

namespace {

int check_ctx(const mde_context* c) {
  if (!c || !c->e) return fail(MDE_ERR_ARG, "null context");
  return MDE_OK;
}

const char* input_name(const mde_engine* e) {
  return e->family == FAMILY_VGGT ? "images" : e->cfg.input_u8 ? "image_u8" : "input";
}
bool is_input(const mde_engine* e, const char* n) { return n && strcmp(n, input_name(e)) == 0; }

// io binding index of a tensor name (0 = input, 1 = depth output, 2 = fov), -1 if unknown
int io_index(const mde_engine* e, const char* n) {
  if (!n) return -1;
  int nio = 0;
  mde_engine_num_io(e, &nio);
  for (int i = 0; i < nio; ++i) {
    mde_io_desc d;
    if (mde_engine_io_desc(e, i, &d) == MDE_OK && strcmp(d.name, n) == 0) return i;
  }
  return -1;
}

hipError_t run_forward(Runner& r, int B, const void* in, float* out, float* out2) {
  if (r.c.e->family == FAMILY_DEPTH_PRO) return r.forward_dp(B, (const float*)in, out, out2);
  if (r.c.e->family == FAMILY_VGGT) return r.forward_vggt(B, (const float*)in, out);
  return r.forward_dav2(B, in, out);
}

}  // namespace

// ============================== C ABI ======================================
extern "C" {

int mde_version(void) { return MDE_ABI_VERSION; }
const char* mde_last_error(void) { return g_err.c_str(); }

int mde_engine_load_memory(const void* data, size_t nbytes, int device, mde_engine** out) {
  if (!data || !out) return fail(MDE_ERR_ARG, "null argument");
  *out = nullptr;
  int rc = load_pack((const uint8_t*)data, nbytes, device, out);
  if (rc != MDE_OK) return rc;
  // the head's 1x1 bias scalar, stashed host-side for the kernel argument
  mde_engine* e = *out;
  hipError_t he = hipMemcpy(&e->head_b2, e->get("head.c3.b")->ptr, 4, hipMemcpyDeviceToHost);
  if (he == hipSuccess && e->family == FAMILY_DEPTH_PRO && e->cfg.use_fov)
    he = hipMemcpy(&e->fov_b, e->get("fov.final.b")->ptr, 4, hipMemcpyDeviceToHost);
  if (he != hipSuccess) {
    mde_engine_destroy(e);
    *out = nullptr;
    return hip_fail(he, "reading head bias");
  }
  return MDE_OK;
}

int mde_engine_load(const char* path, int device, mde_engine** out) {
  if (!path || !out) return fail(MDE_ERR_ARG, "null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(MDE_ERR_FILE, std::string("cannot open packed engine ") + path);
  std::vector<uint8_t> buf;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (n <= 0) {
    fclose(f);
    return fail(MDE_ERR_FILE, std::string("empty packed engine ") + path);
  }
  buf.resize((size_t)n);
  size_t got = fread(buf.data(), 1, (size_t)n, f);
  fclose(f);
  if (got != (size_t)n) return fail(MDE_ERR_FILE, std::string("short read of ") + path);
  return mde_engine_load_memory(buf.data(), buf.size(), device, out);
}

int mde_engine_destroy(mde_engine* e) {
  if (!e) return MDE_OK;
  hipSetDevice(e->device);
  if (e->wmem) hipFree(e->wmem);
  delete e;
  return MDE_OK;
}

int mde_engine_get_info(const mde_engine* e, mde_engine_info* o) {
  if (!e || !o) return fail(MDE_ERR_ARG, "null argument");
  memset(o, 0, sizeof *o);
  const PackConfig& c = e->cfg;
  memcpy(o->encoder, c.encoder, sizeof o->encoder);
  o->encoder[sizeof o->encoder - 1] = 0;
  o->embed_dim = c.embed_dim;
  o->depth = c.depth;
  o->num_heads = c.num_heads;
  o->mlp_hidden = c.mlp_hidden;
  o->patch = c.patch;
  o->img_h = c.img_h;
  o->img_w = c.img_w;
  o->features = c.features;
  o->head_hidden = c.head_hidden;
  o->metric = c.metric;
  for (int i = 0; i < 4; ++i) {
    o->out_channels[i] = c.out_channels[i];
    o->taps[i] = c.taps[i];
  }
  o->max_depth = c.max_depth;
  o->ln_eps = c.ln_eps;
  o->max_batch_hint = 64;
  o->weight_bytes = (int64_t)e->wbytes;
  o->input_format = c.input_u8 ? 1 : 0;
  o->family = e->family;
  return MDE_OK;
}

int mde_engine_num_io(const mde_engine* e, int* n) {
  if (!e || !n) return fail(MDE_ERR_ARG, "null argument");
  *n = (e->family == FAMILY_DEPTH_PRO && e->cfg.use_fov) ? 3 : 2;
  return MDE_OK;
}

int mde_engine_io_desc(const mde_engine* e, int index, mde_io_desc* o) {
  if (!e || !o) return fail(MDE_ERR_ARG, "null argument");
  memset(o, 0, sizeof *o);
  if (e->family == FAMILY_VGGT) {
    // reference input_names=["images"] [1,S,3,518,518], output_names=["depth"]
    // (models/vggt/onnx_export.py:101,125-127); S fixed at pack time
    if (index < 0 || index > 1) return fail(MDE_ERR_ARG, "io index out of range");
    o->dtype = MDE_FLOAT32;
    o->is_input = index == 0;
    o->rank = 5;
    o->dims[0] = -1;
    o->dims[1] = e->S;
    if (index == 0) {
      strcpy(o->name, "images");
      o->dims[2] = 3;
      o->dims[3] = e->cfg.img_h;
      o->dims[4] = e->cfg.img_w;
    } else {
      strcpy(o->name, "depth");
      o->dims[2] = e->cfg.img_h;
      o->dims[3] = e->cfg.img_w;
      o->dims[4] = 1;
    }
    return MDE_OK;
  }
  if (index == 0 && e->cfg.input_u8) {
    strcpy(o->name, "image_u8");
    o->dtype = MDE_UINT8;
    o->is_input = 1;
    o->rank = 4;
    o->dims[0] = -1;
    o->dims[1] = e->cfg.img_h;
    o->dims[2] = e->cfg.img_w;
    o->dims[3] = 3;
  } else if (index == 0) {
    strcpy(o->name, "input");
    o->dtype = MDE_FLOAT32;
    o->is_input = 1;
    o->rank = 4;
    o->dims[0] = -1;
    o->dims[1] = 3;
    o->dims[2] = e->cfg.img_h;
    o->dims[3] = e->cfg.img_w;
  } else if (index == 1 && e->family == FAMILY_DEPTH_PRO) {
    // reference output_names=["canonical_inverse_depth", "fov_deg"] (models/depth_pro/onnx_export.py:56),
    // output shape (1, 1, 1536, 1536) (onnx2trt.py:92)
    strcpy(o->name, "canonical_inverse_depth");
    o->dtype = MDE_FLOAT32;
    o->is_input = 0;
    o->rank = 4;
    o->dims[0] = -1;
    o->dims[1] = 1;
    o->dims[2] = e->cfg.img_h;
    o->dims[3] = e->cfg.img_w;
  } else if (index == 2 && e->family == FAMILY_DEPTH_PRO && e->cfg.use_fov) {
    strcpy(o->name, "fov_deg");
    o->dtype = MDE_FLOAT32;
    o->is_input = 0;
    o->rank = 1;
    o->dims[0] = -1;
  } else if (index == 1) {
    strcpy(o->name, "output");
    o->dtype = MDE_FLOAT32;
    o->is_input = 0;
    o->rank = 3;
    o->dims[0] = -1;
    o->dims[1] = e->cfg.img_h;
    o->dims[2] = e->cfg.img_w;
  } else {
    return fail(MDE_ERR_ARG, "io index out of range");
  }
  return MDE_OK;
}

int mde_engine_profile_shape(const mde_engine* e, const char* name, int which, int64_t* dims, int* rank) {
  if (!e || !name || !dims || !rank) return fail(MDE_ERR_ARG, "null argument");
  if (which < 0 || which > 2) return fail(MDE_ERR_ARG, "which must be 0 (min), 1 (opt) or 2 (max)");
  const int64_t bsel[3] = {1, 1, 64};
  mde_io_desc d;
  int idx = io_index(e, name);
  if (idx < 0) return fail(MDE_ERR_NAME, std::string("unknown tensor ") + name);
  mde_engine_io_desc(e, idx, &d);
  *rank = d.rank;
  for (int i = 0; i < d.rank; ++i) dims[i] = d.dims[i];
  dims[0] = bsel[which];
  return MDE_OK;
}

int mde_context_create(mde_engine* e, int max_batch, mde_context** out) {
  if (!e || !out || max_batch < 1) return fail(MDE_ERR_ARG, "bad argument to mde_context_create");
  *out = nullptr;
  HIP_OR(hipSetDevice(e->device), "hipSetDevice");
  auto* c = new mde_context();
  c->e = e;
  c->device = e->device;
  c->max_batch = max_batch;
  c->batch = 1;
  c->arena_bytes = plan_arena(*e, max_batch, nullptr, nullptr);
  hipError_t he = hipMalloc(&c->arena, c->arena_bytes);
  if (he != hipSuccess) {
    delete c;
    return hip_fail(he, "hipMalloc(activation arena)");
  }
  plan_arena(*e, max_batch, c, (uint8_t*)c->arena);
  // zero once: the q/k/v^T pad rows/columns beyond T must stay 0
  he = hipMemset(c->arena, 0, c->arena_bytes);
  if (he == hipSuccess) he = hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking);
  if (he == hipSuccess) he = hipDeviceSynchronize();
  if (he != hipSuccess) {
    hipFree(c->arena);
    delete c;
    return hip_fail(he, "context init");
  }
  *out = c;
  return MDE_OK;
}

int mde_context_destroy(mde_context* c) {
  if (!c) return MDE_OK;
  hipSetDevice(c->device);
  for (auto& kv : c->graphs) {
    hipGraphExecDestroy(kv.second.second);
    hipGraphDestroy(kv.second.first);
  }
  for (auto& kv : c->graph_done) hipEventDestroy(kv.second);
  for (auto& pe : c->prof_events) {
    hipEventDestroy(pe.second.first);
    hipEventDestroy(pe.second.second);
  }
  if (c->cap_stream) hipStreamDestroy(c->cap_stream);
  if (c->arena) hipFree(c->arena);
  delete c;
  return MDE_OK;
}

int mde_context_set_tensor_address(mde_context* c, const char* name, void* ptr) {
  if (int rc = check_ctx(c)) return rc;
  const int idx = io_index(c->e, name);
  if (idx == 0) c->in = ptr;
  else if (idx == 1) c->out = ptr;
  else if (idx == 2) c->out2 = ptr;
  else return fail(MDE_ERR_NAME, std::string("unknown tensor ") + (name ? name : "(null)"));
  return MDE_OK;
}

int mde_context_set_input_shape(mde_context* c, const char* name, const int64_t* dims, int rank) {
  if (int rc = check_ctx(c)) return rc;
  if (!is_input(c->e, name)) return fail(MDE_ERR_NAME, std::string("not an input: ") + (name ? name : "(null)"));
  const PackConfig& cf = c->e->cfg;
  if (c->e->family == FAMILY_VGGT) {
    const int S = c->e->S;
    if (!dims || rank != 5) return fail(MDE_ERR_SHAPE, "input shape must be rank 5 [B,S,3,H,W]");
    if (dims[1] != S || dims[2] != 3 || dims[3] != cf.img_h || dims[4] != cf.img_w)
      return fail(MDE_ERR_SHAPE, "input shape must be [B," + std::to_string(S) + ",3," + std::to_string(cf.img_h) +
                                     "," + std::to_string(cf.img_w) + "] for this engine");
  } else if (cf.input_u8) {
    if (!dims || rank != 4) return fail(MDE_ERR_SHAPE, "input shape must be rank 4 [B,H,W,3]");
    if (dims[3] != 3 || dims[1] != cf.img_h || dims[2] != cf.img_w)
      return fail(MDE_ERR_SHAPE, "input shape must be [B," + std::to_string(cf.img_h) + "," +
                                     std::to_string(cf.img_w) + ",3] for this engine");
  } else {
    if (!dims || rank != 4) return fail(MDE_ERR_SHAPE, "input shape must be rank 4 [B,3,H,W]");
    if (dims[1] != 3 || dims[2] != cf.img_h || dims[3] != cf.img_w)
      return fail(MDE_ERR_SHAPE, "input shape must be [B,3," + std::to_string(cf.img_h) + "," +
                                     std::to_string(cf.img_w) + "] for this engine");
  }
  if (dims[0] < 1 || dims[0] > c->max_batch)
    return fail(MDE_ERR_SHAPE, "batch " + std::to_string(dims[0]) + " outside [1, " +
                                   std::to_string(c->max_batch) + "]");
  c->batch = (int)dims[0];
  return MDE_OK;
}

int mde_context_get_tensor_shape(const mde_context* c, const char* name, int64_t* dims, int* rank) {
  if (int rc = check_ctx(c)) return rc;
  if (!dims || !rank) return fail(MDE_ERR_ARG, "null argument");
  mde_io_desc d;
  int idx = io_index(c->e, name);
  if (idx < 0) return fail(MDE_ERR_NAME, std::string("unknown tensor ") + (name ? name : "(null)"));
  mde_engine_io_desc(c->e, idx, &d);
  *rank = d.rank;
  for (int i = 0; i < d.rank; ++i) dims[i] = d.dims[i];
  dims[0] = c->batch;
  return MDE_OK;
}

int mde_context_set_graph_mode(mde_context* c, int enable) {
  if (int rc = check_ctx(c)) return rc;
  c->graph_mode = enable != 0;
  return MDE_OK;
}

int mde_context_set_profiler(mde_context* c, mde_layer_cb cb, void* user) {
  if (int rc = check_ctx(c)) return rc;
  c->prof_cb = cb;
  c->prof_user = user;
  return MDE_OK;
}

int mde_context_workspace_bytes(const mde_context* c, size_t* bytes) {
  if (int rc = check_ctx(c)) return rc;
  if (!bytes) return fail(MDE_ERR_ARG, "null argument");
  *bytes = c->arena_bytes;
  return MDE_OK;
}

int mde_context_enqueue(mde_context* c, void* stream) {
  if (int rc = check_ctx(c)) return rc;
  if (!c->in || !c->out) return fail(MDE_ERR_STATE, "set_tensor_address(input / output) before enqueue");
  int nio = 2;
  mde_engine_num_io(c->e, &nio);
  if (nio > 2 && !c->out2) return fail(MDE_ERR_STATE, "set_tensor_address('fov_deg') before enqueue");
  hipStream_t st = (hipStream_t)stream;
  HIP_OR(hipSetDevice(c->e->device), "hipSetDevice");
  const void* in = c->in;
  float* out = (float*)c->out;
  float* out2 = (float*)c->out2;
  if (c->prof_cb) {
    c->prof_used = 0;
    Runner r{*c, st, true};
    hipError_t he = run_forward(r, c->batch, in, out, out2);
    if (he != hipSuccess) return hip_fail(he, "enqueue (profiled)");
    HIP_OR(hipStreamSynchronize(st), "hipStreamSynchronize");
    for (size_t i = 0; i < c->prof_used; ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, c->prof_events[i].second.first, c->prof_events[i].second.second);
      c->prof_cb(c->prof_events[i].first.c_str(), ms, c->prof_user);
    }
    return MDE_OK;
  }
  // a caller capturing its own stream (its own hipGraph / torch.cuda.graph)
  // gets the forward's kernels captured straight into that graph: no graph of
  // ours is launched inside the capture, and none has to outlive it
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_OR(hipStreamIsCapturing(st, &cap), "hipStreamIsCapturing");
  if (!c->graph_mode || cap != hipStreamCaptureStatusNone) {
    Runner r{*c, st, false};
    hipError_t he = run_forward(r, c->batch, in, out, out2);
    if (he != hipSuccess) return hip_fail(he, "enqueue");
    return MDE_OK;
  }
  GraphKey key{c->batch, c->in, c->out, c->out2};
  auto it = c->graphs.find(key);
  if (it == c->graphs.end() && (int)c->graphs.size() >= mde_context::kMaxGraphs) {
    // evict the least recently launched graph; its last replay may still be
    // running on some caller stream: wait for that replay's event only (no
    // device-wide sync, which would also break a caller capturing its stream)
    auto lru = c->graph_used.begin();
    for (auto u = c->graph_used.begin(); u != c->graph_used.end(); ++u)
      if (u->second < lru->second) lru = u;
    auto done = c->graph_done.find(lru->first);
    if (done != c->graph_done.end()) {
      HIP_OR(hipEventSynchronize(done->second), "hipEventSynchronize (graph eviction)");
      hipEventDestroy(done->second);
      c->graph_done.erase(done);
    }
    auto victim = c->graphs.find(lru->first);
    hipGraphExecDestroy(victim->second.second);
    hipGraphDestroy(victim->second.first);
    c->graphs.erase(victim);
    c->graph_used.erase(lru);
  }
  if (it == c->graphs.end()) {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIP_OR(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    Runner r{*c, c->cap_stream, false};
    hipError_t he = run_forward(r, c->batch, in, out, out2);
    hipError_t he2 = hipStreamEndCapture(c->cap_stream, &g);
    if (he != hipSuccess) {
      if (g) hipGraphDestroy(g);
      return hip_fail(he, "capture forward");
    }
    if (he2 != hipSuccess) return hip_fail(he2, "hipStreamEndCapture");
    he = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (he != hipSuccess) {
      hipGraphDestroy(g);
      return hip_fail(he, "hipGraphInstantiate");
    }
    it = c->graphs.emplace(key, std::make_pair(g, ge)).first;
  }
  c->graph_used[key] = ++c->graph_tick;
  HIP_OR(hipGraphLaunch(it->second.second, st), "hipGraphLaunch");
  hipEvent_t& ev = c->graph_done[key];
  if (!ev) HIP_OR(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  HIP_OR(hipEventRecord(ev, st), "hipEventRecord");
  return MDE_OK;
}

// ---- runtime helpers --------------------------------------------------------
int mde_rt_device_count(int* n) {
  if (!n) return fail(MDE_ERR_ARG, "null argument");
  HIP_OR(hipGetDeviceCount(n), "hipGetDeviceCount");
  return MDE_OK;
}
int mde_rt_set_device(int d) {
  HIP_OR(hipSetDevice(d), "hipSetDevice");
  return MDE_OK;
}
int mde_rt_device_name(int d, char* buf, int len) {
  if (!buf || len <= 0) return fail(MDE_ERR_ARG, "null argument");
  hipDeviceProp_t p;
  HIP_OR(hipGetDeviceProperties(&p, d), "hipGetDeviceProperties");
  snprintf(buf, (size_t)len, "%s (%s)", p.name, p.gcnArchName);
  return MDE_OK;
}
int mde_rt_malloc(void** p, size_t n) {
  if (!p) return fail(MDE_ERR_ARG, "null argument");
  HIP_OR(hipMalloc(p, n), "hipMalloc");
  return MDE_OK;
}
int mde_rt_free(void* p) {
  HIP_OR(hipFree(p), "hipFree");
  return MDE_OK;
}
int mde_rt_malloc_host(void** p, size_t n) {
  if (!p) return fail(MDE_ERR_ARG, "null argument");
  HIP_OR(hipHostMalloc(p, n, hipHostMallocDefault), "hipHostMalloc");
  return MDE_OK;
}
int mde_rt_free_host(void* p) {
  HIP_OR(hipHostFree(p), "hipHostFree");
  return MDE_OK;
}
int mde_rt_memcpy_htod_async(void* d, const void* s, size_t n, void* st) {
  HIP_OR(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, (hipStream_t)st), "hipMemcpyAsync(H2D)");
  return MDE_OK;
}
int mde_rt_memcpy_dtoh_async(void* d, const void* s, size_t n, void* st) {
  HIP_OR(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, (hipStream_t)st), "hipMemcpyAsync(D2H)");
  return MDE_OK;
}
int mde_rt_memcpy_dtod_async(void* d, const void* s, size_t n, void* st) {
  HIP_OR(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, (hipStream_t)st), "hipMemcpyAsync(D2D)");
  return MDE_OK;
}
int mde_rt_memset_async(void* d, int v, size_t n, void* st) {
  HIP_OR(hipMemsetAsync(d, v, n, (hipStream_t)st), "hipMemsetAsync");
  return MDE_OK;
}
int mde_rt_stream_create(void** s) {
  if (!s) return fail(MDE_ERR_ARG, "null argument");
  hipStream_t st;
  HIP_OR(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  *s = st;
  return MDE_OK;
}
int mde_rt_stream_destroy(void* s) {
  HIP_OR(hipStreamDestroy((hipStream_t)s), "hipStreamDestroy");
  return MDE_OK;
}
int mde_rt_stream_synchronize(void* s) {
  HIP_OR(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  return MDE_OK;
}
int mde_rt_device_synchronize(void) {
  HIP_OR(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return MDE_OK;
}
int mde_rt_event_create(void** e) {
  if (!e) return fail(MDE_ERR_ARG, "null argument");
  hipEvent_t ev;
  HIP_OR(hipEventCreate(&ev), "hipEventCreate");
  *e = ev;
  return MDE_OK;
}
int mde_rt_event_destroy(void* e) {
  HIP_OR(hipEventDestroy((hipEvent_t)e), "hipEventDestroy");
  return MDE_OK;
}
int mde_rt_event_record(void* e, void* s) {
  HIP_OR(hipEventRecord((hipEvent_t)e, (hipStream_t)s), "hipEventRecord");
  return MDE_OK;
}
int mde_rt_event_elapsed_ms(float* ms, void* a, void* b) {
  if (!ms) return fail(MDE_ERR_ARG, "null argument");
  HIP_OR(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "hipEventElapsedTime");
  return MDE_OK;
}

// ---- kernel-level entry points ------------------------------------------------
#define OP_RET(call, what)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ == hipErrorInvalidValue) return fail(MDE_ERR_ARG, what ": invalid shape/argument"); \
    if (e_ != hipSuccess) return hip_fail(e_, what);          \
    return MDE_OK;                                           \
  } while (0)

int mde_op_patch_prep_u8(const unsigned char* img, int batch, int h, int w, float scale, const float* mean3,
                         const float* std3, void* patches, void* st) {
  if (!img || !mean3 || !std3 || !patches || batch < 1 || h % 14 || w % 14 || h < 14 || w < 14)
    return fail(MDE_ERR_ARG, "mde_op_patch_prep_u8: bad argument (h, w multiples of 14)");
  OP_RET(launch_patch_prep_u8(img, (h16*)patches, nullptr, nullptr, batch, h, w, h / 14, w / 14, 1, 0, scale, mean3,
                              std3, (hipStream_t)st),
         "patch_prep_u8");
}

int mde_op_depth_postprocess(const float* depth, int batch, int ih, int iw, float* out, int oh, int ow, float lo,
                             float hi, void* st) {
  if (!depth || !out || batch < 1 || ih < 1 || iw < 1 || oh < 1 || ow < 1)
    return fail(MDE_ERR_ARG, "mde_op_depth_postprocess: bad argument");
  OP_RET(launch_depth_postprocess(depth, batch, ih, iw, out, oh, ow, lo, hi, (hipStream_t)st), "depth_postprocess");
}

int mde_op_dp_pyramid_patches(const float* img, int batch, int size, void* patches, void* st) {
  if (!img || !patches || batch < 1 || size != 1536) return fail(MDE_ERR_ARG, "mde_op_dp_pyramid_patches: bad argument");
  DpPyramid pyr;
  pyr.nlev = 3;
  const int f[3] = {1, 2, 4}, n[3] = {5, 3, 1}, stride[3] = {288, 192, 384};
  int first = 0;
  for (int i = 0; i < 3; ++i) {
    pyr.first[i] = first;
    pyr.n[i] = n[i];
    pyr.stride[i] = stride[i];
    pyr.f[i] = f[i];
    first += n[i] * n[i];
  }
  pyr.nseq = first;
  OP_RET(launch_dp_patch_prep(img, (h16*)patches, batch, size, 24, pyr, (hipStream_t)st), "dp_pyramid_patches");
}

int mde_op_merge_tokens(const float* x32, int batch, int tokens, int dim, int n, int g, int pad, int base,
                        const float* gamma, const float* beta, float eps, void* out, void* st) {
  if (!x32 || !out || batch < 1 || (gamma == nullptr) != (beta == nullptr))
    return fail(MDE_ERR_ARG, "mde_op_merge_tokens: bad argument");
  DpMerge m;
  m.B = batch;
  m.n = n;
  m.G = g;
  m.pad = pad;
  m.base = base;
  m.T = tokens;
  OP_RET(launch_merge_tokens(x32, (h16*)out, gamma, beta, dim, m, eps, (hipStream_t)st), "merge_tokens");
}

int mde_op_qk_norm_rope(void* q, void* k, const float* qg, const float* qb, const float* kg, const float* kb, int bh,
                        int tokens, int tokens_pad, int frame_tokens, int npre, int grid_w, const float* rope_cos,
                        const float* rope_sin, float q_scale, float eps, void* st) {
  if (!q || !k || !qg || !qb || !kg || !kb || !rope_cos || !rope_sin) return fail(MDE_ERR_ARG, "null argument");
  RopeGeom geo;
  geo.T = tokens;
  geo.Tpad = tokens_pad;
  geo.P = frame_tokens;
  geo.npre = npre;
  geo.gw = grid_w;
  geo.qscale = q_scale;
  geo.eps = eps;
  OP_RET(launch_qk_norm_rope((h16*)q, (h16*)k, qg, qb, kg, kb, rope_cos, rope_sin, bh, geo, (hipStream_t)st),
         "qk_norm_rope");
}

int mde_op_tap_concat_ln(const float* xa, const float* xb, int nseq, int tokens, int npre, int dim, const float* g,
                         const float* b, float eps, void* out, void* st) {
  if (!xa || !xb || !g || !b || !out || nseq < 0) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_tap_concat_ln(xa, xb, (h16*)out, g, b, nseq, tokens, npre, dim, eps, (hipStream_t)st),
         "tap_concat_ln");
}

int mde_op_layernorm_f16(const void* x, void* y, const float* g, const float* b, int rows, int dim, float eps,
                         int tokens, int skip_cls, void* st) {
  if (!x || !y || !g || !b) return fail(MDE_ERR_ARG, "null argument");
  if (skip_cls && tokens < 2) return fail(MDE_ERR_ARG, "skip_cls needs tokens >= 2");
  OP_RET(launch_layernorm(nullptr, (h16*)y, g, b, rows, dim, eps, tokens > 0 ? tokens : 1, skip_cls, (hipStream_t)st,
                          (const h16*)x),
         "layernorm_f16");
}

int mde_op_layernorm(const float* x, void* y, const float* g, const float* b, int rows, int dim, float eps,
                     int tokens, int skip_cls, void* st) {
  if (!x || !y || !g || !b) return fail(MDE_ERR_ARG, "null argument");
  if (skip_cls && tokens < 2) return fail(MDE_ERR_ARG, "skip_cls needs tokens >= 2");
  OP_RET(launch_layernorm(x, (h16*)y, g, b, rows, dim, eps, tokens > 0 ? tokens : 1, skip_cls, (hipStream_t)st),
         "layernorm");
}

int mde_op_linear(const void* a, int lda, const void* w, int ldw, int m, int n, int k, const float* bias, int act,
                  void* out, int ldo, void* st) {
  if (!a || !w || !out) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.A = (const h16*)a;
  g.lda = lda;
  g.W = (const h16*)w;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.act = act;
  g.out16 = (h16*)out;
  g.ldo = ldo;
  OP_RET(launch_gemm(g, (hipStream_t)st), "linear");
}

int mde_op_linear_residual(const void* a, int lda, const void* w, int ldw, int m, int n, int k, const float* bias,
                           const float* ls, float* x32, int ldx, void* st) {
  if (!a || !w || !bias || !ls || !x32) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.emode = E_RESID;
  g.A = (const h16*)a;
  g.lda = lda;
  g.W = (const h16*)w;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.ls = ls;
  g.x32 = x32;
  g.ldo = ldx;
  OP_RET(launch_gemm(g, (hipStream_t)st), "linear_residual");
}

// E_QKV geometry: V^T stores key t at vt_pos(t), which swaps bits 2 and 3 of
// t, so a row of tokens_pad keys holds whole 16-key groups only when
// tokens_pad % 16 == 0 (otherwise the last group's keys land in the next row)
static const char* qkv_geometry_error(int batch, int tokens, int heads, int tokens_pad) {
  if (batch <= 0 || tokens <= 0 || heads <= 0) return "batch, tokens and heads must be > 0";
  if (tokens_pad < tokens) return "tokens_pad < tokens";
  if (tokens_pad % 16) return "tokens_pad % 16 != 0 (V^T key permutation works on 16-key groups)";
  return nullptr;
}

int mde_op_qkv(const void* a, const void* w, int ldw, const float* bias, int batch, int tokens, int heads,
               int tokens_pad, float qscale, void* q, void* k, void* vt, void* st) {
  if (!a || !w || !bias || !q || !k || !vt) return fail(MDE_ERR_ARG, "null argument");
  if (const char* why = qkv_geometry_error(batch, tokens, heads, tokens_pad)) return fail(MDE_ERR_ARG, why);
  GemmParams g;
  g.emode = E_QKV;
  const int D = heads * 64;
  g.A = (const h16*)a;
  g.lda = D;
  g.W = (const h16*)w;
  g.ldw = ldw;
  g.M = batch * tokens;
  g.N = 3 * D;
  g.K = D;
  g.bias = bias;
  g.q = (h16*)q;
  g.k = (h16*)k;
  g.vt = (h16*)vt;
  g.T = tokens;
  g.Tpad = tokens_pad;
  g.heads = heads;
  g.qscale = qscale;
  OP_RET(launch_gemm(g, (hipStream_t)st), "qkv");
}

int mde_op_linear_residual_f16(const void* a, int lda, const void* w, int ldw, int m, int n, int k, const float* bias,
                               const float* ls, void* xh, int ldx, float* ln_partials, void* st) {
  if (!a || !w || !bias || !ls || !xh) return fail(MDE_ERR_ARG, "null argument");
  if (ln_partials && (n & 31)) return fail(MDE_ERR_ARG, "ln_partials need n % 32 == 0");
  GemmParams g;
  g.emode = E_RESID;
  g.A = (const h16*)a;
  g.lda = lda;
  g.W = (const h16*)w;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.ls = ls;
  g.xh = (h16*)xh;
  g.ldo = ldx;
  g.lnst_out = ln_partials;
  g.lnst_ns = n / 32;
  g.lnst_rows = m;
  OP_RET(launch_gemm(g, (hipStream_t)st), "linear_residual_f16");
}

int mde_op_linear_lnfold(const void* x, const float* ln_partials, float eps, const void* wg, int ldw, const float* c1,
                         const float* c2, int m, int n, int k, int act, void* out, int ldo, void* st) {
  if (!x || !ln_partials || !wg || !c1 || !c2 || !out) return fail(MDE_ERR_ARG, "null argument");
  if (k & 31) return fail(MDE_ERR_ARG, "k % 32 != 0");
  GemmParams g;
  g.A = (const h16*)x;
  g.lda = k;
  g.W = (const h16*)wg;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = c2;
  g.act = act;
  g.out16 = (h16*)out;
  g.ldo = ldo;
  g.lnst_in = ln_partials;
  g.lnc1 = c1;
  g.lnst_ns = k / 32;
  g.lnst_rows = m;
  g.ln_eps = eps;
  OP_RET(launch_gemm(g, (hipStream_t)st), "linear_lnfold");
}

int mde_op_qkv_lnfold(const void* x, const float* ln_partials, float eps, const void* wg, int ldw, const float* c1,
                      const float* c2, int batch, int tokens, int heads, int tokens_pad, float qscale, void* q, void* k,
                      void* vt, void* st) {
  if (!x || !ln_partials || !wg || !c1 || !c2 || !q || !k || !vt) return fail(MDE_ERR_ARG, "null argument");
  if (const char* why = qkv_geometry_error(batch, tokens, heads, tokens_pad)) return fail(MDE_ERR_ARG, why);
  GemmParams g;
  g.emode = E_QKV;
  const int D = heads * 64;
  g.A = (const h16*)x;
  g.lda = D;
  g.W = (const h16*)wg;
  g.ldw = ldw;
  g.M = batch * tokens;
  g.N = 3 * D;
  g.K = D;
  g.bias = c2;
  g.q = (h16*)q;
  g.k = (h16*)k;
  g.vt = (h16*)vt;
  g.T = tokens;
  g.Tpad = tokens_pad;
  g.heads = heads;
  g.qscale = qscale;
  g.lnst_in = ln_partials;
  g.lnc1 = c1;
  g.lnst_ns = D / 32;
  g.lnst_rows = g.M;
  g.ln_eps = eps;
  OP_RET(launch_gemm(g, (hipStream_t)st), "qkv_lnfold");
}

int mde_op_attention(const void* q, const void* k, const void* vt, void* o, int batch, int heads, int tokens,
                     int tokens_pad, int ldo, void* st) {
  if (!q || !k || !vt || !o) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_attention((const h16*)q, (const h16*)k, (const h16*)vt, (h16*)o, batch, heads, tokens, tokens_pad,
                          ldo, (hipStream_t)st),
         "attention");
}

int mde_op_attention_ws(const void* q, const void* k, const void* vt, void* o, int batch, int heads, int tokens,
                        int tokens_pad, int ldo, void* ws, size_t ws_bytes, void* st) {
  if (!q || !k || !vt || !o || (!ws && ws_bytes)) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_attention((const h16*)q, (const h16*)k, (const h16*)vt, (h16*)o, batch, heads, tokens, tokens_pad,
                          ldo, (hipStream_t)st, (float*)ws, ws_bytes),
         "attention_ws");
}

int mde_op_attention_cfg(const void* q, const void* k, const void* vt, void* o, int batch, int heads, int tokens,
                         int tokens_pad, int ldo, const char* cfg, void* ws, size_t ws_bytes, void* st) {
  if (!q || !k || !vt || !o || (!ws && ws_bytes)) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_attention((const h16*)q, (const h16*)k, (const h16*)vt, (h16*)o, batch, heads, tokens, tokens_pad,
                          ldo, (hipStream_t)st, (float*)ws, ws_bytes, cfg),
         "attention_cfg");
}

size_t mde_op_attention_ws_bytes(int batch, int heads, int tokens) {
  return batch > 0 && heads > 0 && tokens > 0 ? attention_split_ws_bytes(batch, heads, tokens) : 0;
}

int mde_op_linear32(const float* a, int lda, const float* w, int ldw, int m, int n, int k, const float* bias, int act,
                    float* out, int ldo, void* st) {
  if (!a || !w || !out) return fail(MDE_ERR_ARG, "null argument");
  Gemm32Params g;
  g.A = a;
  g.lda = lda;
  g.W = w;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.act = act;
  g.out32 = out;
  g.ldo = ldo;
  OP_RET(launch_gemm32(g, (hipStream_t)st), "linear32");
}

int mde_op_conv3x3_32(const float* in, int batch, int h, int w, int cin, const float* wt, int ldw, int cout,
                      int stride, int relu_in, const float* bias, int act, const float* res0, const float* res1,
                      float* out, void* st) {
  if (!in || !wt || !out) return fail(MDE_ERR_ARG, "null argument");
  if (stride != 1 && stride != 2) return fail(MDE_ERR_ARG, "stride must be 1 or 2");
  if (batch <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return fail(MDE_ERR_ARG, "bad shape");
  Gemm32Params g;
  g.amode = A_CONV3;
  g.emode = E_STORE;
  g.A = in;
  g.cb = batch;
  g.ch = h;
  g.cw = w;
  g.cc = cin;
  g.stride = stride;
  g.oh = (h - 1) / stride + 1;
  g.ow = (w - 1) / stride + 1;
  g.W = wt;
  g.ldw = ldw;
  g.M = batch * g.oh * g.ow;
  g.N = cout;
  g.K = 9 * cin;
  g.relu_in = relu_in;
  g.bias = bias;
  g.act = act;
  g.res0 = res0;
  g.res1 = res1;
  g.out32 = out;
  g.ldo = cout;
  OP_RET(launch_gemm32(g, (hipStream_t)st), "conv3x3_32");
}

int mde_op_conv_transpose32(const float* in, int batch, int h, int w, int cin, const float* wt, int ldw, int cout,
                            int stride, const float* bias, float* out, void* st) {
  if (!in || !wt || !out) return fail(MDE_ERR_ARG, "null argument");
  if (batch <= 0 || h <= 0 || w <= 0 || stride < 1) return fail(MDE_ERR_ARG, "bad shape");
  Gemm32Params g;
  g.emode = E_CONVT;
  g.A = in;
  g.lda = cin;
  g.W = wt;
  g.ldw = ldw;
  g.M = batch * h * w;
  g.N = stride * stride * cout;
  g.K = cin;
  g.bias = bias;
  g.out32 = out;
  g.ldo = cout;
  g.s = stride;
  g.cout = cout;
  g.cb = batch;
  g.ih = h;
  g.iw = w;
  OP_RET(launch_gemm32(g, (hipStream_t)st), "conv_transpose32");
}

int mde_op_resize32(const float* in, int batch, int h, int w, int c, int oh, int ow, float* out, void* st) {
  if (!in || !out) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_resize32(in, out, batch, h, w, c, oh, ow, (hipStream_t)st), "resize32");
}

int mde_op_linear_residual32(const float* a, int lda, const float* w, int ldw, int m, int n, int k,
                             const float* bias, const float* ls, float* x32, int ldx, void* st) {
  if (!a || !w || !ls || !x32) return fail(MDE_ERR_ARG, "null argument");
  Gemm32Params g;
  g.emode = E_RESID;
  g.A = a;
  g.lda = lda;
  g.W = w;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.ls = ls;
  g.x32 = x32;
  g.ldo = ldx;
  OP_RET(launch_gemm32(g, (hipStream_t)st), "linear_residual32");
}

int mde_op_qkv32(const float* a, const float* w, int ldw, const float* bias, int batch, int tokens, int heads,
                 int tokens_pad, float q_scale, float* q, float* k, float* v, void* st) {
  if (!a || !w || !q || !k || !v) return fail(MDE_ERR_ARG, "null argument");
  Gemm32Params g;
  g.emode = E_QKV;
  g.A = a;
  g.lda = heads * 64;
  g.W = w;
  g.ldw = ldw;
  g.M = batch * tokens;
  g.N = 3 * heads * 64;
  g.K = heads * 64;
  g.bias = bias;
  g.q = q;
  g.k = k;
  g.v = v;
  g.T = tokens;
  g.Tpad = tokens_pad;
  g.heads = heads;
  g.qscale = q_scale;
  OP_RET(launch_gemm32(g, (hipStream_t)st), "qkv32");
}

int mde_op_attention32(const float* q, const float* k, const float* v, float* o, int batch, int heads, int tokens,
                       int tokens_pad, int ldo, void* st) {
  if (!q || !k || !v || !o) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_attention32(q, k, v, o, batch, heads, tokens, tokens_pad, ldo, (hipStream_t)st), "attention32");
}

int mde_op_patch_embed(const float* img, int batch, int h, int w, const void* wt, int ldw, const float* bias,
                       const float* pos_patch, const float* cls_pos, int dim, void* scratch, float* x32, void* st) {
  if (!img || !wt || !bias || !pos_patch || !cls_pos || !scratch || !x32) return fail(MDE_ERR_ARG, "null argument");
  if (h % 14 || w % 14) return fail(MDE_ERR_ARG, "image size must be a multiple of 14");
  const int ph = h / 14, pw = w / 14, T = ph * pw + 1;
  hipError_t e = launch_patch_prep(img, (h16*)scratch, x32, cls_pos, batch, h, w, ph, pw, T, dim, (hipStream_t)st);
  if (e != hipSuccess) return hip_fail(e, "patch_prep");
  GemmParams g;
  g.emode = E_PATCH;
  g.A = (const h16*)scratch;
  g.lda = 672;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = batch * ph * pw;
  g.N = dim;
  g.K = 672;
  g.bias = bias;
  g.x32 = x32;
  g.ldo = dim;
  g.T = T;
  g.pos = pos_patch;
  g.npatch = ph * pw;
  OP_RET(launch_gemm(g, (hipStream_t)st), "patch_embed");
}

namespace {
// GemmParams of a 3x3 / pad-1 conv over an NHWC f16 map (the mde_op_conv3x3* ops)
GemmParams conv3x3_params(const void* in, int batch, int h, int w, int cin, const void* wt, int ldw, int cout,
                          int stride, int relu_in, const float* bias, int act, const void* res0, const void* res1,
                          void* out) {
  GemmParams g;
  g.amode = A_CONV3;
  g.A = (const h16*)in;
  g.cb = batch;
  g.ch = h;
  g.cw = w;
  g.cc = cin;
  g.stride = stride;
  g.oh = (h - 1) / stride + 1;
  g.ow = (w - 1) / stride + 1;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = batch * g.oh * g.ow;
  g.N = cout;
  g.K = 9 * cin;
  g.relu_in = relu_in;
  g.bias = bias;
  g.act = act;
  g.res0 = (const h16*)res0;
  g.res1 = (const h16*)res1;
  g.out16 = (h16*)out;
  g.ldo = cout;
  return g;
}
}  // namespace

int mde_op_conv3x3(const void* in, int batch, int h, int w, int cin, const void* wt, int ldw, int cout, int stride,
                   int relu_in, const float* bias, int act, const void* res0, const void* res1, void* out,
                   void* st) {
  if (!in || !wt || !out) return fail(MDE_ERR_ARG, "null argument");
  if (stride != 1 && stride != 2) return fail(MDE_ERR_ARG, "stride must be 1 or 2");
  const GemmParams g = conv3x3_params(in, batch, h, w, cin, wt, ldw, cout, stride, relu_in, bias, act, res0, res1, out);
  OP_RET(launch_gemm(g, (hipStream_t)st), "conv3x3");
}

int mde_op_conv3x3_ws(const void* in, int batch, int h, int w, int cin, const void* wt, int ldw, int cout, int stride,
                      int relu_in, const float* bias, int act, const void* res0, const void* res1, void* out,
                      float* ws, size_t ws_floats, int* slices, void* st) {
  if (!in || !wt || !out || (!ws && ws_floats)) return fail(MDE_ERR_ARG, "null argument");
  if (stride != 1 && stride != 2) return fail(MDE_ERR_ARG, "stride must be 1 or 2");
  GemmParams g = conv3x3_params(in, batch, h, w, cin, wt, ldw, cout, stride, relu_in, bias, act, res0, res1, out);
  g.partial = ws;
  g.partial_cap = ws_floats;
  if (slices) *slices = gemm_store_split_slices(g);
  OP_RET(launch_gemm(g, (hipStream_t)st), "conv3x3_ws");
}

int mde_op_linear_ws(const void* a, int lda, const void* wt, int ldw, int m, int n, int k, const float* bias, int act,
                     void* out, int ldo, float* ws, size_t ws_floats, int* slices, void* st) {
  if (!a || !wt || !out || (!ws && ws_floats)) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.amode = A_DENSE;
  g.A = (const h16*)a;
  g.lda = lda;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = m;
  g.N = n;
  g.K = k;
  g.bias = bias;
  g.act = act;
  g.out16 = (h16*)out;
  g.ldo = ldo;
  g.partial = ws;
  g.partial_cap = ws_floats;
  if (slices) *slices = gemm_store_split_slices(g);
  OP_RET(launch_gemm(g, (hipStream_t)st), "linear_ws");
}

int mde_op_conv3x3_up(const void* in, int batch, int sh, int sw, int cin, int uh, int uw, const void* wt, int ldw,
                      int cout, const float* bias, int act, void* out, void* st) {
  if (!in || !wt || !out) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.amode = A_CONV3_UP;
  g.A = (const h16*)in;
  g.cb = batch;
  g.ch = sh;
  g.cw = sw;
  g.cc = cin;
  g.uh = uh;
  g.uw = uw;
  g.oh = uh;
  g.ow = uw;
  g.stride = 1;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = batch * uh * uw;
  g.N = cout;
  g.K = 9 * cin;
  g.bias = bias;
  g.act = act;
  g.out16 = (h16*)out;
  g.ldo = cout;
  OP_RET(launch_gemm(g, (hipStream_t)st), "conv3x3_up");
}

int mde_op_conv_transpose(const void* in, int batch, int h, int w, int cin, const void* wt, int ldw, int cout,
                          int stride, const float* bias, void* out, void* st) {
  if (!in || !wt || !bias || !out) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.emode = E_CONVT;
  g.A = (const h16*)in;
  g.lda = cin;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = batch * h * w;
  g.N = stride * stride * cout;
  g.K = cin;
  g.bias = bias;
  g.out16 = (h16*)out;
  g.s = stride;
  g.cout = cout;
  g.ldo = cout;
  g.ih = h;
  g.iw = w;
  OP_RET(launch_gemm(g, (hipStream_t)st), "conv_transpose");
}

int mde_op_resize_bilinear(const void* in, int batch, int ih, int iw, int c, int oh, int ow, void* out, void* st) {
  if (!in || !out) return fail(MDE_ERR_ARG, "null argument");
  OP_RET(launch_resize((const h16*)in, (h16*)out, batch, ih, iw, c, oh, ow, (hipStream_t)st), "resize_bilinear");
}

int mde_op_depth_head(const void* in, int batch, int sh, int sw, int cin, int uh, int uw, const void* wt, int ldw,
                      const float* bias, const float* w2, float b2, int metric, float max_depth, float* out,
                      void* st) {
  if (!in || !wt || !bias || !w2 || !out) return fail(MDE_ERR_ARG, "null argument");
  GemmParams g;
  g.amode = A_CONV3_UP;
  g.emode = E_HEAD;
  g.A = (const h16*)in;
  g.cb = batch;
  g.ch = sh;
  g.cw = sw;
  g.cc = cin;
  g.uh = uh;
  g.uw = uw;
  g.oh = uh;
  g.ow = uw;
  g.stride = 1;
  g.W = (const h16*)wt;
  g.ldw = ldw;
  g.M = batch * uh * uw;
  g.N = 32;
  g.K = 9 * cin;
  g.bias = bias;
  g.w2 = w2;
  g.b2 = b2;
  g.head_metric = metric;
  g.max_depth = max_depth;
  g.out32 = out;
  OP_RET(launch_gemm(g, (hipStream_t)st), "depth_head");
}

}  // extern "C"
