"""Build ablation variants of libmde_hip.so without touching the product source.

    python tools/ablate.py NAME            -> build/var/lib_NAME.so
    python tools/ablate.py --rev HEAD      -> build/var/lib_rev_HEAD.so (A/B side)

Each variant copies csrc/ to build/ablate/NAME/, applies text substitutions
to one kernel file (asserting each pattern is present) and links a library
with the product flags.  The variants answer "where does this kernel's time
go" (cdna_hip_programming.md section 5.4 rule 17: keep stubbed values live
with an empty asm so the compiler cannot delete the work upstream of them);
their outputs are wrong by construction and they are timing tools only
(tools/bench_kernels.py --lib build/var/lib_NAME.so).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name -> (file, [(old, new, count)])
VARIANTS = {
    # persistent RCU conv: no next-patch prefetch (MFMAs re-read the last patch)
    "cp_nopf": ("conv.hip", [("    if (tn < tend) load_patch(tn, BUF ^ 1, std::true_type{});\n", "", 1)]),
    # persistent RCU conv: no tap MFMAs (fragments kept live)
    "cp_nomfma": ("conv.hip", [
        ("acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);  // (tap MFMAs)",
         'asm volatile("" :: "v"(fb[j]), "v"(fa[i]));', 1)]),
    # direct conv: 32-wide tiles with one 64-channel chunk stream their taps (round-4 default: resident)
    "conv_bres32": ("conv.hip", [("#define MDE_CONV_BRES 2", "#define MDE_CONV_BRES 1", 1)]),
    # persistent RCU conv: conv1's input ReLU on the fragment reads, no LDS pass
    "cp_relufrag": ("conv.hip", [("#define MDE_CONVP_RELU_PASS 1", "#define MDE_CONVP_RELU_PASS 0", 1)]),
    # persistent RCU conv: no output stores (values kept live)
    "cp_nostore": ("conv.hip", [
        ("if (mo[it] >= 0) *reinterpret_cast<f16x8*>(out + (size_t)mo[it] * p.ldo + c8 * 8) = h;",
         'asm volatile("" :: "v"(h));', 2)]),
    # attention: the softmax exponentials replaced by their argument
    "attn_noexp": ("attention.hip", [
        ("const float p0 = __builtin_amdgcn_exp2f(sc[r]), p1 = __builtin_amdgcn_exp2f(sc[r + 1]);",
         "const float p0 = sc[r], p1 = sc[r + 1];", 1)]),
    # attention: no P.V MFMAs (P and the V fragments kept live)
    "attn_nopv": ("attention.hip", [
        ("acc[S][db] = mfma32(vf, pb[g], acc[S][db]);",
         'asm volatile("" :: "v"(vf), "v"(pb[g]));', 1)]),
    # attention: no score MFMAs (K fragments kept live, scores = C operand)
    "attn_noqk": ("attention.hip", [
        ("for (int s = 0; s < QS; ++s) sc.v[s] = mfma32(kf, qf[s][st], sc.v[s]);",
         'for (int s = 0; s < QS; ++s) asm volatile("" :: "v"(kf), "v"(qf[s][st]));', 1)]),
    # attention: no K/V waits or barriers (LDS races: wrong values, timing only)
    "attn_nosync": ("attention.hip", [
        ("""MDE_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}""", """MDE_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}""", 1),
        ("""MDE_DEV void wait_vm_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}""", """MDE_DEV void wait_vm_n() {
}""", 1)]),
    # attn16 (16x16x32 attention): the exponentials replaced by their argument
    "a16_noexp": ("attention.hip", [
        ("pb.v[s][r] = (f16)__builtin_amdgcn_exp2f(sc.v[0][s][r]);\n        pb.v[s][4 + r] = (f16)__builtin_amdgcn_exp2f(sc.v[1][s][r]);",
         "pb.v[s][r] = (f16)sc.v[0][s][r];\n        pb.v[s][4 + r] = (f16)sc.v[1][s][r];", 1)]),
    # attn16: no P.V / row-sum MFMAs (operands kept live)
    "a16_nopv": ("attention.hip", [
        ("for (int s = 0; s < 2; ++s) acc[dt][s] = mfma16x16x32(vf, pb.v[s], acc[dt][s]);",
         'for (int s = 0; s < 2; ++s) asm volatile("" :: "v"(vf), "v"(pb.v[s]));', 1),
        ("for (int s = 0; s < 2; ++s) lacc[s] = mfma16x16x32(ones, pb.v[s], lacc[s]);",
         'for (int s = 0; s < 2; ++s) asm volatile("" :: "v"(ones), "v"(pb.v[s]));', 1)]),
    # attn16: no score MFMAs (K fragments kept live, scores = C operand)
    "a16_noqk": ("attention.hip", [
        ("for (int s = 0; s < 2; ++s) sc.v[t][s] = mfma16x16x32(kf, qf[s][d], sc.v[t][s]);",
         'for (int s = 0; s < 2; ++s) asm volatile("" :: "v"(kf), "v"(qf[s][d]));', 1)]),
    # attn16: no rescale check (the running max never moves after the first block)
    "a16_nomax": ("attention.hip", [
        ("      if (FIRST || __any(mx > RESCALE_T)) {\n        mx = grp4_max(mx);",
         '      asm volatile("" :: "v"(mx));\n      if (FIRST) {\n        mx = grp4_max(mx);', 1)]),
    # attention (both kernels): no static priority for waves 4-7
    "attn_noprio": ("attention.hip", [
        ("if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);", "", 2)]),
    # attention (both kernels): the static priority on waves 0-3 instead
    "attn_prio_lo": ("attention.hip", [
        ("if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);",
         "if (NW == 8 && NS == 1 && wave_all < 4) __builtin_amdgcn_s_setprio(1);", 2)]),
    # attention (both kernels): priority 2 / 1 / 0 by wave pair (waves 6-7, 4-5, rest)
    "attn_prio3": ("attention.hip", [
        ("if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);",
         "if (NW == 8 && NS == 1 && wave_all >= 6) __builtin_amdgcn_s_setprio(2); "
         "else if (NW == 8 && NS == 1 && wave_all >= 4) __builtin_amdgcn_s_setprio(1);", 2)]),
    # separable upsampling conv: pass V reduced to its patch stores (no row index math, H reads, lerp)
    "uc_nov": ("conv.hip", [
        ("""        f16x8 v = zero8();
        if (xin && iy >= 0 && iy < p.uh) {
          int y0, y1;""", """        f16x8 v = zero8();
        if (false) {
          int y0, y1;""", 1)]),
    # separable upsampling conv: pass H commits one source column (no lerp)
    "uc_noh": ("conv.hip", [
        ("hin ? lerp8(ha[k], hb[k], hw) : zero8();", "ha[k];", 1)]),
    # separable upsampling conv: no tap MFMAs (fragments kept live)
    "uc_nomfma": ("conv.hip", [
        ("          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);\n        if constexpr (PERSIST)",
         '          for (int j = 0; j < TN; ++j) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));\n        if constexpr (PERSIST)', 1)]),
    # candidate (not an ablation): batch-1 stores / qkv whose 128^2 grid
    # overhangs the CUs by a partial round (ViT-L B=1 qkv 264, fc1 352 tiles)
    # on 256 x 128 tiles (8 waves of 64 x 64, BK 32 x 3 stages, two per CU):
    # one round, 25 % fewer L2 -> LDS bytes per FLOP.  Measured slower (r4s3,
    # same box: ViT-L B=1 3.19 -> 3.32 ms; qkv 0.612 -> 0.702, fc1 0.626 ->
    # 0.696 ms per forward)
    "gemm_wide_small": ("gemm.hip", [
        ("""        if (w8small(big)) return run<128, 128, 2, 4, AM, EM>(p, st);""",
         """        if (w8small(big)) {
          const long long t2 = (long long)((p.M + 255) / 256) * ((p.N + 127) / 128);
          if (t2 <= 256 && p.M >= 256) return run<256, 128, 4, 2, AM, EM, 32>(p, st);
          return run<128, 128, 2, 4, AM, EM>(p, st);
        }""", 1)]),
    # GEMM main loop only: the epilogue returns unless a NaN appears (r02's
    # MDE_EXP_NOEPI, profiles/r02_v10_epilogue_cost_*)
    "gemm_noepi": ("gemm.hip", [
        ("""  // LDS-staged epilogue when every wave's fp32 tile fits in the ring, or""",
         """  {
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) z += acc[i][j][0] + acc[i][j][3];
    if (z == z) return;
  }
  // LDS-staged epilogue when every wave's fp32 tile fits in the ring, or""", 1)]),
    # GEMM: no MFMAs in the main loop (fragments kept live): the load / sync skeleton alone
    "gemm_nomfma": ("gemm.hip", [
        ("for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);",
         'for (int j = 0; j < TN; ++j) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));', 1)]),
    # direct conv, upsampling patch: one source tap per virtual pixel, no blend
    "conv_noblend": ("conv.hip", [
        ("""            const f16x8 bq = *reinterpret_cast<const f16x8*>(img + (r0 + o1 + lc * 8));
            const f16x8 c = *reinterpret_cast<const f16x8*>(img + (r1 + o0 + lc * 8));
            const f16x8 d = *reinterpret_cast<const f16x8*>(img + (r1 + o1 + lc * 8));""", "", 1),
        ("v = lerp8(lerp8(a, bq, (f16)lx1), lerp8(c, d, (f16)lx1), (f16)ly1);", "v = a;", 1)]),
    # direct conv (conv3_kernel and upconv_kernel): no MFMAs (fragments kept live)
    "conv_nomfma": ("conv.hip", [
        ("for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);",
         'for (int j = 0; j < TN; ++j) asm volatile("" :: "v"(fb[j]), "v"(fa[i]));', 4)]),
    # separable upsampling conv: pass V without its vertical lerp (one H row read)
    "upconv_nov": ("conv.hip", [
        ("          v = lerp8(a, bb, (f16)ly1);\n", "          v = a;\n          asm volatile(\"\" :: \"v\"(bb));\n", 1)]),
    # separable upsampling conv: pass H without its horizontal lerp (loads kept)
    "upconv_noh": ("conv.hip", [
        ("hin ? lerp8(ha[k], hb[k], hw) : zero8();",
         "hin ? ha[k] : hb[k];", 1)]),
    # direct conv: weights never loaded (LDS garbage)
    "conv_now": ("conv.hip", [
        ("for (int q = wave; q < BINS; q += NW) glds16c(", "for (int q = wave; q < 0; q += NW) glds16c(", 1)]),
    # direct conv: no patch at all (LDS garbage): weights, MFMA and epilogue only
    "conv_nopatch": ("conv.hip", [
        ("  auto load_patch = [&](int chunk) {\n    const int cbase = chunk * CK;",
         "  auto load_patch = [&](int chunk) {\n    if (chunk >= 0) return;\n    const int cbase = chunk * CK;", 1)]),
}


def build(name: str) -> str:
    from monocular_depth_estimation_trt_amd import _build
    fname, subs = VARIANTS[name]
    work = os.path.join(ROOT, "build", "ablate", name)
    if os.path.exists(work):
        shutil.rmtree(work)
    shutil.copytree(_build.CSRC, work)
    path = os.path.join(work, fname)
    with open(path) as f:
        s = f.read()
    for old, new, count in subs:
        n = s.count(old)
        if n != count:
            raise SystemExit(f"{name}: pattern found {n} times (expected {count}): {old[:60]!r}")
        s = s.replace(old, new)
    with open(path, "w") as f:
        f.write(s)
    out = os.path.join(ROOT, "build", "var", f"lib_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # only the edited file is recompiled (against the product headers); the
    # other objects are the product build's (build/obj, `_build.build_library`)
    _build.build_library()
    cc = _build.hipcc()
    obj = os.path.join(work, fname + ".o")
    cmd = [cc, *_build.FLAGS, *_build.PER_FILE.get(fname, []), "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(f"{name}: hipcc failed\n{r.stderr[-3000:]}")
    objs = [obj if src == fname else os.path.join(_build.OBJDIR, src + ".o") for src in _build.SOURCES]
    subprocess.run([cc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(f"[ablate] built {out}")
    return out


def build_rev(rev: str) -> str:
    """The whole library as of git revision `rev` (the A side of an A/B
    against the working tree): build/var/lib_rev_<rev>.so"""
    import concurrent.futures as cf
    import tarfile
    import io
    from monocular_depth_estimation_trt_amd import _build
    sha = subprocess.run(["git", "rev-parse", "--short", rev], cwd=ROOT, capture_output=True, text=True,
                         check=True).stdout.strip()
    work = os.path.join(ROOT, "build", "ablate", f"rev_{sha}")
    if os.path.exists(work):
        shutil.rmtree(work)
    os.makedirs(work)
    tar = subprocess.run(["git", "archive", sha, "monocular_depth_estimation_trt_amd/csrc", "include"], cwd=ROOT,
                         capture_output=True, check=True).stdout
    with tarfile.open(fileobj=io.BytesIO(tar)) as t:
        t.extractall(work)
    csrc = os.path.join(work, "monocular_depth_estimation_trt_amd", "csrc")
    inc = os.path.join(work, "include")
    flags = [f if f not in (_build.CSRC, _build.INCLUDE) else (csrc if f == _build.CSRC else inc) for f in _build.FLAGS]
    cc = _build.hipcc()

    def one(src):
        obj = os.path.join(work, src + ".o")
        r = subprocess.run([cc, *flags, *_build.PER_FILE.get(src, []), "-c", os.path.join(csrc, src), "-o", obj],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(f"rev {sha}: hipcc failed on {src}\n{r.stderr[-3000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(one, _build.SOURCES))
    out = os.path.join(ROOT, "build", "var", f"lib_rev_{rev}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([cc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(f"[ablate] built {out} ({sha})")
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    if args[:1] == ["--rev"]:
        build_rev(args[1] if len(args) > 1 else "HEAD")
    else:
        for n in args or sorted(VARIANTS):
            build(n)
