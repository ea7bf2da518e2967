"""Per-kernel parity: each HIP kernel (through the C ABI) vs a plain PyTorch
fp32 CPU reference of the same op, on seeded inputs.  Shapes are chosen to hit
tails (M, N, K not tile multiples), both tile configurations, and the DA-V2
shapes where they are cheap.

Tolerances: operands are fp16 and accumulation fp32, outputs rounded to fp16,
so |err| <= atol + rtol*|ref| with rtol = 1e-2, atol scaled to the output
magnitude (stated per test).
"""

import math

import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from gpu_util import close, conv_w, nchw, nhwc, op, pad_w, ptr, stream, vt_perm

pytestmark = pytest.mark.gpu

G = torch.Generator().manual_seed(7)


def rn(*shape, scale=1.0):
    return torch.randn(*shape, generator=G) * scale


def f16(t, dev):
    return t.half().to(dev)


@pytest.mark.parametrize("m,n,k,act", [(300, 200, 96, 0), (1370, 1152, 384, 0), (777, 1536, 384, 2),
                                       (64, 48, 48, 1), (5, 32, 64, 1), (2048, 384, 1536, 0),
                                       (16384, 1536, 384, 2), (33000, 1024, 200, 1), (65537, 512, 64, 0),
                                       # K >= 768 in whole rounds of 256 256^2 tiles: gemm256 (gemm256_eligible)
                                       (20480, 4096, 1024, 2), (16384, 1024, 4096, 0)])
def test_linear(gpu, m, n, k, act):
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    a16, w16 = a.half().float(), w.half().float()
    ref = a16 @ w16.T + b
    if act == 1:
        ref = F.relu(ref)
    elif act == 2:
        ref = F.gelu(ref)
    wp = pad_w(w).to(gpu)
    out = torch.empty(m, n, dtype=torch.float16, device=gpu)
    op("mde_op_linear", ptr(f16(a, gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)), act, ptr(out), n,
       stream())
    close(out, ref, 1e-2, 1e-2, f"linear {m}x{n}x{k} act{act}")


@pytest.mark.parametrize("m,n,k", [(1370, 384, 1536), (43840, 384, 1536)])
def test_linear_residual(gpu, m, n, k):
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ls = 0.5 + 0.05 * rn(n)
    x = rn(m, n)
    ref = x + ls * (a.half().float() @ w.half().float().T + b)
    xg = x.clone().to(gpu)
    wp = pad_w(w).to(gpu)
    op("mde_op_linear_residual", ptr(f16(a, gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)),
       ptr(ls.to(gpu)), ptr(xg), n, stream())
    close(xg, ref, 2e-3, 2e-3, "linear_residual")


@pytest.mark.parametrize("B,T,H", [(2, 50, 6), (16, 1370, 6),
                                   # 128^2 tiles with the LDS-staged V^T quads: image boundaries
                                   # inside tiles at every token alignment (T % 4 = 1, 3)
                                   (100, 37, 6), (3, 1371, 6),
                                   # D 1024, 75 x 12 tiles of 256^2 (>= 80 % of 4 rounds): gemm256 E_QKV
                                   (14, 1370, 16),
                                   # >= 64 panels of 256 rows: the panel kernel (gemm_panel.hip), V^T
                                   # quads cut by image boundaries at T % 4 = 1 / 3
                                   (480, 37, 6), (12, 1371, 6)])
def test_qkv_layout(gpu, B, T, H):
    D = 64 * H
    Tp = -(-T // 64) * 64
    a, w, b = rn(B * T, D), rn(3 * D, D, scale=D ** -0.5), rn(3 * D, scale=0.1)
    full = a.half().float() @ w.half().float().T + b                         # [B*T, 3D]
    full = full.reshape(B, T, 3, H, 64)
    wp = pad_w(w).to(gpu)
    q = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    k = torch.zeros_like(q)
    vt = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    op("mde_op_qkv", ptr(f16(a, gpu)), ptr(wp), wp.shape[1], ptr(b.to(gpu)), B, T, H, Tp, 0.125, ptr(q), ptr(k),
       ptr(vt), stream())
    rq = full[:, :, 0].permute(0, 2, 1, 3).reshape(B * H, T, 64) * 0.125
    rk = full[:, :, 1].permute(0, 2, 1, 3).reshape(B * H, T, 64)
    rv = full[:, :, 2].permute(0, 2, 3, 1).reshape(B * H, 64, T)
    close(q[:, :T], rq, 1e-2, 1e-2, "q")
    close(k[:, :T], rk, 1e-2, 1e-2, "k")
    perm = vt_perm(T).to(gpu)
    close(vt[:, :, perm], rv, 1e-2, 1e-2, "vt (key-permuted storage)")
    pad = torch.ones(Tp, dtype=torch.bool, device=gpu)
    pad[perm] = False
    assert float(q[:, T:].abs().max()) == 0 and float(vt[:, :, pad].abs().max()) == 0, "pad must stay zero"


@pytest.mark.parametrize("case", ["linear_gelu", "linear_none", "linear_relu_tail", "lnfold_gelu",
                                  "qkv_1370", "qkv_37", "qkv_lnfold", "resid_proj", "resid_proj_tail"])
def test_panel_gemm_bit_exact(gpu, case):
    """Switch "panel" (gemm_panel.hip: A-stationary 256-row panels, each
    unit's MFMAs interleaved with the previous unit's epilogue) against the
    128^2 BK 32 kernel it replaces for K = 384 E_STORE at large M: the same
    MFMA k order and the same fp32 epilogue operations (LN statistics through
    the shared ln_merge_stats), so every output must be equal bit for bit,
    with M not a multiple of 256 -- the E_STORE cases and the qkv head split
    (q scaled, k, and V^T at its key-permuted positions; T = 37 puts image
    boundaries inside every panel)."""
    from monocular_depth_estimation_trt_amd import _lib
    k = 384
    if case.startswith("resid"):
        # proj over the f16 residual stream: xh must match bit for bit; the
        # LN partials of the rows written sum the same 32 f16 values in
        # another grouping, so they agree to fp32 rounding
        m, n = (65760, 384) if case == "resid_proj" else (16397, 384)
        a = (rn(m, k) * 2).half().to(gpu)
        w, b = rn(n, k, scale=k ** -0.5), rn(n, scale=0.1).to(gpu)
        ls = (0.5 + 0.1 * rn(n)).to(gpu)
        wp = pad_w(w).to(gpu)
        x0 = (rn(m, n) * 2).half().to(gpu)
        res = []
        for panel in (2, 0):  # proj takes the panel kernel only at panel = 2
            xh = x0.clone()
            part = torch.full((n // 32, m, 2), float("nan"), device=gpu)
            with _lib.tuning(panel=panel):
                op("mde_op_linear_residual_f16", ptr(a), k, ptr(wp), wp.shape[1], m, n, k, ptr(b), ptr(ls), ptr(xh), n,
                   ptr(part), stream())
            res.append((xh, part))
        d = (res[0][0].float() - res[1][0].float()).abs()
        assert torch.equal(res[0][0], res[1][0]), \
            f"{case}: xh differs ({int((d > 0).sum())} elements, max {float(d.max())})"
        assert torch.isfinite(res[0][1]).all(), "partials not all written"
        close(res[0][1], res[1][1].float(), 1e-5, 1e-4, f"{case} ln partials")
        return
    if case.startswith("linear") or case.startswith("lnfold"):
        m = {"linear_gelu": 16384, "linear_none": 21920, "linear_relu_tail": 16397, "lnfold_gelu": 38360}[case]
        n = 1536 if case != "linear_none" else 1152
        act = {"linear_gelu": 2, "linear_none": 0, "linear_relu_tail": 1, "lnfold_gelu": 2}[case]
        x = (rn(m, k) * 2 + 0.3).half().to(gpu)
        w, b = rn(n, k, scale=k ** -0.5), rn(n, scale=0.1).to(gpu)
        wp = pad_w(w).to(gpu)
        part = ln_partials_ref(x.cpu()).float().to(gpu)
        c1 = rn(n).to(gpu)
        outs = []
        for panel in (1, 0):
            out = torch.full((m, n), float("nan"), dtype=torch.float16, device=gpu)
            with _lib.tuning(panel=panel):
                if case == "lnfold_gelu":
                    op("mde_op_linear_lnfold", ptr(x), ptr(part), 1e-6, ptr(wp), wp.shape[1], ptr(c1), ptr(b), m, n,
                       k, act, ptr(out), n, stream())
                else:
                    op("mde_op_linear", ptr(x), k, ptr(wp), wp.shape[1], m, n, k, ptr(b), act, ptr(out), n, stream())
            outs.append(out)
        assert torch.isfinite(outs[0]).all(), case
        d = (outs[0].float() - outs[1].float()).abs()
        rows = torch.nonzero(d.amax(1) > 0).flatten()[:12].tolist()
        if case == "lnfold_gelu" and rows:  # diagnostics: which side is nearer a float64 reference
            xr = x[rows].double().cpu()
            mu = xr.mean(1, keepdim=True)
            rs = 1.0 / torch.sqrt(((xr - mu) ** 2).mean(1, keepdim=True) + 1e-6)
            acc = xr @ wp[:, :k].double().cpu()[:n].T
            ref = F.gelu(rs * (acc - mu * c1.double().cpu()[None, :]) + b.double().cpu()[None, :])
            e0 = (outs[0][rows].double().cpu() - ref).abs().sum().item()
            e1 = (outs[1][rows].double().cpu() - ref).abs().sum().item()
            print(f"lnfold rows {rows}: |panel - ref| {e0:.6g}  |128^2 - ref| {e1:.6g}")
        assert torch.equal(outs[0], outs[1]), \
            f"{case}: panel kernel differs from the 128^2 kernel ({int((d > 0).sum())} elements, max {float(d.max())}," \
            f" {int((d.amax(1) > 0).sum())} rows, first {rows})"
        return
    B, T, H = {"qkv_1370": (16, 1370, 6), "qkv_37": (480, 37, 6), "qkv_lnfold": (16, 1370, 6)}[case]
    D = 64 * H
    Tp = -(-T // 64) * 64
    a = (rn(B * T, D) * 2 + 0.3).half().to(gpu)
    w, b = rn(3 * D, D, scale=D ** -0.5), rn(3 * D, scale=0.1).to(gpu)
    wp = pad_w(w).to(gpu)
    part = ln_partials_ref(a.cpu()).float().to(gpu)
    c1 = rn(3 * D).to(gpu)
    res = []
    for panel in (1, 0):
        q = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
        kk = torch.zeros_like(q)
        vt = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
        with _lib.tuning(panel=panel):
            if case == "qkv_lnfold":
                op("mde_op_qkv_lnfold", ptr(a), ptr(part), 1e-6, ptr(wp), wp.shape[1], ptr(c1), ptr(b), B, T, H, Tp,
                   0.125, ptr(q), ptr(kk), ptr(vt), stream())
            else:
                op("mde_op_qkv", ptr(a), ptr(wp), wp.shape[1], ptr(b), B, T, H, Tp, 0.125, ptr(q), ptr(kk), ptr(vt),
                   stream())
        res.append((q, kk, vt))
    for name, x0, x1 in zip("q k vt".split(), res[0], res[1]):
        d = (x0.float() - x1.float()).abs()
        assert torch.equal(x0, x1), \
            f"{case}: panel kernel {name} differs from the 128^2 kernel ({int((d > 0).sum())} elements, max {float(d.max())})"


@pytest.mark.parametrize("case", ["linear_gelu", "linear_none", "linear_relu_tail", "lnfold_gelu",
                                  "qkv_1370", "qkv_37", "qkv_lnfold"])
def test_panel32_matches_tile_kernel(gpu, case):
    """Switch "panel32" (gemm_panel.hip panel32_kernel: v_mfma_f32_32x32x16,
    the folded LayerNorm's mean term in the accumulator's initial value, 16-B
    stores through v_permlane32_swap) against the 128^2 kernel: another fp32 association of the same sums, so
    every output within the f16 output rounding (2 ulp relative + 1e-3),
    no nearer the float64 reference's error than 1.25x the 128^2 kernel's
    (LN fold cases), and bit-identical from run to run."""
    from monocular_depth_estimation_trt_amd import _lib
    k = 384

    def run(cfg):
        with _lib.tuning(**cfg):
            if case.startswith("qkv"):
                q = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
                kk = torch.zeros_like(q)
                vt = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
                if case == "qkv_lnfold":
                    op("mde_op_qkv_lnfold", ptr(x), ptr(part), 1e-6, ptr(wp), wp.shape[1], ptr(c1), ptr(b), B, T, H,
                       Tp, 0.125, ptr(q), ptr(kk), ptr(vt), stream())
                else:
                    op("mde_op_qkv", ptr(x), ptr(wp), wp.shape[1], ptr(b), B, T, H, Tp, 0.125, ptr(q), ptr(kk),
                       ptr(vt), stream())
                return torch.cat([q.flatten(), kk.flatten(), vt.flatten()])
            out = torch.full((m, n), float("nan"), dtype=torch.float16, device=gpu)
            if case == "lnfold_gelu":
                op("mde_op_linear_lnfold", ptr(x), ptr(part), 1e-6, ptr(wp), wp.shape[1], ptr(c1), ptr(b), m, n, k,
                   act, ptr(out), n, stream())
            else:
                op("mde_op_linear", ptr(x), k, ptr(wp), wp.shape[1], m, n, k, ptr(b), act, ptr(out), n, stream())
            return out.flatten()

    if case.startswith("qkv"):
        B, T, H = {"qkv_1370": (16, 1370, 6), "qkv_37": (480, 37, 6), "qkv_lnfold": (16, 1370, 6)}[case]
        Tp = -(-T // 64) * 64
        m, n = B * T, 3 * 64 * H
    else:
        m = {"linear_gelu": 16384, "linear_none": 21920, "linear_relu_tail": 16397, "lnfold_gelu": 38360}[case]
        n = 1536 if case != "linear_none" else 1152
        act = {"linear_gelu": 2, "linear_none": 0, "linear_relu_tail": 1, "lnfold_gelu": 2}[case]
    x = (rn(m, k) * 2 + 0.3).half().to(gpu)
    w, b = rn(n, k, scale=k ** -0.5), rn(n, scale=0.1).to(gpu)
    wp = pad_w(w).to(gpu)
    part = ln_partials_ref(x.cpu()).float().to(gpu)
    c1 = rn(n).to(gpu)
    y32 = run({"panel": 1, "panel32": 1})
    y32b = run({"panel": 1, "panel32": 1})
    y0 = run({"panel": 0, "panel32": 0})
    assert torch.isfinite(y32).all(), case
    assert torch.equal(y32, y32b), f"{case}: panel32 not deterministic"
    d = (y32.float() - y0.float()).abs()
    lim = 1e-3 + 2.0 ** -9 * y0.float().abs()
    bad = int((d > lim).sum())
    print(f"{case}: {int((d > 0).sum())} of {d.numel()} outputs differ from the 128^2 kernel, max {float(d.max()):.3g}")
    assert bad == 0, f"{case}: {bad} outputs beyond 2 f16 ulp (max {float(d.max())})"
    if case in ("lnfold_gelu", "qkv_lnfold") and not case.startswith("qkv"):
        xr = x.double().cpu()[:4096]
        mu = xr.mean(1, keepdim=True)
        rs = 1.0 / torch.sqrt(((xr - mu) ** 2).mean(1, keepdim=True) + 1e-6)
        acc = xr @ wp[:, :k].double().cpu()[:n].T
        ref = F.gelu(rs * (acc - mu * c1.double().cpu()[None, :]) + b.double().cpu()[None, :])
        e32 = (y32.reshape(m, n)[:4096].double().cpu() - ref).abs().sum().item()
        e0 = (y0.reshape(m, n)[:4096].double().cpu() - ref).abs().sum().item()
        print(f"{case}: |panel32 - f64| {e32:.6g}  |128^2 - f64| {e0:.6g}")
        assert e32 <= 1.25 * e0, (e32, e0)


LOG2E = 1.4426950408889634


def attn_ref(q, k, v):
    """q is pre-scaled by dh^-0.5 * log2(e) (the kernel's contract): scores are
    in log2 units, softmax base 2 == softmax base e of scores * ln 2."""
    qh, kh, vh = q.half().float(), k.half().float(), v.half().float()
    return torch.softmax((qh @ kh.transpose(1, 2)) / LOG2E, dim=-1) @ vh


@pytest.mark.parametrize("B,H,T", [(2, 6, 50), (1, 6, 1370), (1, 2, 64), (3, 1, 65), (1, 16, 130),
                                   (32, 6, 200), (8, 6, 1370), (1, 1, 1)])
def test_attention(gpu, B, H, T):
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T] = q.half().to(gpu)
    kg[:, :T] = k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    o = torch.empty(B * T, H * 64, dtype=torch.float16, device=gpu)
    op("mde_op_attention", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, stream())
    close(o, ref, 2e-2, 5e-3, f"attention B{B} H{H} T{T}")


@pytest.mark.parametrize("B,H,T,spiky", [(1, 6, 1370, False), (1, 16, 1370, False), (1, 2, 700, True),
                                         (2, 6, 1370, False)])
def test_attention_split_kv(gpu, B, H, T, spiky):
    """Small grids split the key range (launch_attention's policy): B=1 at 6
    x 1370 as four key groups of 64 queries in one 8-wave workgroup, at 16 x
    1370 as two groups of 128 (merged through LDS); B=2 at 6 x 1370 (264
    64-query groups: more than the CUs) over workgroups, merging the fp32
    partials (attn_combine_kernel); 2 x 700 unsplit (too few key tiles)."""
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    if spiky:  # a dominant key late in the row, and one in another split
        k[:, T - 10] = q.mean(1) * 60.0
        k[:, 3] = q.mean(1) * 30.0
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    from monocular_depth_estimation_trt_amd import _lib
    nbytes = _lib.lib().mde_op_attention_ws_bytes(B, H, T)
    assert nbytes > 0
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=gpu)
    o = torch.empty(B * T, H * 64, dtype=torch.float16, device=gpu)
    op("mde_op_attention_ws", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, ptr(ws), nbytes, stream())
    close(o, ref, 2e-2, 5e-3, f"attention split-KV B{B} H{H} T{T}")


@pytest.mark.parametrize("cfg", ["4g2", "8g2", "4g4", "8g4", "12g3", "16g4", "6g2", "8g2m", "8g4m"])
@pytest.mark.parametrize("B,H,T,spiky", [(1, 16, 1370, False), (1, 6, 1370, True), (2, 3, 129, False),
                                         (1, 2, 300, True), (1, 1, 200, False)])
def test_attention_key_groups(gpu, cfg, B, H, T, spiky):
    """In-workgroup split-KV (attention.hip, NS key groups of NW / NS query
    waves merged through LDS): uneven group lengths (T 129: 2 + 1 tiles),
    an empty group (T 300 at 4 groups: 2 + 2 + 1 + 0 tiles), the partial last
    tile, and dominant keys in different groups (spiky)."""
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    if spiky:
        k[:, T - 10] = q.mean(1) * 60.0
        k[:, 3] = q.mean(1) * 30.0
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    o = torch.empty(B * T, H * 64, dtype=torch.float16, device=gpu)
    op("mde_op_attention_cfg", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, cfg.encode(), None, 0,
       stream())
    close(o, ref, 2e-2, 5e-3, f"attention {cfg} B{B} H{H} T{T}")


@pytest.mark.parametrize("cfg", ["8", "4", "8q2", "4q2", "8r3", "4r4", "4s2", "4s3"])
@pytest.mark.parametrize("B,H,T", [(2, 3, 300), (1, 6, 1370), (3, 5, 577)])
def test_attention_tuning_configs(gpu, cfg, B, H, T):
    """Every launch shape mde_op_attention_cfg can force: 8 / 4
    waves, two query sub-tiles per wave (q2), 3- and 4-deep K/V rings, split-KV
    over workgroups with the combine kernel -- the same numbers as the policy's
    shapes, against torch."""
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    from monocular_depth_estimation_trt_amd import _lib
    nbytes = _lib.lib().mde_op_attention_ws_bytes(B, H, T)
    ws = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=gpu)
    o = torch.empty(B * T, H * 64, dtype=torch.float16, device=gpu)
    op("mde_op_attention_cfg", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, cfg.encode(), ptr(ws),
       nbytes, stream())
    close(o, ref, 2e-2, 5e-3, f"attention cfg {cfg} B{B} H{H} T{T}")


@pytest.mark.parametrize("cfg", ["8m", "4m"])
@pytest.mark.parametrize("B,H,T,spiky", [(2, 3, 300, False), (1, 6, 1370, True), (3, 5, 577, False), (1, 2, 20, False),
                                         (16, 6, 1370, False), (1, 1, 1, False), (2, 2, 700, True)])
def test_attention_16x16_matches(gpu, cfg, B, H, T, spiky):
    """attn16_fwd_kernel (v_mfma_f32_16x16x32_f16, switch "attn16"): against
    torch, with partial last blocks (T 300, 577, 20, 1), the rescale path
    (spiky: dominant keys early and late), and -- the policy's switch -- the
    default launch with attn16 = 1 bit-identical to the forced "8m" shape."""
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    if spiky:
        k[:, T - 10] = q.mean(1) * 60.0
        k[:, 3] = q.mean(1) * 30.0
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    o = torch.full((B * T, H * 64), float("nan"), dtype=torch.float16, device=gpu)
    op("mde_op_attention_cfg", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, cfg.encode(), None, 0,
       stream())
    close(o, ref, 2e-2, 5e-3, f"attention {cfg} B{B} H{H} T{T}")
    from monocular_depth_estimation_trt_amd import _lib
    o32 = torch.empty_like(o)
    with _lib.tuning(attn16=0):
        op("mde_op_attention", ptr(qg), ptr(kg), ptr(vtg), ptr(o32), B, H, T, Tp, H * 64, stream())
        torch.cuda.synchronize()
    d = (o.float() - o32.float()).abs().max().item()
    print(f"attention {cfg} B{B} H{H} T{T}: max |16x16 - 32x32| {d:.3g}")
    if cfg == "8m" and (B * H * -(-T // 256)) >= 512:  # the policy picks 8 unsplit waves: the switch applies
        with _lib.tuning(attn16=1):
            o16 = torch.empty_like(o)
            op("mde_op_attention", ptr(qg), ptr(kg), ptr(vtg), ptr(o16), B, H, T, Tp, H * 64, stream())
            torch.cuda.synchronize()
        assert torch.equal(o16, o), "attn16 = 1 default launch differs from the forced 8m shape"
        assert not torch.equal(o32, o), "attn16 = 0 should launch the 32x32x16 kernel"


@pytest.mark.parametrize("B,H,T", [(48, 6, 1370), (3, 5, 577), (2, 2, 256), (1, 1, 1)])
def test_attention_tail_order_bit_exact(gpu, B, H, T):
    """Switch "attn_tail" (attention.hip attn16_fwd_kernel): each sequence's
    partial last query block dispatched after every full block instead of
    the XCD-remapped (sequence, block) order.  Work order only -- every
    workgroup computes the same queries the same way -- so the output is
    bit-identical with the switch off (T % 256 == 0 and T = 1: no reorder).
    attn_tail = 2 also runs a partial block of <= 128 queries as two key
    groups of 4 query waves merged through LDS (the <8, 2> body): another
    summation order, within 2 f16 ulp of the single-group block."""
    from monocular_depth_estimation_trt_amd import _lib
    g = torch.Generator().manual_seed(B * 1000 + T)  # own stream: the module's G sequence stays as it was
    Tp = -(-T // 64) * 64
    q = torch.randn(B * H, T, 64, generator=g) * 0.125 * 2.0 * LOG2E
    k = torch.randn(B * H, T, 64, generator=g) * 2.0
    v = torch.randn(B * H, T, 64, generator=g)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    outs = []
    for tail in (1, 0, 2):
        o = torch.full((B * T, H * 64), float("nan"), dtype=torch.float16, device=gpu)
        with _lib.tuning(attn_tail=tail):
            op("mde_op_attention_cfg", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, b"8m", None, 0,
               stream())
            torch.cuda.synchronize()
        outs.append(o)
    assert torch.isfinite(outs[0].float()).all(), "every query row written"
    assert torch.equal(outs[0], outs[1]), "attn_tail changed the attention output"
    assert torch.isfinite(outs[2].float()).all(), "attn_tail = 2: every query row written"
    d = (outs[2].float() - outs[0].float()).abs().max().item()
    assert d <= 2e-3, f"attn_tail = 2 vs 1: max |d| {d:.3g}"
    if T > 1:
        ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
        close(outs[0][:4096], ref[:4096], 2e-2, 5e-3, f"attention tail order B{B} H{H} T{T}")


@pytest.mark.parametrize("cfg", ["8m", "8g2m"])
def test_attention_16x16_pending_rescale(gpu, cfg):
    """attn16 scores a tile's second 32-key block before block 0's P.V; when
    block 1 moves the running max, block 0's pending f16 P is scaled with O
    (attention.hip rescale(..., pend)).  Dominant keys only in second blocks
    (key % 64 >= 32: 50, 120, 250), each larger than the last, force that path
    in the first tile (after the FIRST block), a middle and the last tile."""
    B, H, T = 2, 3, 300
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    for key, mag in ((50, 20.0), (120, 40.0), (250, 80.0)):
        k[:, key] = q.mean(1) * mag
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    o = torch.full((B * T, H * 64), float("nan"), dtype=torch.float16, device=gpu)
    op("mde_op_attention_cfg", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, cfg.encode(), None, 0,
       stream())
    close(o, ref, 2e-2, 5e-3, f"attention {cfg} pending-P rescale")


def test_attention_spiky_rows(gpu):
    """Force the online-softmax rescale: one key dominates late in the row."""
    B, H, T = 1, 2, 300
    Tp = 320
    q = rn(B * H, T, 64) * 0.1
    k = rn(B * H, T, 64)
    k[:, 290] = q[:, :].mean(1) * 60.0                 # huge score for key 290 (last tile)
    k[:, 5] = q[:, :].mean(1) * 30.0                   # large early key
    v = rn(B * H, T, 64)
    ref = attn_ref(q, k, v).reshape(B, H, T, 64).permute(0, 2, 1, 3)
    ref = ref.reshape(B * T, H * 64)
    qg = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=gpu)
    kg = torch.zeros_like(qg)
    vtg = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=gpu)
    qg[:, :T], kg[:, :T] = q.half().to(gpu), k.half().to(gpu)
    vtg[:, :, vt_perm(T).to(gpu)] = v.transpose(1, 2).half().to(gpu)
    o = torch.empty(B * T, H * 64, dtype=torch.float16, device=gpu)
    op("mde_op_attention", ptr(qg), ptr(kg), ptr(vtg), ptr(o), B, H, T, Tp, H * 64, stream())
    close(o, ref, 2e-2, 5e-3, "attention spiky")


@pytest.mark.parametrize("D,skip", [(384, 0), (384, 1), (1024, 0), (768, 1)])
def test_layernorm(gpu, D, skip):
    B, T = 2, 50
    x = rn(B * T, D) * 3 + 1.5
    g, b = 1 + 0.1 * rn(D), 0.02 * rn(D)
    ref = F.layer_norm(x, (D,), g, b, 1e-6)
    if skip:
        ref = ref.reshape(B, T, D)[:, 1:].reshape(B * (T - 1), D)
    y = torch.empty(ref.shape, dtype=torch.float16, device=gpu)
    op("mde_op_layernorm", ptr(x.to(gpu)), ptr(y), ptr(g.to(gpu)), ptr(b.to(gpu)), B * T, D, 1e-6, T, skip,
       stream())
    close(y, ref, 1e-2, 1e-2, f"layernorm D{D} skip{skip}")


@pytest.mark.parametrize("D,skip", [(384, 0), (384, 1), (1024, 0), (768, 1), (128, 0)])
def test_layernorm_f16_stream(gpu, D, skip):
    """LayerNorm over the f16 residual stream of precision "fp16" engines."""
    B, T = 3, 50
    x = (rn(B * T, D) * 3 + 1.5).half()
    g, b = 1 + 0.1 * rn(D), 0.02 * rn(D)
    ref = F.layer_norm(x.float(), (D,), g, b, 1e-6)
    if skip:
        ref = ref.reshape(B, T, D)[:, 1:].reshape(B * (T - 1), D)
    y = torch.empty(ref.shape, dtype=torch.float16, device=gpu)
    op("mde_op_layernorm_f16", ptr(x.to(gpu)), ptr(y), ptr(g.to(gpu)), ptr(b.to(gpu)), B * T, D, 1e-6, T, skip,
       stream())
    close(y, ref, 1e-2, 1e-2, f"layernorm_f16 D{D} skip{skip}")


@pytest.mark.parametrize("B,Hh,Ww", [(2, 98, 98), (1, 126, 182), (16, 518, 518), (48, 98, 140)])
def test_patch_embed(gpu, B, Hh, Ww):
    """Patch gather (elementwise.hip patch_prep_kernel: one thread per image
    row run of a patch, so a wave reads whole image rows) + the patch-embed
    GEMM, and the gathered matrix bit-exact."""
    D = 384
    ph, pw = Hh // 14, Ww // 14
    img = rn(B, 3, Hh, Ww)
    w, b = rn(D, 3, 14, 14, scale=588 ** -0.5), rn(D, scale=0.02)
    pos, cls_pos = rn(ph * pw, D, scale=0.5), rn(D, scale=0.5)
    imc = img[..., :ph * 14, :pw * 14]
    t = F.conv2d(imc.half().float(), w.half().float(), b, stride=14).flatten(2).transpose(1, 2) + pos
    ref = torch.cat([cls_pos.expand(B, 1, D), t], 1).reshape(B * (ph * pw + 1), D)
    w16 = torch.zeros(D, 3, 14, 16)
    w16[..., :14] = w
    wp = pad_w(w16.reshape(D, 672)).to(gpu)
    scratch = torch.full((B * ph * pw, 672), float("nan"), dtype=torch.float16, device=gpu)
    x = torch.empty(B * (ph * pw + 1), D, device=gpu)
    op("mde_op_patch_embed", ptr(img.to(gpu)), B, Hh, Ww, ptr(wp), wp.shape[1], ptr(b.to(gpu)), ptr(pos.to(gpu)),
       ptr(cls_pos.to(gpu)), D, ptr(scratch), ptr(x), stream())
    close(x, ref, 1e-3, 2e-3, "patch_embed")
    # the gathered patch matrix itself, exactly: [patch][c][ky][16] f16 of the
    # image, columns 14 and 15 of every kernel row zero
    pm = torch.zeros(B, ph, pw, 3, 14, 16, dtype=torch.float16)
    pm[..., :14] = imc.half().reshape(B, 3, ph, 14, pw, 14).permute(0, 2, 4, 1, 3, 5)
    assert torch.equal(scratch.cpu(), pm.reshape(B * ph * pw, 672)), "patch matrix differs"


@pytest.mark.parametrize("B,h,w,cin,cout,stride,relu_in,act,nres", [
    (2, 19, 19, 64, 64, 1, 1, 1, 0), (1, 37, 37, 64, 64, 1, 0, 0, 2), (1, 37, 37, 384, 384, 2, 0, 0, 0),
    (1, 74, 74, 96, 64, 1, 0, 0, 0), (2, 28, 28, 48, 64, 1, 0, 0, 1), (1, 148, 148, 64, 32, 1, 0, 1, 0),
    (1, 7, 7, 256, 256, 2, 0, 0, 0), (2, 19, 19, 384, 64, 1, 1, 1, 1), (1, 19, 19, 256, 64, 2, 1, 0, 2),
    (2, 30, 45, 32, 32, 1, 1, 1, 1), (4, 296, 296, 64, 64, 1, 1, 0, 2)])
def test_conv3x3(gpu, B, h, w, cin, cout, stride, relu_in, act, nres):
    x = rn(B, cin, h, w)
    wt, b = rn(cout, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(cout, scale=0.02)
    xin = x.half().float()
    ref = F.conv2d(F.relu(xin) if relu_in else xin, wt.half().float(), b, stride=stride, padding=1)
    if act == 1:
        ref = F.relu(ref)
    res = [rn(*ref.shape) for _ in range(nres)]
    for r in res:
        ref = ref + r.half().float()
    wp = conv_w(wt).to(gpu)
    ho, wo = ref.shape[2], ref.shape[3]
    out = torch.empty(B, ho, wo, cout, dtype=torch.float16, device=gpu)
    rg = [nhwc(r).half().to(gpu) for r in res] + [None, None]
    op("mde_op_conv3x3", ptr(nhwc(x).half().to(gpu)), B, h, w, cin, ptr(wp), wp.shape[1], cout, stride, relu_in,
       ptr(b.to(gpu)), act, ptr(rg[0]), ptr(rg[1]), ptr(out), stream())
    close(nchw(out), ref, 1e-2, 1e-2, f"conv3x3 {h}x{w} {cin}->{cout} s{stride}")


@pytest.mark.parametrize("h,cin,cout", [(148, 64, 64), (148, 256, 256), (75, 128, 128)])
def test_conv_narrow_tiles_bit_exact(gpu, h, cin, cout):
    """Batch-1 grids take narrower channel tiles (conv.hip conv_tiles: 32 of 64
    channels, 64 of > 64): against torch, and bit for bit against the wide
    tiles (MDE_CONV_NARROW=0) -- an output channel's K order is the tile's,
    whatever the tile width."""
    x = rn(1, cin, h, h)
    wt, b = rn(cout, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(cout, scale=0.02)
    ref = F.relu(F.conv2d(F.relu(x.half().float()), wt.half().float(), b, padding=1))
    wp = conv_w(wt).to(gpu)
    xg, bg = nhwc(x).half().to(gpu), b.to(gpu)
    from monocular_depth_estimation_trt_amd import _lib
    got = []
    for flag in (1, 0):
        with _lib.tuning(conv_narrow=flag):
            out = torch.empty(1, h, h, cout, dtype=torch.float16, device=gpu)
            op("mde_op_conv3x3", ptr(xg), 1, h, h, cin, ptr(wp), wp.shape[1], cout, 1, 1, ptr(bg), 1, None, None,
               ptr(out), stream())
        got.append(out)
    close(nchw(got[0]), ref, 1e-2, 1e-2, f"conv narrow tiles {h}^2 {cin}->{cout}")
    assert torch.equal(got[0], got[1]), "narrow conv tiles must equal the wide ones bit for bit"


# the persistent 64-channel RCU conv (conv.hip conv64p_kernel): both RCU
# forms (conv1: ReLU'd input, bias, ReLU; conv2: bias + one or two residuals)
# on full and ragged tile grids, both tile shapes, bit for bit against the
# per-tile kernel (conv_persist=0) and against torch
@pytest.mark.parametrize("B,h,w,relu_in,act,nres,bias", [(12, 148, 148, 1, 1, 0, 1), (12, 148, 148, 0, 0, 1, 1),
                                                         (12, 148, 148, 0, 0, 2, 1), (14, 150, 133, 1, 1, 0, 1),
                                                         (14, 150, 133, 0, 0, 2, 1), (12, 148, 148, 0, 0, 0, 0),
                                                         (14, 150, 133, 0, 0, 0, 1)])
def test_conv_persist_bit_exact(gpu, B, h, w, relu_in, act, nres, bias):
    x = rn(B, 64, h, w)
    wt, b = rn(64, 64, 3, 3, scale=(9 * 64) ** -0.5), rn(64, scale=0.02)
    if not bias:
        b = torch.zeros(64)
    xin = x.half().float()
    ref = F.conv2d(F.relu(xin) if relu_in else xin, wt.half().float(), b, padding=1)
    if act:
        ref = F.relu(ref)
    res = [rn(*ref.shape) for _ in range(nres)]
    for r in res:
        ref = ref + r.half().float()
    wp = conv_w(wt).to(gpu)
    rg = [nhwc(r).half().to(gpu) for r in res] + [None, None]
    xg, bg = nhwc(x).half().to(gpu), b.to(gpu)
    from monocular_depth_estimation_trt_amd import _lib
    got = []
    for flag in (0, 1, 2):
        with _lib.tuning(conv_persist=flag):
            out = torch.empty(B, h, w, 64, dtype=torch.float16, device=gpu)
            op("mde_op_conv3x3", ptr(xg), B, h, w, 64, ptr(wp), wp.shape[1], 64, 1, relu_in, ptr(bg) if bias else None,
               act, ptr(rg[0]), ptr(rg[1]), ptr(out), stream())
        torch.cuda.synchronize()
        got.append(out)
    close(nchw(got[1]), ref, 1e-2, 1e-2, f"persistent conv {B}x{h}x{w} relu_in={relu_in} nres={nres}")
    assert torch.equal(got[1], got[0]), "persistent conv (8 x 16 tiles) must equal the per-tile kernel bit for bit"
    assert torch.equal(got[2], got[0]), "persistent conv (16 x 16 tiles) must equal the per-tile kernel bit for bit"


# E_STORE split-K (launch_gemm's small-grid policy): the batch-1 ViT-L DPT
# shapes -- layer4_rn (19^2, 1024 -> 256, im2col), layer3_rn (37^2, direct conv
# grid), conv_s2 (37^2 -> 19^2, stride 2), an RCU conv with pre-ReLU, bias,
# ReLU and two residual adds, layer2_rn (74^2, 512 -> 256)
@pytest.mark.parametrize("B,h,w,cin,cout,stride,relu_in,act,nres",
                         [(1, 19, 19, 1024, 256, 1, 0, 0, 0), (1, 37, 37, 1024, 256, 1, 0, 0, 0),
                          (1, 37, 37, 1024, 1024, 2, 0, 0, 0), (1, 37, 37, 256, 256, 1, 1, 1, 2),
                          (1, 74, 74, 512, 256, 1, 0, 0, 0), (2, 19, 19, 384, 64, 1, 1, 0, 1)])
def test_conv3x3_splitk(gpu, B, h, w, cin, cout, stride, relu_in, act, nres):
    x = rn(B, cin, h, w)
    wt, b = rn(cout, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(cout, scale=0.02)
    xin = x.half().float()
    ref = F.conv2d(F.relu(xin) if relu_in else xin, wt.half().float(), b, stride=stride, padding=1)
    if act == 1:
        ref = F.relu(ref)
    res = [rn(*ref.shape) for _ in range(nres)]
    for r in res:
        ref = ref + r.half().float()
    wp = conv_w(wt).to(gpu)
    ho, wo = ref.shape[2], ref.shape[3]
    rg = [nhwc(r).half().to(gpu) for r in res] + [None, None]
    xg, bg = nhwc(x).half().to(gpu), b.to(gpu)
    ws = torch.empty(5 << 20, dtype=torch.float32, device=gpu)
    got = []
    for cap in (0, ws.numel()):
        out = torch.empty(B, ho, wo, cout, dtype=torch.float16, device=gpu)
        sl = C.c_int(0)
        op("mde_op_conv3x3_ws", ptr(xg), B, h, w, cin, ptr(wp), wp.shape[1], cout, stride, relu_in, ptr(bg), act,
           ptr(rg[0]), ptr(rg[1]), ptr(out), ptr(ws if cap else None), cap, C.byref(sl), stream())
        assert (sl.value > 1) == (cap > 0), f"split slices {sl.value} with workspace {cap}"
        close(nchw(out), ref, 1e-2, 1e-2, f"conv3x3 split {sl.value} {h}x{w} {cin}->{cout} s{stride}")
        got.append(out.float())
    # the split only reassociates the fp32 sum
    assert (got[0] - got[1]).abs().max().item() < 2e-2


@pytest.mark.parametrize("m,n,k,act", [(1369, 256, 1024, 0), (361, 1024, 1024, 2), (1370, 384, 384, 1)])
def test_linear_splitk(gpu, m, n, k, act):
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ref = a.half().float() @ w.half().float().T + b
    ref = F.relu(ref) if act == 1 else (F.gelu(ref) if act == 2 else ref)
    wp = pad_w(w).to(gpu)
    ws = torch.empty(5 << 20, dtype=torch.float32, device=gpu)
    out = torch.empty(m, n, dtype=torch.float16, device=gpu)
    sl = C.c_int(0)
    op("mde_op_linear_ws", ptr(f16(a, gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)), act, ptr(out), n,
       ptr(ws), ws.numel(), C.byref(sl), stream())
    assert sl.value > 1 or k < 512, f"expected a split, got {sl.value}"
    close(out, ref, 1e-2, 1e-2, f"linear split {sl.value} {m}x{n}x{k} act{act}")


@pytest.mark.parametrize("B,sh,sw,uh,uw,cin,cout", [(1, 10, 10, 19, 19, 64, 32), (2, 16, 12, 28, 21, 32, 64),
                                                    (1, 148, 148, 296, 296, 64, 32), (2, 40, 40, 73, 71, 32, 32),
                                                    # separable upconv kernel: 96 / 128 channels, 1-pixel-wide map
                                                    (2, 37, 45, 64, 77, 128, 32), (1, 18, 3, 33, 5, 96, 32),
                                                    (1, 74, 74, 130, 130, 32, 32)])
def test_conv3x3_up(gpu, B, sh, sw, uh, uw, cin, cout):
    x = rn(B, cin, sh, sw)
    wt, b = rn(cout, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(cout, scale=0.02)
    up = F.interpolate(x.half().float(), size=(uh, uw), mode="bilinear", align_corners=True).half().float()
    ref = F.conv2d(up, wt.half().float(), b, padding=1)
    wp = conv_w(wt).to(gpu)
    out = torch.empty(B, uh, uw, cout, dtype=torch.float16, device=gpu)
    op("mde_op_conv3x3_up", ptr(nhwc(x).half().to(gpu)), B, sh, sw, cin, uh, uw, ptr(wp), wp.shape[1], cout,
       ptr(b.to(gpu)), 0, ptr(out), stream())
    close(nchw(out), ref, 1e-2, 1.5e-2, "conv3x3_up")


@pytest.mark.parametrize("s,cin,B,h,w", [(4, 48, 2, 7, 9), (2, 96, 2, 7, 9), (4, 256, 2, 7, 9),
                                        (4, 48, 32, 37, 37), (2, 512, 8, 37, 37),
                                        # M 16384, N 4096, K 1024: gemm256's LDS-staged E_CONVT epilogue
                                        (2, 1024, 4, 64, 64)])
def test_conv_transpose(gpu, s, cin, B, h, w):
    cout = cin
    x = rn(B, cin, h, w)
    wt, b = rn(cin, cout, s, s, scale=cin ** -0.5), rn(cout, scale=0.02)
    ref = F.conv_transpose2d(x.half().float(), wt.half().float(), b, stride=s)
    wp = pad_w(wt.permute(2, 3, 1, 0).reshape(s * s * cout, cin)).to(gpu)
    out = torch.empty(B, h * s, w * s, cout, dtype=torch.float16, device=gpu)
    op("mde_op_conv_transpose", ptr(nhwc(x).half().to(gpu)), B, h, w, cin, ptr(wp), wp.shape[1], cout, s,
       ptr(b.to(gpu)), ptr(out), stream())
    close(nchw(out), ref, 1e-2, 1e-2, f"convT s{s}")


@pytest.mark.parametrize("ih,iw,oh,ow,c", [(19, 19, 37, 37, 64), (37, 37, 74, 74, 64), (148, 148, 296, 296, 64),
                                           (4, 4, 7, 7, 256), (5, 7, 1, 9, 16), (296, 296, 518, 518, 32)])
def test_resize(gpu, ih, iw, oh, ow, c):
    B = 2
    x = rn(B, c, ih, iw)
    ref = F.interpolate(x.half().float(), size=(oh, ow), mode="bilinear", align_corners=True)
    out = torch.empty(B, oh, ow, c, dtype=torch.float16, device=gpu)
    op("mde_op_resize_bilinear", ptr(nhwc(x).half().to(gpu)), B, ih, iw, c, oh, ow, ptr(out), stream())
    close(nchw(out), ref, 1e-2, 1e-2, "resize")


def test_resize_constant_map(gpu):
    """The blend's weights sum to exactly 1 on each axis (lerp form), so a
    constant map -- e.g. the out_conv bias folded before the fusion resize --
    comes out bit-exact."""
    B, c, ih, iw, oh, ow = 2, 64, 19, 23, 37, 45
    vals = torch.tensor([0.1, -3.7, 1234.0, 6.1e-5])
    x = vals.repeat(c // 4).view(1, c, 1, 1).expand(B, c, ih, iw).contiguous()
    out = torch.empty(B, oh, ow, c, dtype=torch.float16, device=gpu)
    op("mde_op_resize_bilinear", ptr(nhwc(x).half().to(gpu)), B, ih, iw, c, oh, ow, ptr(out), stream())
    assert torch.equal(nchw(out).cpu(), x.half()[:, :, :1, :1].expand(B, c, oh, ow))


@pytest.mark.parametrize("metric", [1, 0])
def test_depth_head(gpu, metric):
    B, sh, sw, uh, uw, cin = 2, 24, 24, 42, 42, 32
    x = rn(B, cin, sh, sw)
    w1, b1 = rn(32, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(32, scale=0.02)
    w2, b2 = rn(32, scale=32 ** -0.5), 0.05
    up = F.interpolate(x.half().float(), size=(uh, uw), mode="bilinear", align_corners=True).half().float()
    h = F.relu(F.conv2d(up, w1.half().float(), b1, padding=1))
    z = (h * w2.view(1, 32, 1, 1)).sum(1) + b2
    ref = torch.sigmoid(z) * 20.0 if metric else F.relu(z)
    wp = conv_w(w1).to(gpu)
    out = torch.empty(B, uh, uw, device=gpu)
    op("mde_op_depth_head", ptr(nhwc(x).half().to(gpu)), B, sh, sw, cin, uh, uw, ptr(wp), wp.shape[1],
       ptr(b1.to(gpu)), ptr(w2.to(gpu)), b2, metric, 20.0, ptr(out), stream())
    close(out, ref, 1e-2, 2e-2, "depth_head")


@pytest.mark.parametrize("B,sh,sw,uh,uw,cin,head", [(2, 296, 296, 518, 518, 32, 1), (1, 148, 148, 296, 296, 64, 0),
                                                   (3, 21, 17, 37, 30, 32, 1), (2, 37, 45, 64, 77, 128, 0),
                                                   (1, 9, 40, 16, 70, 32, 0), (1, 1, 1, 1, 1, 32, 1),
                                                   # grids past the persistent size at 64 / 128 channels
                                                   (2, 148, 148, 296, 296, 64, 0), (2, 100, 100, 200, 200, 128, 1)])
def test_upconv_matches_conv3(gpu, B, sh, sw, uh, uw, cin, head):
    """The separable upsampling conv (conv.hip upconv_kernel: one tile per
    workgroup on small grids, persistent when the grid exceeds what the chip
    holds at once -- the last two cases) against the 4-tap conv3_kernel it
    replaces (switch "upconv" = 0) and an fp32 torch reference: the same
    two-level f16 blend in the same order, so at 32 input channels (one
    chunk, same MFMA order) the outputs are bit-identical; wider inputs sum
    32-channel chunks in another order (fp32).  Both paths are held to the
    fp32 reference (upconv's mean |error| within 1.1x of conv3's, max within
    2x) -- round 6 measured a matrix-core vertical blend against this bar
    (slower, not kept: DESIGN.md section 9)."""
    from monocular_depth_estimation_trt_amd import _lib
    x = rn(B, cin, sh, sw)
    w1, b1 = rn(32, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(32, scale=0.02)
    w2 = rn(32, scale=32 ** -0.5)
    wp = conv_w(w1).to(gpu)
    xin = nhwc(x).half().to(gpu)
    outs = []
    for flag in (0, 1):  # conv3_kernel, upconv_kernel
        with _lib.tuning(upconv=flag):
            if head:
                out = torch.empty(B, uh, uw, device=gpu)
                op("mde_op_depth_head", ptr(xin), B, sh, sw, cin, uh, uw, ptr(wp), wp.shape[1], ptr(b1.to(gpu)),
                   ptr(w2.to(gpu)), 0.05, 1, 20.0, ptr(out), stream())
            else:
                out = torch.empty(B, uh, uw, 32, dtype=torch.float16, device=gpu)
                op("mde_op_conv3x3_up", ptr(xin), B, sh, sw, cin, uh, uw, ptr(wp), wp.shape[1], 32, ptr(b1.to(gpu)),
                   0, ptr(out), stream())
            torch.cuda.synchronize()
        outs.append(out.float().cpu())
    old, new = outs
    xr = xin.float().cpu().permute(0, 3, 1, 2)
    up = F.interpolate(xr, size=(uh, uw), mode="bilinear", align_corners=True)
    hid = F.conv2d(up, w1.half().float(), b1, padding=1)
    if head:
        ref = torch.sigmoid(F.conv2d(F.relu(hid), w2.reshape(1, 32, 1, 1)) + 0.05)[:, 0] * 20.0
    else:
        ref = hid.permute(0, 2, 3, 1)
    e_old, e_new = (old - ref).abs(), (new - ref).abs()
    print(f"upconv vs fp32: mean {float(e_new.mean()):.3g} max {float(e_new.max()):.3g}; conv3: mean "
          f"{float(e_old.mean()):.3g} max {float(e_old.max()):.3g}")
    assert float(e_new.mean()) <= 1.1 * float(e_old.mean()) + 1e-6, (e_new.mean(), e_old.mean())
    assert float(e_new.max()) <= 2.0 * float(e_old.max()) + 1e-4, (e_new.max(), e_old.max())
    if cin == 32:
        assert torch.equal(old, new), (old - new).abs().max()
    else:
        assert torch.allclose(old, new, rtol=2e-3, atol=2e-3), (old - new).abs().max()


@pytest.mark.parametrize("M,N,K,act", [(1370, 3072, 1024, 2), (2740, 1024, 4096, 0), (600, 768, 768, 0)])
def test_gemm256_modes_match(gpu, M, N, K, act):
    """Switch "gemm256" (tuning.h): 0 never the 256^2 phase-pipelined kernel,
    1 the auto policy, 2 whenever legal.  Every mode against torch, and the
    modes against each other (a different tile sums K in the same 64-deep
    order per output, so 0 and 2 agree to fp32 rounding of the epilogue)."""
    from monocular_depth_estimation_trt_amd import _lib
    a = rn(M, K)
    w, b = rn(N, K, scale=K ** -0.5), rn(N, scale=0.02)
    ref = a.half().float() @ w.half().float().t() + b
    if act == 2:
        ref = F.gelu(ref)
    wp = torch.zeros(-(-N // 128) * 128, -(-K // 64) * 64, dtype=torch.float16)
    wp[:N, :K] = w.half()
    wp, ag, bg = wp.to(gpu), a.half().to(gpu), b.to(gpu)
    outs = []
    for mode in (0, 1, 2):
        with _lib.tuning(gemm256=mode):
            out = torch.empty(M, N, dtype=torch.float16, device=gpu)
            op("mde_op_linear", ptr(ag), K, ptr(wp), wp.shape[1], M, N, K, ptr(bg), act, ptr(out), N, stream())
            torch.cuda.synchronize()
        close(out, ref, 1e-2, 1e-2, f"linear gemm256={mode} {M}x{N}x{K}")
        outs.append(out.float().cpu())
    assert torch.allclose(outs[0], outs[2], rtol=2e-3, atol=2e-3), (outs[0] - outs[2]).abs().max()


def test_bad_arguments_raise(gpu):
    from monocular_depth_estimation_trt_amd._lib import MDEError
    with pytest.raises(MDEError):
        op("mde_op_linear", ptr(None), 8, ptr(None), 32, 4, 4, 8, ptr(None), 0, ptr(None), 4, stream())
    x = torch.zeros(64, device=gpu, dtype=torch.float16)
    with pytest.raises(MDEError):  # K not a multiple of 8
        op("mde_op_linear", ptr(x), 7, ptr(x), 32, 1, 1, 7, ptr(None), 0, ptr(x), 1, stream())



def ln_partials_ref(xh):
    """(sum, squared deviations from the slice mean) per 32-column slice and
    row of f16 rows, fp64, slice-major [k/32][m][2] (GemmParams::lnst_*)."""
    v = xh.double().reshape(xh.shape[0], -1, 32)
    m2 = ((v - v.mean(-1, keepdim=True)) ** 2).sum(-1)
    return torch.stack([v.sum(-1), m2], -1).transpose(0, 1).contiguous()


@pytest.mark.parametrize("m,n,k", [(300, 384, 384), (38360, 384, 384), (1370, 384, 1536), (2740, 1024, 1024),
                                   # >= 512 tiles of 256 x 128: the 8-wave residual tile (gemm.hip dispatch)
                                   (43840, 384, 384), (43850, 384, 1536)])
def test_linear_residual_f16(gpu, m, n, k):
    """proj / fc2 over the f16 residual stream of precision "fp16" engines:
    xh += ls * (a W^T + b), fp32 update, one rounding to f16; plus the
    folded-LayerNorm partials of the rows written (64^2 and 128^2 tiles)."""
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ls = 0.5 + 0.1 * rn(n)
    x0 = (rn(m, n) * 2).half()
    ref = x0.float() + ls * (a.half().float() @ w.half().float().T + b)
    wp = pad_w(w).to(gpu)
    xh = x0.to(gpu)
    part = torch.full((n // 32, m, 2), float("nan"), device=gpu)
    op("mde_op_linear_residual_f16", ptr(f16(a, gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)),
       ptr(ls.to(gpu)), ptr(xh), n, ptr(part), stream())
    close(xh, ref, 1e-2, 1e-2, f"linear_residual_f16 m{m}")
    # partials of exactly the f16 values written (fp32 sums of <= 32 terms)
    close(part, ln_partials_ref(xh.cpu()).float(), 1e-5, 1e-3, "ln partials")


@pytest.mark.parametrize("m,n,k,act", [(300, 1152, 384, 0), (38360, 1536, 384, 2), (1370, 2048, 512, 2), (1370, 3072, 1024, 2), (10960, 4096, 1024, 2), (2740, 3072, 768, 0),
                                       (5, 64, 384, 0)])
def test_linear_lnfold(gpu, m, n, k, act):
    """LayerNorm folded into the next linear: act(LN(x) W^T + b) from the
    raw f16 rows, W * gamma, c1, c2 and the row partials -- against the
    reference order (LN in fp32, rounded to f16, then the linear)."""
    x = (rn(m, k) * 2 + 0.7).half()
    g, bt = 1 + 0.2 * rn(k), 0.05 * rn(k)
    w, b = rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ref = F.layer_norm(x.float(), (k,), g, bt, 1e-6).half().float() @ w.half().float().T + b
    if act == 2:
        ref = F.gelu(ref)
    wg = (w.double() * g.double()[None, :]).float()
    c1 = wg.half().double().sum(1).float()
    c2 = (b.double() + w.half().double() @ bt.double()).float()
    wgp = pad_w(wg).to(gpu)
    part = ln_partials_ref(x).float().to(gpu)
    out = torch.empty(m, n, dtype=torch.float16, device=gpu)
    op("mde_op_linear_lnfold", ptr(x.to(gpu)), ptr(part), 1e-6, ptr(wgp), wgp.shape[1], ptr(c1.to(gpu)),
       ptr(c2.to(gpu)), m, n, k, act, ptr(out), n, stream())
    close(out, ref, 1e-2, 1.5e-2, f"linear_lnfold {m}x{n}x{k}")


# ---- exact-fp32 kernels (fp32.hip; precision "fp32" engines) -----------------
# fp32 operands and accumulation on v_mfma_f32_16x16x4_f32 / 32x32x2_f32: the
# only differences from a float64 reference are fp32 rounding and summation
# order (K up to 4096: relative error ~1e-6), so the bars are three orders of
# magnitude tighter than the f16 kernels' (stated per test).

def pad_w32(w, n_mult=128, k_mult=32):
    n, k = w.shape
    out = torch.zeros(-(-n // n_mult) * n_mult, -(-k // k_mult) * k_mult, dtype=torch.float32)
    out[:n, :k] = w
    return out


@pytest.mark.parametrize("m,n,k,act", [(1370, 1152, 384, 0), (2740, 1536, 384, 2), (1370, 384, 1536, 1),
                                       (43840, 1536, 384, 2), (77, 96, 40, 0)])
def test_linear32(gpu, m, n, k, act):
    """mde_op_linear32 vs a float64 torch reference: 64^2 tiles (small grids)
    and 128^2 tiles (>= 512 of them), K tails (40 = 32 + 8), GELU(erf) / ReLU."""
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ref = a.double() @ w.double().T + b.double()
    ref = F.relu(ref) if act == 1 else (F.gelu(ref) if act == 2 else ref)
    wp = pad_w32(w).to(gpu)
    out = torch.empty(m, n, device=gpu)
    op("mde_op_linear32", ptr(a.to(gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)), act, ptr(out), n,
       stream())
    close(out, ref.float(), 2e-5, 2e-5, f"linear32 {m}x{n}x{k} act{act}")


def test_linear32_k_below_one_step(gpu):
    """K = 16 < one 32-deep K-step, A rows padded to lda = 32 with NaN: the
    tail lanes must not read columns >= K (NaN * 0 = NaN)."""
    m, n, k, lda = 77, 96, 16, 32
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ap = torch.full((m, lda), float("nan"))
    ap[:, :k] = a
    ref = F.relu(a.double() @ w.double().T + b.double())
    wp = pad_w32(w).to(gpu)
    out = torch.empty(m, n, device=gpu)
    op("mde_op_linear32", ptr(ap.to(gpu)), lda, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)), 1, ptr(out), n,
       stream())
    assert torch.isfinite(out).all()
    close(out, ref.float(), 2e-5, 2e-5, "linear32 K=16")


@pytest.mark.parametrize("B,h,w,cin,cout,stride,relu_in,act,res", [
    (2, 20, 22, 48, 64, 1, 0, 0, 0),     # layer1_rn: 48 input channels (ViT-S), K = 432 (tail)
    (1, 37, 37, 64, 64, 1, 1, 1, 0),     # RCU conv1: ReLU on the operand and the output
    (2, 19, 19, 64, 64, 1, 0, 0, 2),     # RCU conv2: + x + fusion skip
    (1, 37, 37, 384, 384, 2, 0, 0, 0),   # resize_layers.3: stride 2
    (1, 41, 53, 32, 32, 1, 0, 1, 0),     # output_conv2 shape (32 -> 32, ReLU)
])
def test_conv3x3_32(gpu, B, h, w, cin, cout, stride, relu_in, act, res):
    """The exact-fp32 DPT head's conv (implicit im2col on the fp32 MFMA)
    against a float64 torch conv2d: fp32 rounding only (2e-5)."""
    x, wt, b = rn(B, cin, h, w), rn(cout, cin, 3, 3, scale=(9 * cin) ** -0.5), rn(cout, scale=0.1)
    xin = F.relu(x.double()) if relu_in else x.double()
    ref = F.conv2d(xin, wt.double(), b.double(), stride=stride, padding=1)
    if act:
        ref = F.relu(ref)
    r0 = rn(*ref.shape) if res >= 1 else None
    r1 = rn(*ref.shape) if res >= 2 else None
    if r0 is not None:
        ref = ref + r0.double()
    if r1 is not None:
        ref = ref + r1.double()
    wp = pad_w32(wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin)).to(gpu)
    oh, ow = ref.shape[2], ref.shape[3]
    out = torch.empty(B, oh, ow, cout, device=gpu)
    keep = [nhwc(t).contiguous().to(gpu) for t in (r0, r1) if t is not None]
    op("mde_op_conv3x3_32", ptr(nhwc(x).contiguous().to(gpu)), B, h, w, cin, ptr(wp), wp.shape[1], cout, stride,
       relu_in, ptr(b.to(gpu)), act, ptr(keep[0]) if len(keep) > 0 else None, ptr(keep[1]) if len(keep) > 1 else None,
       ptr(out), stream())
    close(nchw(out), ref.float(), 2e-5, 2e-5, f"conv3x3_32 {h}x{w} {cin}->{cout} s{stride}")


@pytest.mark.parametrize("s,cin,cout,B,h,w", [(4, 48, 48, 2, 7, 9), (2, 96, 96, 1, 37, 37), (4, 256, 256, 1, 5, 5)])
def test_conv_transpose32(gpu, s, cin, cout, B, h, w):
    """resize_layers 0 / 1 (ConvTranspose k = s) in fp32 against float64 torch."""
    x = rn(B, cin, h, w)
    wt, b = rn(cin, cout, s, s, scale=cin ** -0.5), rn(cout, scale=0.02)
    ref = F.conv_transpose2d(x.double(), wt.double(), b.double(), stride=s)
    wp = pad_w32(wt.permute(2, 3, 1, 0).reshape(s * s * cout, cin)).to(gpu)
    out = torch.empty(B, h * s, w * s, cout, device=gpu)
    op("mde_op_conv_transpose32", ptr(nhwc(x).contiguous().to(gpu)), B, h, w, cin, ptr(wp), wp.shape[1], cout, s,
       ptr(b.to(gpu)), ptr(out), stream())
    close(nchw(out), ref.float(), 2e-5, 2e-5, f"convT32 s{s}")


@pytest.mark.parametrize("ih,iw,oh,ow,c", [(19, 19, 37, 37, 64), (148, 148, 296, 296, 64), (296, 296, 518, 518, 32),
                                           (28, 37, 56, 74, 256), (5, 7, 1, 9, 16)])
def test_resize32(gpu, ih, iw, oh, ow, c):
    """fp32 bilinear align_corners against torch's fp32 F.interpolate (the
    same index math: fp32 source coordinate, then the two-axis blend)."""
    B = 2
    x = rn(B, c, ih, iw)
    ref = F.interpolate(x, size=(oh, ow), mode="bilinear", align_corners=True)
    out = torch.empty(B, oh, ow, c, device=gpu)
    op("mde_op_resize32", ptr(nhwc(x).contiguous().to(gpu)), B, ih, iw, c, oh, ow, ptr(out), stream())
    close(nchw(out), ref, 2e-6, 2e-6, "resize32")


def test_linear_residual32(gpu):
    m, n, k = 1370, 384, 1536
    a, w, b = rn(m, k), rn(n, k, scale=k ** -0.5), rn(n, scale=0.1)
    ls = 0.5 + 0.05 * rn(n)
    x = rn(m, n) * 1e5  # far past the f16 range: fp32 storage end to end
    ref = x.double() + ls.double() * (a.double() @ w.double().T + b.double())
    xg = x.clone().to(gpu)
    wp = pad_w32(w).to(gpu)
    op("mde_op_linear_residual32", ptr(a.to(gpu)), k, ptr(wp), wp.shape[1], m, n, k, ptr(b.to(gpu)),
       ptr(ls.to(gpu)), ptr(xg), n, stream())
    close(xg, ref.float(), 2e-6, 2e-3, "linear_residual32")


@pytest.mark.parametrize("B,T,H", [(2, 50, 6), (1, 1370, 6)])
def test_qkv32_layout(gpu, B, T, H):
    """E_QKV of the fp32 GEMM: q (scaled) / k / v as fp32 [B*H][Tpad][64] rows."""
    D = H * 64
    Tp = -(-T // 64) * 64
    a, w, b = rn(B * T, D), rn(3 * D, D, scale=D ** -0.5), rn(3 * D, scale=0.1)
    y = (a.double() @ w.double().T + b.double()).reshape(B, T, 3, H, 64).permute(2, 0, 3, 1, 4).reshape(3, B * H, T, 64)
    qs = 0.125 * LOG2E
    wp = pad_w32(w).to(gpu)
    q, k, v = (torch.zeros(B * H, Tp, 64, device=gpu) for _ in range(3))
    op("mde_op_qkv32", ptr(a.to(gpu)), ptr(wp), wp.shape[1], ptr(b.to(gpu)), B, T, H, Tp, qs, ptr(q), ptr(k), ptr(v),
       stream())
    close(q[:, :T], (y[0] * qs).float(), 2e-5, 2e-5, "qkv32 q")
    close(k[:, :T], y[1].float(), 2e-5, 2e-5, "qkv32 k")
    close(v[:, :T], y[2].float(), 2e-5, 2e-5, "qkv32 v")
    assert float(q[:, T:].abs().max()) == 0.0 if Tp > T else True


@pytest.mark.parametrize("B,H,T", [(1, 6, 1370), (2, 3, 50), (1, 1, 1), (4, 6, 300), (1, 16, 1370), (24, 6, 1370)])
def test_attention32(gpu, B, H, T):
    """mde_op_attention32 vs float64 softmax: the key-group form (small grids,
    4 waves on one 32-query block, merged through LDS) and the 128-query form
    (B = 24 at 1370: >= 512 workgroups); masked key tails at every T % 32."""
    Tp = -(-T // 64) * 64
    q = rn(B * H, T, 64) * 0.125 * 2.0 * LOG2E
    k = rn(B * H, T, 64) * 2.0
    v = rn(B * H, T, 64)
    ref = torch.softmax((q.double() @ k.double().transpose(1, 2)) / LOG2E, dim=-1) @ v.double()
    ref = ref.reshape(B, H, T, 64).permute(0, 2, 1, 3).reshape(B * T, H * 64)
    qg, kg, vg = (torch.zeros(B * H, Tp, 64, device=gpu) for _ in range(3))
    qg[:, :T], kg[:, :T], vg[:, :T] = q.to(gpu), k.to(gpu), v.to(gpu)
    o = torch.empty(B * T, H * 64, device=gpu)
    op("mde_op_attention32", ptr(qg), ptr(kg), ptr(vg), ptr(o), B, H, T, Tp, H * 64, stream())
    close(o, ref.float(), 1e-4, 1e-5, f"attention32 B{B} H{H} T{T}")
