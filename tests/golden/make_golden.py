"""Generate the committed golden fixtures (run in the dev container only).

    python tests/golden/make_golden.py

Pins the oracle (oracle/dav2_ref.py) against transformers'
`DepthAnythingForDepthEstimation` + `Dinov2Backbone` (5.15.0, in-container),
built from a LOCAL config -- no `from_pretrained`, nothing fetched -- and
loaded with the same seeded synthetic upstream-keyed weights the oracle and
the HIP engine use (monocular_depth_estimation_trt_amd/weights.py), mapped to
HF key names.  The upstream Depth-Anything-V2 repo the reference clones at
run time is absent here, so HF is the executable stand-in.

Fixtures written (small, npz, float32 unless noted):
  dav2_vits_metric_98.npz    B=2 98x98 ViT-S metric: input, HF output, digest
  dav2_vits_relative_98.npz  B=1 98x98 ViT-S relative head
  dav2_vitb_relative_98.npz  B=1 98x98 ViT-B relative head (D=768, 12 heads, F=128)
  dav2_vitl_metric_98.npz    B=1 98x98 ViT-L metric (taps 4/11/17/23, F=256)
  dav2_vits_metric_518.npz   B=1 518x518 ViT-S metric: the full output map
                             stored in float16 (0.5 MB) + full-map stats;
                             the input is regenerated from its seed
  dav2_vitl_metric_518.npz   B=1 518x518 ViT-L metric (BASELINE config 3's
                             per-GPU unit), stored the same way
  posembed_upstream.npz      pos-embed interpolation 37x37 -> 7x7 and 9x13
                             (torch bicubic, 0.1 offset), checked against an
                             independent numpy restatement of that formula

The 98x98 cases give HF a 7x7 positional grid directly (config image_size=98),
with the upstream interpolation of the 37x37 table done once beforehand, so
HF's own (different, size-based) interpolation path is never taken.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from monocular_depth_estimation_trt_amd import weights as W  # noqa: E402
from oracle import dav2_ref  # noqa: E402


def hf_model(cfg: dict, image_size: int):
    from transformers import DepthAnythingConfig, DepthAnythingForDepthEstimation, Dinov2Config
    n = cfg["depth"]
    bb = Dinov2Config(image_size=image_size, patch_size=cfg["patch"], hidden_size=cfg["embed_dim"],
                      num_hidden_layers=n, num_attention_heads=cfg["num_heads"], mlp_ratio=4,
                      out_indices=[t + 1 for t in cfg["taps"]], apply_layernorm=True,
                      reshape_hidden_states=False, layer_norm_eps=cfg["ln_eps"], layerscale_value=1.0,
                      hidden_act="gelu", qkv_bias=True)
    c = DepthAnythingConfig(backbone_config=bb, neck_hidden_sizes=cfg["out_channels"],
                            fusion_hidden_size=cfg["features"], head_hidden_size=cfg["head_hidden"],
                            depth_estimation_type=cfg["depth_type"], max_depth=int(cfg["max_depth"]),
                            patch_size=cfg["patch"], reassemble_factors=[4, 2, 1, 0.5],
                            reassemble_hidden_size=cfg["embed_dim"])
    return DepthAnythingForDepthEstimation(c).eval()


def upstream_to_hf(sd: dict, cfg: dict, ph: int, pw: int) -> dict:
    """Upstream DA-V2 key names -> transformers key names."""
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    D = cfg["embed_dim"]
    o = {}
    p = "pretrained."
    e = "backbone.embeddings."
    o[e + "cls_token"] = t[p + "cls_token"]
    o[e + "mask_token"] = t[p + "mask_token"]
    o[e + "position_embeddings"] = dav2_ref.interpolate_pos_embed(t[p + "pos_embed"], ph, pw)
    o[e + "patch_embeddings.projection.weight"] = t[p + "patch_embed.proj.weight"]
    o[e + "patch_embeddings.projection.bias"] = t[p + "patch_embed.proj.bias"]
    for i in range(cfg["depth"]):
        b, hb = f"{p}blocks.{i}.", f"backbone.encoder.layer.{i}."
        for n in ("norm1", "norm2"):
            o[hb + n + ".weight"] = t[b + n + ".weight"]
            o[hb + n + ".bias"] = t[b + n + ".bias"]
        qw, qb = t[b + "attn.qkv.weight"], t[b + "attn.qkv.bias"]
        for j, n in enumerate(("query", "key", "value")):
            o[f"{hb}attention.attention.{n}.weight"] = qw[j * D:(j + 1) * D]
            o[f"{hb}attention.attention.{n}.bias"] = qb[j * D:(j + 1) * D]
        o[hb + "attention.output.dense.weight"] = t[b + "attn.proj.weight"]
        o[hb + "attention.output.dense.bias"] = t[b + "attn.proj.bias"]
        o[hb + "layer_scale1.lambda1"] = t[b + "ls1.gamma"]
        o[hb + "layer_scale2.lambda1"] = t[b + "ls2.gamma"]
        for n in ("fc1", "fc2"):
            o[f"{hb}mlp.{n}.weight"] = t[f"{b}mlp.{n}.weight"]
            o[f"{hb}mlp.{n}.bias"] = t[f"{b}mlp.{n}.bias"]
    o["backbone.layernorm.weight"] = t[p + "norm.weight"]
    o["backbone.layernorm.bias"] = t[p + "norm.bias"]
    h = "depth_head."
    r = "neck.reassemble_stage.layers."
    for i in range(4):
        o[f"{r}{i}.projection.weight"] = t[f"{h}projects.{i}.weight"]
        o[f"{r}{i}.projection.bias"] = t[f"{h}projects.{i}.bias"]
    for i in (0, 1, 3):
        o[f"{r}{i}.resize.weight"] = t[f"{h}resize_layers.{i}.weight"]
        o[f"{r}{i}.resize.bias"] = t[f"{h}resize_layers.{i}.bias"]
    for i in range(4):
        o[f"neck.convs.{i}.weight"] = t[f"{h}scratch.layer{i + 1}_rn.weight"]
    for j in range(4):
        up, hf = f"{h}scratch.refinenet{4 - j}.", f"neck.fusion_stage.layers.{j}."
        o[hf + "projection.weight"] = t[up + "out_conv.weight"]
        o[hf + "projection.bias"] = t[up + "out_conv.bias"]
        for u in (1, 2):
            for c in (1, 2):
                for kind in ("weight", "bias"):
                    o[f"{hf}residual_layer{u}.convolution{c}.{kind}"] = t[f"{up}resConfUnit{u}.conv{c}.{kind}"]
    s = h + "scratch."
    for a, bname in (("output_conv1", "conv1"), ("output_conv2.0", "conv2"), ("output_conv2.2", "conv3")):
        o[f"head.{bname}.weight"] = t[f"{s}{a}.weight"]
        o[f"head.{bname}.bias"] = t[f"{s}{a}.bias"]
    return o


def run_case(name, encoder, depth_type, batch, size, seed=1234, full=True):
    cfg = W.model_config(encoder, depth_type)
    sd = W.synthetic_state_dict(cfg, seed)
    x = W.synthetic_images(batch, size, size, first_seed=100)
    ph = pw = size // cfg["patch"]
    model = hf_model(cfg, size)
    hf_sd = upstream_to_hf(sd, cfg, ph, pw)
    missing, unexpected = model.load_state_dict(hf_sd, strict=True), None
    with torch.no_grad():
        y_hf = model(torch.from_numpy(x)).predicted_depth.numpy()
        y_or = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    err = np.abs(y_hf - y_or)
    rel = err.mean() / np.abs(y_hf).mean()
    print(f"{name}: out {y_hf.shape} range [{y_hf.min():.4f}, {y_hf.max():.4f}] "
          f"mean {y_hf.mean():.4f}  oracle-vs-HF max_abs {err.max():.3e} rel_mean {rel:.3e}")
    assert err.max() < 1e-3 and rel < 1e-5, (name, err.max(), rel)
    rec = dict(encoder=np.array(encoder), depth_type=np.array(depth_type), seed=np.array(seed),
               input_first_seed=np.array(100), batch=np.array(batch), size=np.array(size),
               weights_sha256=np.array(W.state_dict_digest(sd)),
               out_min=np.float64(y_hf.min()), out_max=np.float64(y_hf.max()),
               out_mean=np.float64(y_hf.mean()), out_std=np.float64(y_hf.std()))
    if full:
        rec["input"] = x
        rec["output_hf"] = y_hf.astype(np.float32)
    else:
        # full map at f16 (quantisation <= 2^-11 relative, far below the
        # engine tolerance); the input is regenerated from input_first_seed
        rec["output_hf_f16"] = y_hf.astype(np.float16)
        q = np.abs(rec["output_hf_f16"].astype(np.float64) - y_hf).max()
        print(f"  f16 storage max quantisation {q:.2e}")
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)


def _cubic_w(t, A=-0.75):
    """Keys cubic convolution weights (A=-0.75, PyTorch's bicubic)."""
    def c1(x):  # |x| <= 1
        return ((A + 2) * x - (A + 3)) * x * x + 1
    def c2(x):  # 1 < |x| < 2
        return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A
    return np.array([c2(t + 1), c1(t), c1(1 - t), c2(2 - t)])


def numpy_pos_interp(pos: np.ndarray, ph: int, pw: int) -> np.ndarray:
    """Independent restatement of upstream's F.interpolate(bicubic,
    scale_factor=((ph+0.1)/M, (pw+0.1)/M), align_corners=False): source
    coordinate = (dst + 0.5) / scale - 0.5, border-clamped taps."""
    N = pos.shape[1] - 1
    M = int(round(np.sqrt(N)))
    D = pos.shape[-1]
    g = pos[0, 1:].reshape(M, M, D).astype(np.float64)

    def axis_weights(n_out, scale):
        rows = []
        for d in range(n_out):
            src = (d + 0.5) / scale - 0.5
            i0 = int(np.floor(src))
            wts = _cubic_w(src - i0)
            idx = [min(max(i0 - 1 + k, 0), M - 1) for k in range(4)]
            r = np.zeros(M)
            for k in range(4):
                r[idx[k]] += wts[k]
            rows.append(r)
        return np.stack(rows)

    Ay = axis_weights(ph, (ph + 0.1) / M)
    Ax = axis_weights(pw, (pw + 0.1) / M)
    out = np.einsum("ym,mnd,xn->yxd", Ay, g, Ax).reshape(ph * pw, D)
    return np.concatenate([pos[0, :1].astype(np.float64), out], 0)[None].astype(np.float32)


def pos_case():
    cfg = W.model_config("vits")
    sd = W.synthetic_state_dict(cfg, 1234)
    pos = sd["pretrained.pos_embed"]
    rec = {}
    for ph, pw in ((7, 7), (9, 13)):
        t = dav2_ref.interpolate_pos_embed(torch.from_numpy(pos), ph, pw).numpy()
        n = numpy_pos_interp(pos, ph, pw)
        e = np.abs(t - n).max()
        print(f"pos interp {ph}x{pw}: torch vs numpy max_abs {e:.3e}")
        assert e < 1e-5
        rec[f"pos_{ph}x{pw}"] = t
    rec["pos_37_first_rows"] = pos[:, :8]
    np.savez_compressed(os.path.join(HERE, "posembed_upstream.npz"), **rec)


CASES = {
    "dav2_vits_metric_98": ("vits", "metric", 2, 98, True),
    "dav2_vits_relative_98": ("vits", "relative", 1, 98, True),
    "dav2_vitb_relative_98": ("vitb", "relative", 1, 98, True),
    "dav2_vitl_metric_98": ("vitl", "metric", 1, 98, True),
    "dav2_vits_metric_518": ("vits", "metric", 1, 518, False),
    "dav2_vitl_metric_518": ("vitl", "metric", 1, 518, False),
}


def main():
    """python tests/golden/make_golden.py [case ...]  (default: all + pos-embed)"""
    torch.set_num_threads(os.cpu_count() or 8)
    only = sys.argv[1:]
    if not only:
        pos_case()
    for name, (enc, dt, b, size, full) in CASES.items():
        if not only or name in only:
            run_case(name, enc, dt, b, size, full=full)


if __name__ == "__main__":
    main()
