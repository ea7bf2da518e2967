"""Generate the committed VGGT golden fixtures (run in the dev container only).

    python tests/golden/make_golden_vggt.py

Two pins for the VGGT oracle (oracle/vggt_ref.py):

1. vggt_export_compat.npz -- outputs of the reference's OWN export patches,
   imported from /root/reference/core/export_compat.py and executed here:
     * no_cartesian_prod (export_compat.py:84-93): the RoPE patch-grid
       positions PositionGetter returns at 37x37 (518^2), 7x7 (98^2) and a
       5x9 grid, batch 2;
     * float32_sincos_pos_embed (export_compat.py:145-152): the fp32
       make_sincos_pos_embed the reference's engine computes, for the UV grid
       coordinates of a 37-wide map and for embed dims 64 / 128.
   Stored are the inputs and outputs only (data, no reference source).
2. vggt_dino_tiny.npz -- transformers' Dinov2WithRegistersModel (in-container,
   built from a LOCAL config, nothing fetched) loaded with the seeded "tiny"
   VGGT weights' aggregator.patch_embed.* tensors: the normalised input and
   HF's final-norm patch tokens, against which the oracle's DINOv2-with-
   registers encoder (the aggregator's patch embedding) is checked.

The aggregator blocks and the DPT head have no executable reference in this
container (upstream vggt is cloned at run time and not vendored; transformers
has no VGGT): those parts of the oracle stay unpinned.
"""

from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from monocular_depth_estimation_trt_amd import weights_vggt as WV  # noqa: E402
from oracle import vggt_ref  # noqa: E402


def export_compat_case() -> dict:
    sys.path.insert(0, REF)
    from core import export_compat as EC   # the reference's own module (study + vectors only)

    class Getter:   # a PositionGetter-shaped holder: the patch replaces __call__
        def __init__(self):
            self.position_cache = {}

    rec = {}
    with EC.no_cartesian_prod(Getter):
        g = Getter()
        for h, w in ((37, 37), (7, 7), (5, 9)):
            pos = g(2, h, w, torch.device("cpu"))
            rec[f"pos_{h}x{w}"] = pos.numpy().astype(np.int64)
            mine = vggt_ref.position_grid(h, w)
            assert torch.equal(pos[0], mine) and torch.equal(pos[1], mine), (h, w)
    holder = types.SimpleNamespace(make_sincos_pos_embed=None)
    coords = vggt_ref.create_uv_grid(37, 37, 1.0).reshape(-1, 2)
    rec["uv_37"] = coords.numpy()
    with EC.float32_sincos_pos_embed(holder):
        for dim in (64, 128):
            for axis in (0, 1):
                out = holder.make_sincos_pos_embed(dim // 2, coords[:, axis], 100)
                rec[f"sincos_{dim}_{axis}"] = out.numpy()
                mine = vggt_ref.make_sincos_pos_embed(dim // 2, coords[:, axis], 100)
                err = float((out - mine).abs().max())
                print(f"sincos dim {dim} axis {axis}: reference fp32 patch vs oracle max_abs {err:.3e}")
                assert err < 1e-6
    return rec


def hf_dino(cfg: dict):
    from transformers import Dinov2WithRegistersConfig, Dinov2WithRegistersModel
    c = Dinov2WithRegistersConfig(hidden_size=cfg["embed_dim"], num_hidden_layers=cfg["depth"],
                                  num_attention_heads=cfg["num_heads"], mlp_ratio=4, hidden_act="gelu",
                                  layer_norm_eps=cfg["ln_eps"], image_size=cfg["img"], patch_size=cfg["patch"],
                                  qkv_bias=True, layerscale_value=1.0, num_register_tokens=WV.NUM_REG,
                                  use_swiglu_ffn=False)
    return Dinov2WithRegistersModel(c).eval()


def upstream_dino_to_hf(sd: dict, cfg: dict) -> dict:
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    D = cfg["embed_dim"]
    p = "aggregator.patch_embed."
    o = {"embeddings.cls_token": t[p + "cls_token"], "embeddings.mask_token": t[p + "mask_token"],
         "embeddings.register_tokens": t[p + "register_tokens"],
         "embeddings.position_embeddings": t[p + "pos_embed"],
         "embeddings.patch_embeddings.projection.weight": t[p + "patch_embed.proj.weight"],
         "embeddings.patch_embeddings.projection.bias": t[p + "patch_embed.proj.bias"],
         "layernorm.weight": t[p + "norm.weight"], "layernorm.bias": t[p + "norm.bias"]}
    for i in range(cfg["depth"]):
        b, hb = f"{p}blocks.{i}.", f"encoder.layer.{i}."
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
    return o


def dino_case(seed: int = 2468) -> dict:
    cfg = WV.vggt_config("tiny")
    sd = WV.synthetic_state_dict(cfg, seed)
    x = WV.synthetic_images(2, 1, cfg["img"], first_seed=100)[:, 0]
    mean = torch.tensor(WV.RESNET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(WV.RESNET_STD).view(1, 3, 1, 1)
    xn = (torch.from_numpy(x) - mean) / std
    model = hf_dino(cfg)
    model.load_state_dict(upstream_dino_to_hf(sd, cfg), strict=True)
    with torch.no_grad():
        hf = model(pixel_values=xn).last_hidden_state[:, 1 + WV.NUM_REG:].numpy()
        mine = vggt_ref.dinov2_reg(vggt_ref.to_torch(sd), cfg, xn).numpy()
    err = np.abs(hf - mine).max()
    print(f"dinov2-reg tiny: HF vs oracle max_abs {err:.3e}")
    assert err < 1e-4
    return dict(seed=np.array(seed), weights_sha256=np.array(WV.state_dict_digest(sd)), input_norm=xn.numpy(),
                tokens_hf=hf.astype(np.float32))


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    np.savez_compressed(os.path.join(HERE, "vggt_export_compat.npz"), **export_compat_case())
    np.savez_compressed(os.path.join(HERE, "vggt_dino_tiny.npz"), **dino_case())


if __name__ == "__main__":
    main()
