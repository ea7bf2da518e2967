"""Generate the committed Depth Pro golden fixtures (dev container only).

    python tests/golden/make_golden_depth_pro.py

Pins the oracle (oracle/depth_pro_ref.py) against transformers'
`DepthProForDepthEstimation` (5.15.0, in-container), built from a LOCAL
config -- no `from_pretrained`, nothing fetched -- and loaded with the seeded
synthetic HF-keyed weights of monocular_depth_estimation_trt_amd/
weights_depth_pro.py.  apple/ml-depth-pro, which the reference clones at run
time, is absent here, so HF is the executable stand-in.

The fixtures use the "tiny" preset: the full 1536x1536 geometry (35 patches of
384^2, 24x24 tokens, identity merges, 5 fusion levels, 768^2 / 1536^2 head)
with narrow layers.  The input (synthetic_images, seeds 200..) is regenerated
by the tests, not stored; outputs are stored subsampled every 8th pixel with
full-map statistics, plus the FOV scalars.

  depth_pro_tiny_b2.npz          B=2, use_fov=True
  depth_pro_shallow_b1.npz       B=1, use_fov=True, the "dinov2l16_384_shallow"
                                 preset: the real widths (D 1024, 16 heads,
                                 decoder 256, scaled dims 1024/1024/512) with 4
                                 blocks per encoder; output every 2nd pixel in
                                 f16 (768x768) + full-map statistics
  depth_pro_full_b1.npz          B=1, use_fov=True, the full "dinov2l16_384"
                                 preset (24 blocks per encoder, hooks [11, 5]):
                                 the bench model itself; output every 2nd
                                 pixel in f16 + full-map statistics + FOV
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from monocular_depth_estimation_trt_amd import weights_depth_pro as WD  # noqa: E402
from oracle import depth_pro_ref  # noqa: E402


def hf_config(cfg: dict):
    from transformers import DepthProConfig
    sub = dict(model_type="dinov2", image_size=cfg["vit_size"], patch_size=cfg["patch"],
               hidden_size=cfg["embed_dim"], num_hidden_layers=cfg["depth"], num_attention_heads=cfg["num_heads"],
               mlp_ratio=4, layerscale_value=1.0, qkv_bias=True, layer_norm_eps=cfg["ln_eps"], hidden_act="gelu",
               use_swiglu_ffn=False)
    return DepthProConfig(
        fusion_hidden_size=cfg["fusion"], patch_size=cfg["vit_size"], intermediate_hook_ids=list(cfg["hooks"]),
        intermediate_feature_dims=list(cfg["inter_dims"]), scaled_images_ratios=list(cfg["ratios"]),
        scaled_images_overlap_ratios=list(cfg["overlaps"]), scaled_images_feature_dims=list(cfg["scaled_dims"]),
        merge_padding_value=cfg["merge_pad"], use_batch_norm_in_fusion_residual=False,
        use_bias_in_fusion_residual=True, use_fov_model=cfg["use_fov"], num_fov_head_layers=cfg["fov_layers"],
        image_model_config=dict(sub), patch_model_config=dict(sub), fov_model_config=dict(sub))


def run_case(name, preset, batch, use_fov=True, seed=4321, first_seed=200, sub=8, f16=False):
    from transformers import DepthProForDepthEstimation
    cfg = WD.depth_pro_config(preset, use_fov=use_fov)
    sd = WD.synthetic_state_dict(cfg, seed)
    x = WD.synthetic_images(batch, cfg["img"], first_seed=first_seed)
    model = DepthProForDepthEstimation(hf_config(cfg)).eval()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        out = model(torch.from_numpy(x))
        y_hf = out.predicted_depth.numpy()
        fov_hf = out.field_of_view.numpy() if use_fov else None
        y_or, fov_or = depth_pro_ref.forward(depth_pro_ref.to_torch(sd), cfg, x)
    y_or = y_or.numpy()
    err = np.abs(y_hf - y_or)
    rel = err.mean() / np.abs(y_hf).mean()
    pos = float((y_hf > 0).mean())
    print(f"{name}: out {y_hf.shape} range [{y_hf.min():.4f}, {y_hf.max():.4f}] mean {y_hf.mean():.4f} "
          f"positive {pos:.3f}; oracle-vs-HF max_abs {err.max():.3e} rel_mean {rel:.3e}")
    assert err.max() < 1e-3 and rel < 1e-5, (name, err.max(), rel)
    rec = dict(preset=np.array(preset), seed=np.array(seed), input_first_seed=np.array(first_seed),
               batch=np.array(batch), use_fov=np.array(int(use_fov)),
               weights_sha256=np.array(WD.state_dict_digest(sd)),
               out_min=np.float64(y_hf.min()), out_max=np.float64(y_hf.max()), out_mean=np.float64(y_hf.mean()),
               out_std=np.float64(y_hf.std()))
    if f16:
        rec[f"output_hf_sub{sub}_f16"] = y_hf[:, ::sub, ::sub].astype(np.float16)
    else:
        rec[f"output_hf_sub{sub}"] = y_hf[:, ::sub, ::sub].astype(np.float32)
    if use_fov:
        e = np.abs(fov_hf - fov_or.numpy()).max()
        print(f"  fov HF {fov_hf}  oracle {fov_or.numpy()}  max_abs {e:.3e}")
        assert e < 1e-3
        rec["fov_hf"] = fov_hf.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)


CASES = {
    "depth_pro_tiny_b2": dict(preset="tiny", batch=2),
    "depth_pro_shallow_b1": dict(preset="dinov2l16_384_shallow", batch=1, first_seed=300, sub=2, f16=True),
    "depth_pro_full_b1": dict(preset="dinov2l16_384", batch=1, first_seed=400, sub=2, f16=True),
}

if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name, kw in CASES.items():
        if len(sys.argv) == 1 or name in sys.argv[1:]:
            run_case(name, **kw)
