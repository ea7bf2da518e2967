"""The oracle (oracle/dav2_ref.py) against the committed golden fixtures,
which tests/golden/make_golden.py generated from transformers'
DepthAnythingForDepthEstimation (the in-container stand-in for the
un-vendored upstream Depth-Anything-V2 repo).  CPU only."""

import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from monocular_depth_estimation_trt_amd import pack, weights
from oracle import dav2_ref


def _load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", ["dav2_vits_metric_98", "dav2_vits_relative_98", "dav2_vitb_relative_98", "dav2_vitl_metric_98"])
def test_oracle_matches_hf_golden(name):
    z = _load(name)
    cfg = weights.model_config(str(z["encoder"]), str(z["depth_type"]))
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    assert weights.state_dict_digest(sd) == str(z["weights_sha256"]), "weight generator drifted"
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    y = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, z["input"]).numpy()
    ref = z["output_hf"]
    assert y.shape == ref.shape
    err = np.abs(y - ref)
    assert err.max() < 1e-3 and err.mean() / np.abs(ref).mean() < 1e-5, (err.max(), err.mean())


@pytest.mark.parametrize("name,encoder", [("dav2_vits_metric_518", "vits"), ("dav2_vitl_metric_518", "vitl")])
def test_oracle_518_golden_full_map(name, encoder):
    """Full 518x518 map (stored f16: <= 7.9e-3 quantisation at depths < 32)."""
    z = _load(name)
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    assert weights.state_dict_digest(sd) == str(z["weights_sha256"]), "weight generator drifted"
    x = weights.synthetic_images(1, 518, 518, first_seed=int(z["input_first_seed"]))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    y = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    ref = z["output_hf_f16"].astype(np.float32)
    assert y.shape == ref.shape == (1, 518, 518)
    np.testing.assert_allclose(y, ref, atol=8e-3, rtol=0)
    assert abs(y.mean() - float(z["out_mean"])) < 1e-4
    assert abs(y.std() - float(z["out_std"])) < 1e-4


def test_pos_embed_interpolation_golden():
    """Upstream DINOv2 bicubic + 0.1-offset interpolation, oracle and packer."""
    z = _load("posembed_upstream")
    cfg = weights.model_config("vits")
    pos = weights.synthetic_state_dict(cfg, 1234)["pretrained.pos_embed"]
    np.testing.assert_array_equal(pos[:, :8], z["pos_37_first_rows"])
    for ph, pw in ((7, 7), (9, 13)):
        o = dav2_ref.interpolate_pos_embed(torch.from_numpy(pos), ph, pw).numpy()
        p = pack.interpolate_pos_embed(pos, ph, pw)
        np.testing.assert_allclose(o, z[f"pos_{ph}x{pw}"], atol=1e-6)
        np.testing.assert_allclose(p, z[f"pos_{ph}x{pw}"], atol=1e-6)
    assert pack.interpolate_pos_embed(pos, 37, 37) is not None


def test_synthetic_inputs_are_the_spec_domain():
    x = weights.synthetic_images(2, 28, 42, first_seed=0)
    assert x.shape == (2, 3, 28, 42) and x.dtype == np.float32
    lo = (0 - weights.IMAGENET_MEAN) / weights.IMAGENET_STD
    hi = (1 - weights.IMAGENET_MEAN) / weights.IMAGENET_STD
    for c in range(3):
        assert x[:, c].min() >= lo[c] - 1e-5 and x[:, c].max() <= hi[c] + 1e-5
    assert not np.array_equal(x[0], x[1])
    np.testing.assert_array_equal(x, weights.synthetic_images(2, 28, 42, first_seed=0))


def test_output_depends_on_input():
    """Fan-in scaled weights give a depth map that depends on the image
    (HF default init is flat: SURVEY.md 0.5)."""
    cfg = weights.model_config("vits")
    sd = dav2_ref.to_torch(weights.synthetic_state_dict(cfg, 1234))
    a = dav2_ref.forward(sd, cfg, weights.synthetic_images(1, 70, 70, first_seed=1)).numpy().ravel()
    b = dav2_ref.forward(sd, cfg, weights.synthetic_images(1, 70, 70, first_seed=2)).numpy().ravel()
    assert a.std() > 0.1 and abs(np.corrcoef(a, b)[0, 1]) < 0.9
