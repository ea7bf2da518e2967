"""get_engine() build-or-load logic (core/common.py:120-312 semantics) without
a GPU: the packed file, fingerprint and staleness decisions; the final load is
stubbed.  The real load is covered by tests/test_gpu_dropin.py."""

import os
import tempfile

import numpy as np
import pytest

from monocular_depth_estimation_trt_amd import common, weights
from monocular_depth_estimation_trt_amd.engine import Engine


@pytest.fixture
def stub_load(monkeypatch):
    calls = []

    def fake(path, device=0, **kw):
        calls.append((path, kw))
        return ("engine", path, kw)

    monkeypatch.setattr(Engine, "from_file", staticmethod(fake))
    return calls


def test_builds_then_reuses_then_rebuilds(stub_load, capsys):
    with tempfile.TemporaryDirectory() as td:
        eng = os.path.join(td, "engine", "dav2_vits_98.mdeng")
        src = "synthetic:vits:metric:3"
        common.get_engine(src, eng, "fp16", input_hw=(98, 98))
        assert os.path.exists(eng) and os.path.exists(os.path.splitext(eng)[0] + ".fingerprint")
        assert "Build engine" in capsys.readouterr().out
        m1 = os.path.getmtime(eng)
        common.get_engine(src, eng, "fp16", input_hw=(98, 98))
        assert "Load engine from file" in capsys.readouterr().out and os.path.getmtime(eng) == m1
        common.get_engine(src, eng, "fp16", input_hw=(112, 112))   # option change -> stale
        assert "Rebuilding engine" in capsys.readouterr().out
        assert len(stub_load) == 3


def test_dynamic_profile_passed_to_engine(stub_load):
    with tempfile.TemporaryDirectory() as td:
        eng = os.path.join(td, "e.mdeng")
        common.get_engine("synthetic:vits", eng, "fp16",
                          dynamic_input_shapes=[[1, 3, 70, 70], [4, 3, 70, 70], [8, 3, 70, 70]])
        kw = stub_load[-1][1]
        assert kw["profile"] == ((1, 3, 70, 70), (4, 3, 70, 70), (8, 3, 70, 70))


def test_checkpoint_source_npz(stub_load):
    cfg = weights.model_config("vits")
    sd = weights.synthetic_state_dict(cfg, 11)
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "ckpt.npz")
        np.savez(ck, **sd)
        eng = os.path.join(td, "e.mdeng")
        common.get_engine(ck, eng, "fp16", input_hw=(70, 70))
        assert os.path.getsize(eng) > 40e6
        assert common.load_checkpoint(ck)["pretrained.cls_token"].shape == (1, 1, 384)


def test_errors(stub_load):
    with tempfile.TemporaryDirectory() as td:
        with pytest.raises(FileNotFoundError):
            common.get_engine(os.path.join(td, "missing.pth"), os.path.join(td, "e.mdeng"), "fp16")
        with pytest.raises(ValueError):
            common.get_engine("synthetic:vits", os.path.join(td, "e.mdeng"), "int8")
        with pytest.raises(ValueError):
            common.get_engine("synthetic:vits", "", "fp16",
                              dynamic_input_shapes=[[1, 3, 70, 70], [1, 3, 84, 84], [2, 3, 70, 70]])


def test_precision_sets_residual_stream(stub_load):
    """precision "fp16" packs resid_f16 = 1 (f16 residual stream), "fp32" --
    the reference's default -- packs 0 (PackConfig byte 196)."""
    import struct
    with tempfile.TemporaryDirectory() as td:
        for prec, flag in (("fp16", 1), ("fp32", 0)):
            eng = os.path.join(td, f"e_{prec}.mdeng")
            common.get_engine("synthetic:vits", eng, prec, input_hw=(70, 70))
            blob = open(eng, "rb").read(32 + 256)
            assert struct.unpack_from("<i", blob, 32 + 196)[0] == flag, prec
            # byte 200: enc_f32 -- the exact-fp32 encoder of precision "fp32" (fp32.hip)
            assert struct.unpack_from("<i", blob, 32 + 200)[0] == (1 if prec == "fp32" else 0), prec
        common.get_engine("synthetic:vits", os.path.join(td, "d.mdeng"), input_hw=(70, 70))   # default: fp32
        assert struct.unpack_from("<i", open(os.path.join(td, "d.mdeng"), "rb").read(288), 228)[0] == 0


def test_fp32_pack_carries_fp32_encoder_weights():
    """precision "fp32" packs the patch embed and every block linear as fp32
    [Npad][Kpad32] (`*.w32`, the exact-fp32 GEMM's operand) and no f16 copy."""
    import numpy as np
    from monocular_depth_estimation_trt_amd import pack, weights
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 3)
    t = pack.packed_tensors(sd, cfg, 70, 70, enc_f32=True)
    assert t["patch.w32"].dtype == np.float32 and t["patch.w32"].shape == (384, 672)
    for i in range(cfg["depth"]):
        for n, shape in (("qkv", (1152, 384)), ("proj", (384, 384)), ("fc1", (1536, 384)), ("fc2", (384, 1536))):
            a = t[f"b{i}.{n}.w32"]
            assert a.dtype == np.float32 and a.shape == shape, (i, n, a.shape)
            assert f"b{i}.{n}.w" not in t
    w = sd["pretrained.blocks.0.attn.qkv.weight"]
    assert np.array_equal(t["b0.qkv.w32"][:w.shape[0], :w.shape[1]], w.astype(np.float32))


def test_staleness_rules():
    with tempfile.TemporaryDirectory() as td:
        e, f = os.path.join(td, "x.mdeng"), os.path.join(td, "x.fingerprint")
        assert common.engine_staleness(e, f, "fp", True) == "no engine file"
        open(e, "wb").write(b"x")
        assert common.engine_staleness(e, f, "fp", False) is None      # engine-only deployment
        assert common.engine_staleness(e, f, "fp", True) == "no fingerprint recorded"
        open(f, "w").write("other")
        assert "changed" in common.engine_staleness(e, f, "fp", True)
        open(f, "w").write("fp")
        assert common.engine_staleness(e, f, "fp", True) is None
