"""spec.py mirrors core/spec.py validation; the shipped DA-V2 spec is valid and
agrees with what the engine builds."""

import json
import os
import tempfile

import pytest

from monocular_depth_estimation_trt_amd import spec

REF_SPEC = "/root/reference/models/depth_anything_v2/spec.json"


def test_shipped_spec():
    s = spec.load("depth_anything_v2")
    assert spec.size_of(s) == (518, 518)
    assert s["input"]["name"] == "input" and s["outputs"][0]["name"] == "output"
    assert s["build_targets"][0]["precision"] == "fp16"
    assert spec.model_config_of(s) == {"encoder": "vits", "depth_type": "metric", "max_depth": 20.0,
                                       "input_hw": (518, 518), "postprocess": "resize_clamp"}
    assert {"depth_anything_v2", "depth_anything_ac", "distill_any_depth"} <= set(spec.load_all())


@pytest.mark.parametrize("name,post", [("depth_anything_ac", "resize_clamp"), ("distill_any_depth", "none")])
def test_family_specs(name, post):
    """The DA-V2 family: the same ViT-S graph with the
    relative head; distill_any_depth's 'small' is the vits graph."""
    mc = spec.model_config_of(spec.load(name))
    assert mc["encoder"] == "vits" and mc["depth_type"] == "relative" and mc["postprocess"] == post
    assert mc["input_hw"] == (518, 518)


@pytest.mark.parametrize("name", ["depth_anything_ac", "distill_any_depth"])
def test_reference_family_specs_load_unchanged(name):
    p = f"/root/reference/models/{name}/spec.json"
    if not os.path.exists(p):
        pytest.skip("reference checkout not present")
    mc = spec.model_config_of(spec.load(p))
    assert mc["encoder"] == "vits" and mc["depth_type"] == "relative"


@pytest.mark.skipif(not os.path.exists(REF_SPEC), reason="reference checkout not present")
def test_reference_spec_loads_unchanged():
    s = spec.load(REF_SPEC)
    assert spec.size_of(s) == (518, 518) and s["encoder"]["used"] == "vits"


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: d.pop("outputs"), "missing"),
    (lambda d: d.update(schema=2), "schema"),
    (lambda d: d["input"].update(rank=3), "rank"),
    (lambda d: d["profiles"]["bench"].update(size=[518]), "size"),
    (lambda d: d.update(build_targets=[{"profile": "nope"}]), "unknown profile"),
    (lambda d: d.update(build_targets=[]), "empty"),
])
def test_invalid_specs_raise(mutate, msg):
    d = json.load(open(spec.path_for("depth_anything_v2")))
    mutate(d)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "spec.json")
        json.dump(d, open(p, "w"))
        with pytest.raises(spec.SpecError, match=msg):
            spec.load(p)


def test_spec_module_is_stdlib_only():
    src = open(spec.__file__).read()
    imports = {l.split()[1].split(".")[0] for l in src.splitlines() if l.startswith(("import ", "from "))}
    assert imports <= {"json", "os"}, imports
