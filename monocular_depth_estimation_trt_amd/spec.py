"""Read and validate models/<name>/spec.json -- the drop-in for the
reference's `core/spec.py` (:39-111): same schema, same REQUIRED keys, same
SpecError on a malformed spec, stdlib-only.  The reference's own spec files
load with it unchanged (tests/test_spec_loader.py)."""

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
MODELS = os.path.join(HERE, "models")

SCHEMA = 1
REQUIRED = ("schema", "name", "env", "input", "outputs", "profiles", "build_targets")


class SpecError(ValueError):
    pass


def path_for(name, models_dir=None):
    return os.path.join(models_dir or MODELS, name, "spec.json")


def load(name_or_path, models_dir=None):
    """One spec by model name (under models_dir) or by path to a .json."""
    p = name_or_path if name_or_path.endswith(".json") else path_for(name_or_path, models_dir)
    if not os.path.isfile(p):
        raise SpecError(f"no spec at {p}")
    with open(p, encoding="utf-8") as f:
        spec = json.load(f)
    validate(spec, p)
    return spec


def load_all(models_dir=None):
    root = models_dir or MODELS
    out = {}
    if not os.path.isdir(root):
        return out
    for d in sorted(os.listdir(root)):
        p = path_for(d, root)
        if os.path.isfile(p):
            out[d] = load(p)
    return out


def validate(spec, where="<spec>"):
    missing = [k for k in REQUIRED if k not in spec]
    if missing:
        raise SpecError(f"{where}: missing {missing}")
    if spec["schema"] != SCHEMA:
        raise SpecError(f"{where}: schema {spec['schema']}, expected {SCHEMA}")
    inp = spec["input"]
    for k in ("name", "rank", "dtype", "layout"):
        if k not in inp:
            raise SpecError(f"{where}: input.{k} missing")
    if inp["rank"] not in (4, 5):
        raise SpecError(f"{where}: input.rank {inp['rank']} is not 4 or 5")
    if not spec["outputs"]:
        raise SpecError(f"{where}: outputs is empty")
    for o in spec["outputs"]:
        for k in ("name", "meaning"):
            if k not in o:
                raise SpecError(f"{where}: output.{k} missing in {o}")
    if not spec["profiles"]:
        raise SpecError(f"{where}: profiles is empty")
    for pname, prof in spec["profiles"].items():
        size = prof.get("size")
        if not (isinstance(size, list) and len(size) == 2 and all(isinstance(v, int) and v > 0 for v in size)):
            raise SpecError(f"{where}: profile {pname} size must be [h, w], got {size}")
    if not spec["build_targets"]:
        raise SpecError(f"{where}: build_targets is empty")
    for t in spec["build_targets"]:
        if t.get("profile") not in spec["profiles"]:
            raise SpecError(f"{where}: build target {t} names an unknown profile")
    return spec


def size_of(spec, profile=None):
    if profile is None:
        profile = spec["build_targets"][0]["profile"]
    return tuple(spec["profiles"][profile]["size"])


def caveats(spec):
    return list(spec.get("caveats", []))


# checkpoint-family encoder names -> DA-V2 encoder (distill_any_depth uses
# small/base/large for the vits/vitb/vitl graphs, reference
# models/distill_any_depth/infer.py:32-69)
ENCODER_ALIASES = {"small": "vits", "base": "vitb", "large": "vitl"}


def model_config_of(spec):
    """The engine build config a DA-V2-family spec implies (encoder, head,
    size, post-process)."""
    enc = spec.get("encoder", {}).get("used", "vits")
    enc = ENCODER_ALIASES.get(enc, enc)
    depth_type = "metric" if spec.get("depth_scale", "metric") == "metric" else "relative"
    return {"encoder": enc, "depth_type": depth_type, "max_depth": float(spec.get("max_depth", 20.0)),
            "input_hw": size_of(spec), "postprocess": spec.get("postprocess", "resize_clamp")}
