"""models/<name>/spec.json reader for the HIP engine's drivers.

Contract (what the reference's `core/spec.py` promises its callers, :39-111):
the same schema number and required keys, `SpecError` (a ValueError) naming
the file and the first rule a spec breaks, `load` by model name or by path,
`load_all` keyed by folder name, `size_of` defaulting to the first build
target, `caveats`.  The reference's own spec files load here unchanged
(tests/test_spec_loader.py).  Standard library only, so a driver can read a
spec without importing torch or the engine.

The checks are a table of (rule, predicate) pairs run in order; the first
failing predicate raises.  On top of the reference contract this module maps
a DA-V2-family spec to the engine build config (`model_config_of`).
"""

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
MODELS = os.path.join(HERE, "models")

SCHEMA = 1
REQUIRED = ("schema", "name", "env", "input", "outputs", "profiles", "build_targets")
INPUT_KEYS = ("name", "rank", "dtype", "layout")
OUTPUT_KEYS = ("name", "meaning")


class SpecError(ValueError):
    """A spec.json that breaks the schema."""


def _is_hw(v):
    return isinstance(v, list) and len(v) == 2 and all(isinstance(x, int) and x > 0 for x in v)


def _rules(spec):
    """Yield (message, ok) in check order; messages keep the reference's
    wording for the conditions its tests match on."""
    absent = [k for k in REQUIRED if k not in spec]
    yield f"missing {absent}", not absent
    yield f"schema {spec['schema']}, expected {SCHEMA}", spec["schema"] == SCHEMA
    inp = spec["input"]
    for k in INPUT_KEYS:
        yield f"input.{k} missing", k in inp
    yield f"input.rank {inp['rank']} is not 4 or 5", inp["rank"] in (4, 5)
    yield "outputs is empty", bool(spec["outputs"])
    for out in spec["outputs"]:
        for k in OUTPUT_KEYS:
            yield f"output.{k} missing in {out}", k in out
    yield "profiles is empty", bool(spec["profiles"])
    for name, prof in spec["profiles"].items():
        yield f"profile {name} size must be [h, w], got {prof.get('size')}", _is_hw(prof.get("size"))
    yield "build_targets is empty -- nothing would be built", bool(spec["build_targets"])
    for tgt in spec["build_targets"]:
        yield f"build target {tgt} names an unknown profile", tgt.get("profile") in spec["profiles"]


def validate(spec, where="<spec>"):
    for msg, ok in _rules(spec):
        if not ok:
            raise SpecError(f"{where}: {msg}")
    return spec


def path_for(name, models_dir=None):
    return os.path.join(models_dir or MODELS, name, "spec.json")


def load(name_or_path, models_dir=None):
    """One spec, by model folder name (under models_dir) or by a .json path."""
    path = name_or_path if name_or_path.endswith(".json") else path_for(name_or_path, models_dir)
    if not os.path.isfile(path):
        raise SpecError(f"no spec at {path}")
    with open(path, encoding="utf-8") as f:
        return validate(json.load(f), path)


def load_all(models_dir=None):
    """{folder name: spec} for every folder of models_dir holding a spec.json."""
    root = models_dir or MODELS
    if not os.path.isdir(root):
        return {}
    names = sorted(d for d in os.listdir(root) if os.path.isfile(path_for(d, root)))
    return {d: load(path_for(d, root)) for d in names}


def size_of(spec, profile=None):
    """(h, w) of a profile; the first build target's profile by default."""
    prof = profile if profile is not None else spec["build_targets"][0]["profile"]
    h, w = spec["profiles"][prof]["size"]
    return (h, w)


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
