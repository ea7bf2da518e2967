"""Timing loop and result record -- the drop-in for the reference's
`core/bench.py` (schema 1), restated for the HIP engine.

Semantics kept exactly (pinned by the reference's tests/test_bench.py:30-245
and by tests/test_bench_record.py here):

* wall clock of one call, `sync` INSIDE the timed region, warmup excluded
  (core/bench.py:182-210);
* nearest-rank percentiles, rank = ceil(q/100 * N) (:110-121);
* optional GPU stage split + `host_overhead_ms` clamped at 0 (:123-150);
* record file `<model>_<H>x<W>_<profile>_<variant>_<precision>.json`
  (:322-340), `schema` stamped, loading another schema raises ValueError.

Differences: `backend` defaults to "mde-hip"; `collect_env` reads the AMD
device through libmde_hip (or torch) instead of nvidia-smi.
"""

from __future__ import annotations

import json
import math
import os
import platform
import statistics
import time
from dataclasses import asdict, dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np

SCHEMA = 1


@dataclass
class Bench:
    """Timing samples plus everything needed to reproduce them."""

    model: str
    samples_ms: List[float] = field(default_factory=list)
    warmup: int = 0
    stage_samples_ms: Dict[str, List[float]] = field(default_factory=dict)
    backend: str = "mde-hip"
    precision: str = "fp16"
    profile: str = "bench"
    variant: str = "single"
    encoder: str = ""
    input_h: int = 0
    input_w: int = 0
    device: str = ""
    driver: str = ""
    clock_mhz: int = 0
    clock_max_mhz: int = 0
    versions: Dict[str, str] = field(default_factory=dict)
    host: str = field(default_factory=platform.node)
    outputs: Dict[str, dict] = field(default_factory=dict)
    engine_path: str = ""
    engine_bytes: int = 0
    engine_mtime: int = 0
    onnx_sha256: str = ""
    timestamp: str = ""
    notes: str = ""

    @property
    def iterations(self) -> int:
        return len(self.samples_ms)

    @property
    def mean_ms(self) -> float:
        return statistics.fmean(self.samples_ms) if self.samples_ms else 0.0

    @property
    def fps(self) -> float:
        m = self.mean_ms
        return 1000.0 / m if m else 0.0

    def pct(self, q: float) -> float:
        """Nearest-rank percentile, q in [0, 100]: always an observed sample."""
        if not self.samples_ms:
            return 0.0
        s = sorted(self.samples_ms)
        rank = math.ceil(q / 100.0 * len(s))
        return s[min(len(s) - 1, max(0, rank - 1))]

    def stats(self) -> dict:
        if not self.samples_ms:
            return {}
        n = self.iterations
        out = {
            "iterations": n,
            "warmup": self.warmup,
            "mean_ms": round(self.mean_ms, 4),
            "min_ms": round(min(self.samples_ms), 4),
            "p50_ms": round(self.pct(50), 4),
            "p90_ms": round(self.pct(90), 4),
            "p99_ms": round(self.pct(99), 4),
            "max_ms": round(max(self.samples_ms), 4),
            "stdev_ms": round(statistics.stdev(self.samples_ms), 4) if n > 1 else 0.0,
            "fps": round(self.fps, 2),
        }
        for name, vals in self.stage_samples_ms.items():
            if vals:
                out[name] = round(statistics.fmean(vals), 4)
        if self.stage_samples_ms:
            covered = sum(out.get(k, 0.0) for k in ("h2d_ms", "compute_ms", "d2h_ms"))
            out["host_overhead_ms"] = round(max(0.0, out["mean_ms"] - covered), 4)
        return out

    def report(self) -> str:
        if not self.samples_ms:
            return "[MDET] no samples"
        s = self.stats()
        total = sum(self.samples_ms) / 1000.0
        lines = [
            f"[MDET] {self.iterations} iterations time: {total:.4f} [sec]",
            f"[MDET] Average FPS: {s['fps']:.2f} [fps]",
            f"[MDET] Average inference time: {s['mean_ms']:.2f} [msec]",
            f"[MDET] p50 {s['p50_ms']:.2f} / p90 {s['p90_ms']:.2f} / p99 {s['p99_ms']:.2f} [msec], "
            f"min {s['min_ms']:.2f}, stdev {s['stdev_ms']:.2f}",
        ]
        if "compute_ms" in s:
            lines.append(f"[MDET] h2d {s.get('h2d_ms', 0):.3f} / compute {s['compute_ms']:.3f} / "
                         f"d2h {s.get('d2h_ms', 0):.3f} / host {s.get('host_overhead_ms', 0):.3f} [msec]")
        return "\n".join(lines)

    def to_dict(self) -> dict:
        d = asdict(self)
        d["schema"] = SCHEMA
        d["stats"] = self.stats()
        d["samples_ms"] = [round(x, 4) for x in self.samples_ms]
        return d


def _default_sync() -> Callable[[], None]:
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.synchronize
    except ImportError:
        pass
    return lambda: None


def measure(fn: Callable[[], object], *, warmup: int = 10, iterations: int = 100,
            sync: Optional[Callable[[], None]] = None):
    """Run fn; return (last return value, per-iteration ms).  `sync` runs
    inside the timed region and must block until the work is finished."""
    sync = sync or _default_sync()
    for _ in range(warmup):
        fn()
    sync()
    out, samples = None, []
    for _ in range(iterations):
        t0 = time.perf_counter()
        out = fn()
        sync()
        samples.append((time.perf_counter() - t0) * 1000.0)
    return out, samples


def measure_staged(fn: Callable[[], object], probe: Callable[[], Dict[str, float]], *, warmup: int = 10,
                   iterations: int = 100, sync: Optional[Callable[[], None]] = None):
    """measure() plus one probe() (e.g. StageTimer.last) per iteration, read
    outside the timed region.  Returns (out, samples_ms, {phase: [ms...]})."""
    sync = sync or _default_sync()
    for _ in range(warmup):
        fn()
    sync()
    out, samples, stages = None, [], {}
    for _ in range(iterations):
        t0 = time.perf_counter()
        out = fn()
        sync()
        samples.append((time.perf_counter() - t0) * 1000.0)
        for name, ms in (probe() or {}).items():
            stages.setdefault(name, []).append(float(ms))
    return out, samples, stages


def summarize_outputs(outputs: Dict[str, np.ndarray]) -> Dict[str, dict]:
    """Shape/dtype/min/max/mean of each output; non-finite values counted,
    never folded into the statistics."""
    res = {}
    for name, arr in outputs.items():
        a = np.asarray(arr)
        fin = np.isfinite(a)
        v = a[fin]
        res[name] = {"shape": list(a.shape), "dtype": str(a.dtype), "finite": int(fin.sum()),
                     "nonfinite": int(a.size - fin.sum()),
                     "min": float(v.min()) if v.size else None,
                     "max": float(v.max()) if v.size else None,
                     "mean": float(v.mean()) if v.size else None}
    return res


def collect_env() -> dict:
    """Versions and device (AMD: through libmde_hip / torch, no nvidia-smi)."""
    env, device = {}, ""
    env["python"] = platform.python_version()
    try:
        import torch
        env["torch"] = torch.__version__
        env["hip"] = str(getattr(torch.version, "hip", "") or "")
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(0)
            device = f"{p.name} ({getattr(p, 'gcnArchName', '')})"
    except Exception:
        pass
    try:
        from . import _lib
        env["mde_abi"] = str(_lib.lib().mde_version())
    except Exception:
        pass
    return {"versions": env, "device": device, "driver": "", "clock_mhz": 0, "clock_max_mhz": 0}


def save(bench: Bench, out_dir: str) -> str:
    """Write <out_dir>/<model>[_HxW]_<profile>_<variant>_<precision>.json."""
    os.makedirs(out_dir, exist_ok=True)
    if not bench.timestamp:
        bench.timestamp = time.strftime("%Y-%m-%dT%H:%M:%S")
    if not bench.device:
        bench.__dict__.update(collect_env())
    parts = [bench.model, bench.profile, bench.variant, bench.precision]
    if bench.input_h and bench.input_w:
        parts.insert(1, f"{bench.input_h}x{bench.input_w}")
    path = os.path.join(out_dir, "_".join(str(p) for p in parts if p) + ".json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(bench.to_dict(), f, indent=2, ensure_ascii=False)
    return path


REPORTS = os.path.join(os.getcwd(), "reports", "bench")


def record(model: str, samples_ms, *, outputs: Optional[Dict[str, np.ndarray]] = None,
           model_input: Optional[np.ndarray] = None, out_dir: Optional[str] = None, echo: bool = True,
           **kw) -> Bench:
    """Print the [MDET] report and write the record (one call per run)."""
    b = Bench(model=model, samples_ms=list(samples_ms), **kw)
    if b.engine_path and os.path.exists(b.engine_path):
        st = os.stat(b.engine_path)
        b.engine_bytes, b.engine_mtime = int(st.st_size), int(st.st_mtime)
    if outputs:
        b.outputs = summarize_outputs(outputs)
    out_dir = out_dir or REPORTS
    if model_input is not None:
        inputs = os.path.join(os.path.dirname(out_dir), "inputs")
        os.makedirs(inputs, exist_ok=True)
        np.save(os.path.join(inputs, f"{model}.npy"), np.ascontiguousarray(model_input))
    if echo:
        print(b.report())
    path = save(b, out_dir)
    if echo:
        print(f"[MDET] result -> {path}")
    return b


def load(path: str) -> dict:
    with open(path, encoding="utf-8") as f:
        d = json.load(f)
    if d.get("schema") != SCHEMA:
        raise ValueError(f"{path}: schema {d.get('schema')}, expected {SCHEMA}")
    return d


def load_all(bench_dir: str) -> List[dict]:
    if not os.path.isdir(bench_dir):
        return []
    return [load(os.path.join(bench_dir, n)) for n in sorted(os.listdir(bench_dir)) if n.endswith(".json")]
