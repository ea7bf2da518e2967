"""Fold the bench lines of tools/batch_sweep.sh into one JSON document:
per point img/s, ms per step, per-image latency and the model MFMA fraction
(model GFLOP x img/s / 2.5 PF/s), plus the dominant layer class."""
import glob
import json
import os
import sys


def main(d):
    pts = []
    for f in sorted(glob.glob(os.path.join(d, "vit*_b*.json"))):
        with open(f) as fh:
            lines = [ln for ln in fh.read().splitlines() if ln.startswith("{")]
        if not lines:
            continue
        r = json.loads(lines[-1])
        c = r["config"]
        pts.append({"encoder": c["encoder"], "batch": c["batch_per_gpu"], "img_s": r["value"],
                    "ms_per_step": r["ms_per_step"], "ms_per_image": round(r["ms_per_step"] / c["batch_per_gpu"], 4),
                    "model_mfma_frac": r["model_mfma_frac"], "dominant": r["roofline"]["kernel"],
                    "dominant_frac": r["roofline"]["frac"]})
    pts.sort(key=lambda p: (p["encoder"], p["batch"]))
    print(json.dumps({"what": "SURVEY 8(d) batch sweep, DA-V2 518x518 fp16, one MI355X, HBM-resident inputs, "
                              "hipGraph replay (bench.py --no-b1 --no-pcie)", "points": pts}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
