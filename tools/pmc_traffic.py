"""HBM traffic per kernel launch from tools/profile_round.sh's PMC passes.

    python tools/pmc_traffic.py OUTDIR [layers.json]  > traffic.json

With the bench's --layers-json (the engine's layer names in launch order),
the dispatches of the LAST forward of each pass are matched to the layers
one for one (a split-K fc2's second kernel, splitk_resid_kernel, is added to
its layer), giving "layers": {name: bytes per launch} -- what bench.py's
roofline.traffic reads for the dominant layer class.

Per (kernel name, grid size): mean FETCH_SIZE and WRITE_SIZE over the
launches (rocprofv3 reports KiB), bytes = 2 x FETCH + WRITE (gfx950: FETCH_SIZE
tallies 128-B fabric reads at 64 B, MI355X_MICROARCH.md "HBM").  Infinity-
Cache hits are counted by these counters, so this is fabric traffic below
L2, an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def collect(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row.get("Kernel_Name", ""), int(float(row.get("Grid_Size", 0) or 0)))
                did = int(float(row.get("Dispatch_Id", 0) or 0))
                acc[key][row["Counter_Name"]].append((did, float(row["Counter_Value"])))

    def mean(v):
        return sum(v) / max(1, len(v))

    out = []
    for (name, grid), d in acc.items():
        fs = [v for _, v in sorted(d.get("FETCH_SIZE", []))]
        ws = [v for _, v in sorted(d.get("WRITE_SIZE", []))]
        f, w = mean(fs), mean(ws)
        rec = {"kernel": name, "grid": grid, "launches": len(fs),
               "fetch_kib": round(f, 1), "write_kib": round(w, 1),
               "hbm_bytes_per_launch": int((2 * f + w) * 1024)}
        # two layers sharing one kernel + grid alternate in dispatch order
        # (VGGT: attn.proj then mlp.fc2 per block): bytes of even / odd launches
        if len(fs) >= 4 and len(ws) == len(fs):
            rec["alternating_bytes_per_launch"] = [int((2 * mean(fs[i::2]) + mean(ws[i::2])) * 1024) for i in (0, 1)]
        out.append(rec)
    out.sort(key=lambda r: -r["hbm_bytes_per_launch"] * max(1, r["launches"]))
    return out


HELPERS = ("splitk_resid_kernel", "splitk_store_kernel", "attn_combine_kernel")  # second kernels of one engine step


def per_pass_rows(root):
    """{pass dir: [(dispatch id, kernel, {counter: value})] sorted by dispatch}"""
    out = {}
    for f in glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        rows = defaultdict(dict)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                did = int(float(row.get("Dispatch_Id", 0) or 0))
                names[did] = row.get("Kernel_Name", "")
                rows[did][row["Counter_Name"]] = float(row["Counter_Value"])
        out[f] = [(d, names[d], rows[d]) for d in sorted(rows)]
    return out


def layer_traffic(root, layer_names):
    """bytes per launch of each layer of the last forward (FETCH x2 + WRITE)."""
    fetch, write = {}, {}
    # with "resize_fold" on there are no ".resize" steps: a fusion resize that
    # a conv route cannot fold is launched inside the consumer conv's step,
    # ahead of it -- count it as a helper (its bytes go to the step before)
    helpers = HELPERS + (() if any(n.endswith(".resize") for n in layer_names) else ("resize_kernel",))
    for f, rows in per_pass_rows(root).items():
        # walk back from the end until len(layer_names) engine steps are covered
        n, i = 0, len(rows)
        while i > 0 and n < len(layer_names):
            i -= 1
            if not any(h in rows[i][1] for h in helpers):
                n += 1
        if n != len(layer_names):
            raise SystemExit(f"{f}: fewer dispatches than layers")
        fwd = rows[i:]
        j = 0
        for name in layer_names:
            d, kern, cnt = fwd[j]
            vals = [cnt]
            j += 1
            while j < len(fwd) and any(h in fwd[j][1] for h in helpers):
                vals.append(fwd[j][2])
                j += 1
            if ".attn" in name and "attn" not in kern:
                raise SystemExit(f"{f}: layer {name} aligned with kernel {kern}")
            for c, tgt in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write)):
                if c in cnt:
                    tgt[name] = sum(v.get(c, 0.0) for v in vals)
            fetch.setdefault("_kernels", {})[name] = kern.split("(")[0][:120]
    kern = fetch.pop("_kernels", {})
    return {n: {"kernel": kern.get(n, ""), "fetch_kib": round(fetch.get(n, 0.0), 1),
                "write_kib": round(write.get(n, 0.0), 1),
                "hbm_bytes_per_launch": int((2 * fetch.get(n, 0.0) + write.get(n, 0.0)) * 1024)}
            for n in layer_names if n in fetch and n in write}


if __name__ == "__main__":
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; bytes = 2*FETCH + WRITE",
           "kernels": collect(sys.argv[1])}
    if len(sys.argv) > 2:
        with open(sys.argv[2]) as f:
            names = list(json.load(f)["layer_ms"])
        doc["layers"] = layer_traffic(sys.argv[1], names)
    json.dump(doc, sys.stdout, indent=1)
