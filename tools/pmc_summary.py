"""Summarise tools/pmc_profile.sh output: mean counter value per (kernel, grid)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")[:90]
            grid = int(float(row.get("Grid_Size", 0) or 0))
            vals[(name, grid)][row["Counter_Name"]].append(float(row["Counter_Value"]))
for (k, g), d in sorted(vals.items(), key=lambda kv: -max(sum(v) / len(v) for v in kv[1].values())):
    print(f"{k}  grid={g}")
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
