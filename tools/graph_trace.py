"""Per-kernel timing INSIDE the replayed forward graph, from a rocprofv3
--kernel-trace CSV of bench.py (the per-layer pass times each layer alone,
with events between layers; in the graph consecutive kernels overlap at
their boundaries and a kernel's ramp / tail depends on its neighbours).

    python tools/graph_trace.py <dir with *kernel_trace.csv> [first-kernel-substring] [--last N] [--drop-last K] [--all]

A forward starts at each dispatch of the first kernel (default
patch_prep_kernel).  For the last N complete forwards (default 10) it
prints, per kernel position: mean duration, mean start gap after the
previous kernel's END (negative = overlapped), and the forward span.
"""
import csv
import re  # noqa: F401
import glob
import os
import statistics
import sys


def load(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main(argv):
    d = argv[0]
    first = argv[1] if len(argv) > 1 and not argv[1].startswith("--") else "patch_prep_kernel"
    last = int(argv[argv.index("--last") + 1]) if "--last" in argv else 10
    rows = load(d)
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    fw = [rows[a:b] for a, b in zip(starts, starts[1:])]
    if "--drop-last" in argv:  # e.g. bench.py's eager per-layer forward after the timed replays
        fw = fw[:len(fw) - int(argv[argv.index("--drop-last") + 1])]
    n = min(len(k) for k in fw[-last:])
    fw = [k for k in fw[-last:] if len(k) == n]
    print(f"{len(fw)} forwards of {n} kernels; span mean "
          f"{statistics.mean((k[-1][1] - k[0][0]) / 1e3 for k in fw):.1f} us")
    agg = {}
    for i in range(n):
        name = fw[0][i][2].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        dur = statistics.mean((k[i][1] - k[i][0]) / 1e3 for k in fw)
        gap = statistics.mean((k[i][0] - k[i - 1][1]) / 1e3 for k in fw) if i else 0.0
        a = agg.setdefault(name, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += dur
        a[2] += gap
        if "--all" in argv:
            print(f"{i:4d} {name:60s} {dur:8.1f} us  gap {gap:6.1f}")
    print(f"{'kernel':60s} {'n':>3s} {'sum dur us':>11s} {'sum gap us':>11s}")
    for name, (c, dsum, gsum) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{name:60s} {c:3d} {dsum:11.1f} {gsum:11.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
