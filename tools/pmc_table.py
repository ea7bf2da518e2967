"""One row per (kernel, grid) of a tools/pmc_profile.sh output directory,
with the derived rates the limiter analysis needs (MI355X_MICROARCH.md units:
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs;
FETCH_SIZE / WRITE_SIZE in KB).

    python tools/pmc_table.py OUTDIR [--cus 256] [--match SUBSTR]

Columns: avg duration (us, kernel trace of pass 0); clock = GRBM / 8 / dur;
mfma% = MFMA busy cycles / (SIMDs x kernel cycles); valu% = VALU issue
cycles (ACTIVE_INST_VALU x 4) / (SIMDs x kernel cycles); waves = resident
waves per SIMD (WAVE_CYCLES x 4 / (SIMDs x kernel cycles)); wait% = WAIT_ANY /
WAVE_CYCLES; lds% = LDS-active / WAVE_CYCLES; MB = HBM bytes per launch
(FETCH_SIZE + WRITE_SIZE; the guide's gfx950 corrections are tools/pmc_traffic.py's).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row.get("Kernel_Name", ""), int(float(row.get("Grid_Size", 0) or 0)))
                vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(root, "p0", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                g = int(row.get("Grid_Size_X", 0) or 0) * int(row.get("Grid_Size_Y", 1) or 1) * \
                    int(row.get("Grid_Size_Z", 1) or 1)
                durs[(row["Kernel_Name"], g)].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals, durs


def main(argv):
    root = argv[0]
    cus = int(argv[argv.index("--cus") + 1]) if "--cus" in argv else 256
    match = argv[argv.index("--match") + 1] if "--match" in argv else ""
    vals, durs = load(root)
    simds = 4 * cus
    rows = []
    for (name, grid), d in vals.items():
        if match and match not in name:
            continue
        m = {k: sum(v) / len(v) for k, v in d.items()}
        dl = durs.get((name, grid)) or []
        dur = sum(dl) / len(dl) if dl else 0.0
        grbm = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # kernel cycles per XCD
        if grbm <= 0:
            continue
        kc = simds * grbm
        rows.append((m.get("GRBM_GUI_ACTIVE", 0.0), name, grid, dur / 1e3, grbm / dur * 1e3 if dur else 0.0,
                     100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / kc,
                     100 * 4 * m.get("SQ_ACTIVE_INST_VALU", 0.0) / kc,
                     4 * m.get("SQ_WAVE_CYCLES", 0.0) / kc,
                     100 * m.get("SQ_WAIT_ANY", 0.0) / max(1.0, m.get("SQ_WAVE_CYCLES", 0.0)),
                     100 * m.get("SQ_ACTIVE_INST_LDS", 0.0) / max(1.0, m.get("SQ_WAVE_CYCLES", 0.0)),
                     m.get("SQ_INSTS_VALU", 0.0) / max(1.0, m.get("SQ_INSTS_MFMA", 0.0)),
                     (m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) / 1e3,
                     m.get("SQ_LDS_BANK_CONFLICT", 0.0)))
    rows.sort(reverse=True)
    print(f"{'kernel':70s} {'grid':>9s} {'us':>7s} {'GHz':>5s} {'mfma%':>6s} {'valu%':>6s} {'waves':>5s} "
          f"{'wait%':>6s} {'lds%':>5s} {'v/mf':>5s} {'MB':>7s} {'bankc':>8s}")
    for _, name, grid, us, ghz, mf, va, wv, wt, ld, vm, mb, bc in rows:
        short = name.replace("mde::(anonymous namespace)::", "").replace("void ", "")[:70]
        print(f"{short:70s} {grid:9d} {us:7.1f} {ghz / 1e3:5.2f} {mf:6.1f} {va:6.1f} {wv:5.2f} {wt:6.1f} {ld:5.1f} "
              f"{vm:5.1f} {mb:7.1f} {bc:8.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
