"""Summarise rocprofv3 output dirs: per-kernel mean duration (kernel trace) and mean PMC counter
values per dispatch, plus the derived per-dispatch HBM bytes (FETCH_SIZE/WRITE_SIZE are KiB; gfx950
needs the x2 correction of MI355X_MICROARCH.md's HBM section)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")[:80]


def main(root):
    out = []
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        out.append(f"# kernel stats: {os.path.relpath(f, root)}")
        for row in csv.DictReader(open(f)):
            out.append(f"{short(row['Name']):80s} calls={row['Calls']:>4s} avg_ms={float(row['AverageNs']) / 1e6:9.4f}"
                       f" total_ms={float(row['TotalDurationNs']) / 1e6:9.3f} pct={row['Percentage']}")
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        out.append(f"# PMC means per dispatch: {k}")
        for c, v in sorted(cs.items()):
            out.append(f"  {c:28s} {sum(v) / len(v):16.6g}   (n={len(v)})")
        if "FETCH_SIZE" in cs:
            fb = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
            out.append(f"  HBM read bytes/dispatch (FETCH_SIZE KiB x1024 x2 gfx950) {fb:.4g}")
        if "WRITE_SIZE" in cs:
            wb = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024 * 2
            out.append(f"  HBM write bytes/dispatch (WRITE_SIZE KiB x1024 x2 gfx950) {wb:.4g}")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
