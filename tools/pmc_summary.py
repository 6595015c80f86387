"""Summarise rocprofv3 output dirs: per-kernel mean duration (kernel trace) and mean PMC counter
values per dispatch, plus the derived per-dispatch HBM bytes (FETCH_SIZE/WRITE_SIZE are KiB; gfx950
FETCH_SIZE needs the x2 correction of MI355X_MICROARCH.md's HBM section).

  python tools/pmc_summary.py DIR                        # text summary
  python tools/pmc_summary.py DIR --traffic-json PREFIX  # JSON for the kernel whose name starts with PREFIX
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")[:80]


def collect(root):
    stats = []
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            stats.append((short(row["Name"]), int(row["Calls"]), float(row["AverageNs"]), float(row["TotalDurationNs"]),
                          row["Percentage"]))
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return stats, vals


def mean(v):
    return sum(v) / len(v)


def main(root, traffic_prefix=None):
    stats, vals = collect(root)
    if traffic_prefix:
        # the dominant (longest total) kernel with this prefix
        cands = [s for s in stats if s[0].startswith(traffic_prefix)]
        cands.sort(key=lambda s: -s[3])
        if not cands:
            print(json.dumps({}))
            return
        name, calls, avg_ns = cands[0][0], cands[0][1], cands[0][2]
        cs = vals.get(name, {})
        out = {"kernel": name, "avg_ms": avg_ns / 1e6, "calls": calls}
        if "FETCH_SIZE" in cs:
            out["hbm_read_bytes_per_launch"] = mean(cs["FETCH_SIZE"]) * 1024 * 2
        if "WRITE_SIZE" in cs:
            out["hbm_write_bytes_per_launch"] = mean(cs["WRITE_SIZE"]) * 1024
        print(json.dumps(out))
        return
    out = []
    out.append(f"# kernel stats ({root})")
    for name, calls, avg, tot, pct in stats:
        out.append(f"{name:80s} calls={calls:>4d} avg_ms={avg / 1e6:9.4f} total_ms={tot / 1e6:9.3f} pct={pct}")
    for k, cs in vals.items():
        out.append(f"# PMC means per dispatch: {k}")
        for c, v in sorted(cs.items()):
            out.append(f"  {c:28s} {mean(v):16.6g}   (n={len(v)})")
        if "FETCH_SIZE" in cs:
            out.append(f"  HBM read bytes/dispatch (FETCH_SIZE KiB x1024 x2 gfx950) {mean(cs['FETCH_SIZE']) * 2048:.4g}")
        if "WRITE_SIZE" in cs:
            out.append(f"  HBM write bytes/dispatch (WRITE_SIZE KiB x1024) {mean(cs['WRITE_SIZE']) * 1024:.4g}")
    print("\n".join(out))


if __name__ == "__main__":
    args = sys.argv[1:]
    root = args[0] if args else "gpurun_out/prof"
    prefix = args[args.index("--traffic-json") + 1] if "--traffic-json" in args else None
    main(root, prefix)
