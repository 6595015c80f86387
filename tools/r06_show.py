"""Summarise a tools/r06_fold_check.sh output directory: test verdicts, the C2 line, top kernels."""
import csv
import json
import sys

d = sys.argv[1]
try:
    for line in open(f"{d}/fold.log"):
        if "PASSED" in line or "FAILED" in line or "Error" in line:
            print(line.rstrip()[:160])
except OSError:
    pass
try:
    L = [l for l in open(f"{d}/bench.json") if l.startswith("{")]
    b = json.loads(L[-1])
    r = b["roofline"]
    print("C2 ms/step %.3f  value %.3e  frac %.4f  kernel %.3f  busy %.3f" % (
        b["ms_per_step"], b["value"], r["frac"], r.get("kernel_ms_per_step", 0), r.get("busy_ms_per_step", 0)))
    print("config:", {k: b["config"].get(k) for k in ("fold_trees", "ref_fold", "exact_trees")})
except (OSError, IndexError, KeyError) as e:
    print("no bench line", e)
try:
    rows = list(csv.DictReader(open(f"{d}/kt/kt_kernel_stats.csv")))
    for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:10]:
        print(x["Calls"], "%.1f us" % (float(x["AverageNs"]) / 1e3), "%.2f ms" % (float(x["TotalDurationNs"]) / 1e6), x["Name"][:90])
except OSError:
    pass
