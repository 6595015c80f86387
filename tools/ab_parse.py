"""Summarise an A/B microbenchmark log (tools/ab_libs.sh / ab_env.sh): kernel / step / exact ms per
variant and population, the two passes side by side."""
import re
import sys
from collections import defaultdict

rows = defaultdict(list)
order, cur = [], None
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_libs.txt"):
    if line.startswith("=="):
        cur = line[3:].rsplit(" (pass", 1)[0].strip()
        if cur not in order:
            order.append(cur)
        continue
    m = re.search(r"^(\S+).*kernel=\s*([\d.]+)ms step=\s*([\d.]+)ms", line)
    if m and cur is not None:
        rows[(cur, m.group(1))].append((float(m.group(2)), float(m.group(3))))
mixes = []
for (v, mx) in rows:
    if mx not in mixes:
        mixes.append(mx)
print(f"{'variant':34s} " + " ".join(f"{m[:14]:>22s}" for m in mixes))
for v in order:
    cells = []
    for mx in mixes:
        r = rows.get((v, mx), [])
        cells.append("/".join(f"{k:.2f}" for k, _ in r) if r else "-")
    print(f"{v:34s} " + " ".join(f"{c:>22s}" for c in cells))
