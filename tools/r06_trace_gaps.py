"""Round 6: summarise a rocprofv3 kernel (+ HIP API) trace database — per-kernel averages, the average
idle gap before each kernel, and one call's window (analysis only).
usage: python tools/r06_trace_gaps.py <results.db> [window_start_index]"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
w0 = int(sys.argv[2]) if len(sys.argv) > 2 else None
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))


def short(n):
    return re.sub(r"\(.*", "", n)[:56]


dur = defaultdict(list)
gap = defaultdict(list)
for i, (n, s, e) in enumerate(rows):
    dur[short(n)].append((e - s) / 1000)
    if i:
        g = (s - rows[i - 1][2]) / 1000
        if g < 200:  # (gaps inside a call; longer ones are the host between search iterations)
            gap[short(rows[i - 1][0]) + " -> " + short(n)].append(g)
print(f"{len(rows)} kernels")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:56s} n {len(v):6d} avg {sum(v) / len(v):8.2f} us  total {sum(v) / 1000:8.2f} ms")
print("gaps (< 200 us) by kernel pair:")
for k, v in sorted(gap.items(), key=lambda kv: -sum(kv[1]))[:12]:
    print(f"  {k:110s} n {len(v):6d} avg {sum(v) / len(v):7.2f} us")
if w0 is None:
    w0 = len(rows) // 2
base = rows[w0][1]
ev = [(s, "K " + short(n), e) for n, s, e in rows[w0:w0 + 12]]
try:
    t1 = rows[min(len(rows) - 1, w0 + 12)][2]
    ev += [(s, "A " + n, e) for n, s, e in c.execute(
        f"select name, start, end from regions where start >= {base - 30000} and start <= {t1} order by start")]
except sqlite3.Error:
    pass
for s, n, e in sorted(ev):
    print(f"{(s - base) / 1000:9.1f} {(e - base) / 1000:9.1f} {n}")
