"""Device occupancy of a traced run: union of the kernel (and copy) intervals over the traced span,
the time with >= 2 kernels in flight, and per-kernel counts / mean durations.
usage: python tools/trace_union.py <dir holding rocprofv3 *_kernel_trace.csv [and *_memory_copy_trace.csv]>"""
import collections
import csv
import glob
import os
import sys


def load(pattern):
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append(r)
    return rows


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def overlap2(iv):  # time with >= 2 intervals open
    ev = sorted([(s, 1) for s, e in iv] + [(e, -1) for s, e in iv])
    n, last, tot = 0, None, 0
    for t, d in ev:
        if n >= 2:
            tot += t - last
        n += d
        last = t
    return tot


k = load("*kernel_trace.csv")
c = load("*memory_copy_trace.csv")
kiv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in k]
civ = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in c]
if not kiv:
    sys.exit("no kernel trace rows")
# the search's own span: from its first interpreter launch to the last kernel
t0 = min(s for s, e in kiv)
t1 = max(e for s, e in kiv)
span = t1 - t0
print(f"kernels {len(kiv)}  copies {len(civ)}  span {span / 1e6:.1f} ms")
print(f"kernel union {union(kiv) / 1e6:.1f} ms = {union(kiv) / span:.3f} of span; >=2 kernels in flight {overlap2(kiv) / 1e6:.1f} ms")
if civ:
    print(f"copy union {union(civ) / 1e6:.1f} ms; kernels+copies union {union(kiv + civ) / span:.3f} of span")
by = collections.defaultdict(list)
for r in k:
    by[r["Kernel_Name"][:90]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for name, d in sorted(by.items(), key=lambda x: -sum(x[1])):
    print(f"{len(d):8d} x {sum(d) / len(d) / 1e3:8.2f} us  total {sum(d) / 1e6:8.1f} ms  {name}")
if civ:
    d = [e - s for s, e in civ]
    print(f"{len(d):8d} copies x {sum(d) / len(d) / 1e3:8.2f} us")
