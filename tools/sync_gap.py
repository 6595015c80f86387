"""Where a small scoring call's wall time goes, from a rocprofv3 trace of tools/small_call_bench.py
(kernel, memory-copy and HIP API traces): per hipStreamSynchronize, the gap between the end of the last
device operation of its call and the return of the synchronize, and the device-side chain (copy start
-> interpreter start -> interpreter end).  usage: python3 tools/sync_gap.py TRACE_DIR"""
import csv
import glob
import os
import sys

import numpy as np


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main(d):
    api = rows(d, "*hip_api_trace.csv")
    kt = rows(d, "*kernel_trace.csv")
    mc = rows(d, "*memory_copy_trace.csv")
    syncs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                   if r["Function"] in ("hipStreamSynchronize", "hipEventSynchronize"))
    launches = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                      if r["Function"] in ("hipLaunchKernel", "hipExtLaunchKernel", "hipModuleLaunchKernel"))
    copies_api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                        if r["Function"] in ("hipMemcpyAsync",))
    dev = sorted([(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "k:" + r["Kernel_Name"][:40]) for r in kt] +
                 [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy") for r in mc])
    ends = np.array([e for _, e, _ in dev])
    starts = np.array([s for s, _, _ in dev])
    gaps, waits, chain = [], [], []
    for s0, s1 in syncs[len(syncs) // 4:]:  # (skip the warm-up)
        i = np.searchsorted(ends, s1) - 1  # last device op ending before the sync returns
        if i < 0:
            continue
        gaps.append((s1 - ends[i]) / 1e3)
        waits.append((s1 - s0) / 1e3)
    for name, a in (("sync return - last device end (us)", gaps), ("hipStreamSynchronize duration (us)", waits)):
        a = np.array(a)
        print(f"{name:40s} median {np.median(a):7.2f}  p10 {np.percentile(a, 10):7.2f}  p90 {np.percentile(a, 90):7.2f}  n {len(a)}")
    for name, a in (("hipLaunchKernel (us)", launches), ("hipMemcpyAsync (us)", copies_api)):
        d_ = np.array([(e - s) / 1e3 for s, e in a[len(a) // 4:]])
        if len(d_):
            print(f"{name:40s} median {np.median(d_):7.2f}  p90 {np.percentile(d_, 90):7.2f}  n {len(d_)}")
    kd = np.array([(e - s) / 1e3 for s, e, n in dev[len(dev) // 4:] if n.startswith("k:")])
    cd = np.array([(e - s) / 1e3 for s, e, n in dev[len(dev) // 4:] if n == "copy"])
    if len(kd):
        print(f"{'kernel duration (us)':40s} median {np.median(kd):7.2f}  p90 {np.percentile(kd, 90):7.2f}  n {len(kd)}")
    if len(cd):
        print(f"{'device copy duration (us)':40s} median {np.median(cd):7.2f}  p90 {np.percentile(cd, 90):7.2f}  n {len(cd)}")
    # device gaps between consecutive ops (copy -> kernel within a call)
    g2 = np.array([(starts[i + 1] - ends[i]) / 1e3 for i in range(len(dev) // 4, len(dev) - 1)])
    print(f"{'device idle between ops (us)':40s} median {np.median(g2):7.2f}  p10 {np.percentile(g2, 10):7.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
