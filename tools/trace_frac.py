"""Recompute bench.py's roofline from a rocprofv3 kernel trace of the same command.

  python3 tools/trace_frac.py OUTDIR      (OUTDIR from tools/bench_evidence.sh)

Reads OUTDIR/kt/kt_kernel_trace.csv and OUTDIR/bench_traced.json (the bench line printed by the
traced run).  The interpreter launches of the C2 step are the f32 BASIC loss kernel
(sr_tile_kernel<float, R, 0, ...> with the bench line's R, probes included: the bench's HIP events bracket them too); the
last steps x launches_per_step of them are the timed region.  Prints the per-step kernel time and
roofline fraction from the trace next to the bench's own (HIP-event) values, and, when the PMC pass
ran, the HBM bytes per step from FETCH_SIZE (x 1024 B/KiB x 2, the gfx950 correction of
MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import re
import sys


def main(out, workload="c2"):
    line = json.loads(open(os.path.join(out, "bench_traced.json")).read().strip().splitlines()[-1])
    if workload == "c4":  # the c4 sub-object: its launches are the last ones of the run
        line = line["c4"]
    rf = line["roofline"]
    steps, per_step = line["steps"], rf["launches_per_step"]
    rows = list(csv.DictReader(open(glob.glob(os.path.join(out, "kt", "*kernel_trace.csv"))[0])))
    rpl = rf["kernel"].split("<float,")[1].split(",")[0]  # rows per lane of the build the bench ran
    # every f32 BASIC-tier LOSS launch (mode 0, no gather, tier 0, 4 waves): the bench's build and the
    # dead-tree probe, which runs on the classic 8-rows/lane build whatever the main launches use
    pat = re.compile(r"void sr_tile_kernel<float, \d+, 0, (false|true), 0, 4, ")
    prefix = f"void sr_tile_kernel<float, {rpl}, 0,"
    interp = [r for r in rows if pat.match(r["Kernel_Name"])]
    interp.sort(key=lambda r: int(r["Start_Timestamp"]))
    # probes: dead-tree probe launches (small grids) before the large chunks — since round 5 before a
    # large first chunk too; when every launch of the run belongs to its warm-up + timed steps (the
    # C2-only command of tools/r05_evidence.sh), the launches per step follow from the count
    warm = line.get("warmup", 0)
    if len(interp) % (steps + warm) == 0 and len(interp) // (steps + warm) >= per_step:
        probes_per_step = len(interp) // (steps + warm) - per_step
    else:
        probes_per_step = 1 if per_step == 2 else 0
    k = steps * (per_step + probes_per_step)
    timed = interp[-k:]
    ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed)
    trace_ms = ns / 1e6 / steps
    achieved = rf["flops_per_step"] / (trace_ms * 1e-3) / 1e12
    print(f"bench (traced run) : kernel {rf['kernel_ms_per_step']:.3f} ms/step (HIP events), frac {rf['frac']:.4f}")
    print(f"kernel trace       : {len(interp)} interpreter launches, last {k} = {steps} timed steps x "
          f"({per_step} + {probes_per_step} probe)")
    print(f"                     kernel {trace_ms:.3f} ms/step, achieved {achieved:.2f} TFLOP/s, "
          f"frac {achieved / rf['peak']:.4f} (peak {rf['peak']})")
    print(f"agreement          : trace / events = {trace_ms / rf['kernel_ms_per_step']:.4f}")
    pm = glob.glob(os.path.join(out, "pmc", "*counter_collection.csv"))
    if pm:
        fetch = {}
        for r in csv.DictReader(open(pm[0])):
            if r.get("Counter_Name") == "FETCH_SIZE" and pat.match(r["Kernel_Name"]):
                fetch[r["Dispatch_Id"]] = fetch.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        vals = [fetch[d] for d in sorted(fetch, key=int)][-k:]
        if vals:
            per_step_bytes = sum(vals) * 1024 * 2 / steps
            print(f"HBM (FETCH_SIZE)   : {per_step_bytes / 1e6:.1f} MB/step over the timed launches "
                  f"(algorithmic {rf['algorithmic_bytes_per_step'] / 1e6:.1f} MB)")
            json.dump({"workload": workload, "kernel": f"sr_tile_kernel<float, {rpl}, 0, ...> + the probe launches",
                       "profiled_steps": steps, "launches": len(vals),
                       "n_trees": line.get("config", line).get("n_trees", line.get("n_trees")),
                       "rows_per_gpu": line.get("config", line).get("rows_per_gpu", line.get("rows_per_gpu")),
                       "hbm_read_bytes_per_step": per_step_bytes,
                       "source_cmd": "tools/bench_evidence.sh"},
                      open(os.path.join(out, "traffic.json" if workload == "c2" else f"traffic_{workload}.json"), "w"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c2")
