"""Summarise tools/r06_c2_variants.sh output: walk statistics and one line per variant."""
import glob
import json
import os
import sys

d = sys.argv[1]
for line in open(f"{d}/stats.err"):
    if "[sr fold]" in line:
        print(line.rstrip()[:200])
for f in sorted(glob.glob(f"{d}/v*.json")):
    env = open(f[:-5] + ".env").read().strip()
    try:
        b = json.loads([l for l in open(f) if l.startswith("{")][-1])
        rf = b["config"].get("ref_fold") or {}
        print(f"{os.path.basename(f)} [{env or 'defaults'}] ms/step {b['ms_per_step']:.3f} min/med/max "
              f"{b['step_ms_min_median_max']} busy {b['roofline'].get('busy_ms_per_step', 0):.3f} fold {rf}")
    except (IndexError, KeyError, ValueError) as e:
        print(f, env, "no line", e)
