"""C4's 8-rank projection term: rank 0's 8M-row shard of the 100k-tree C4 population through
sr_eval_loss_sharded at world size 1, per tuning knob setting (alternating passes).  One JSON line per
(pass, setting): ms per call, kernel ms, host phases, exact trees.
usage: python tools/c4_shard_probe.py [max_row_blocks=512,256,128] [probe=2,1] [passes=2]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, gen_random_batch  # noqa: E402
from sr_amd.distributed import eval_loss_sharded, init_device_comm  # noqa: E402


def main():
    knobs, passes = [], 2
    for a in sys.argv[1:]:
        k, v = a.split("=")
        if k == "passes":
            passes = int(v)
        else:
            knobs.append((k, [int(x) for x in v.split(",")]))
    settings = [{}] + [{k: v} for k, vs in knobs for v in vs]
    comm = bench.Comm(1, 0)
    ctx = sr_amd.get_context()
    init_device_comm(ctx=ctx)
    opts = Options(**bench.C2_OPS)
    tb = gen_random_batch(100_000, opts, 5, max_size=30, seed=4)
    X, y = bench.c4_shard(0, 8, 1 << 26)
    ds = Dataset(X, y)
    ds.device_handle(ctx)
    del X, y
    defaults = {"max_row_blocks": 512, "probe": 2, "chunk_min": 1024}
    for p in range(passes):
        for s in settings:
            for k, v in s.items():
                ctx.set_tuning(k, v)
            st = {}
            dt, _, kms = bench.timed(bench.lib_step(ctx, lambda: eval_loss_sharded(tb, ds, opts), st), 3, 1, comm.barrier)
            print(json.dumps({"pass": p, "setting": s, "ms": dt / 3 * 1e3, "kernel_ms": float(np.mean(kms)),
                              "phases": [round(float(v), 3) for v in ctx.last_phase_ms()],
                              "exact_trees": ctx.last_exact_trees()}), flush=True)
            for k in s:
                ctx.set_tuning(k, defaults[k])
    comm.close()


if __name__ == "__main__":
    main()
