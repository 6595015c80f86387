"""Interpreter kernel time per tree against population size (the tree-sharding share's regime):
the first n trees of the C2 population (n = 1,250 .. 10,000) over the 1M-row C2 data in one chunk, and
the 1,250-tree share under a few launch knobs.  One JSON line per measurement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, flatten_trees, gen_random_population  # noqa: E402
from sr_amd.distributed import tree_owners  # noqa: E402


def main():
    ctx = sr_amd.get_context()
    opts = Options(**bench.C2_OPS)
    X, y = bench.c2_data(1 << 20, 0)
    ds = Dataset(X, y)
    tb = flatten_trees(gen_random_population(10_000, opts, 5, max_size=30, seed=1), np.float32)
    share = tb.take(np.nonzero(tree_owners(tb, 8) == 0)[0])

    def measure(b, n=10, w=3):
        call, _ = bench.single_gpu_call(ctx, b, ds, opts)
        st = {}
        dt, _, kms = bench.timed(bench.lib_step(ctx, call, st), n, w, lambda: None)
        return {"trees": int(b.n_trees), "ms": dt / n * 1e3, "kernel_ms": float(np.mean(kms)),
                "launches": st["launches"][-1], "phases": [round(x, 4) for x in ctx.last_phase_ms()]}

    ctx.set_tuning("chunk_min", 1 << 30)  # one chunk at every size
    for n in (1250, 2500, 5000, 10000):
        m = measure(tb.take(np.arange(n)))
        m["kernel_us_per_tree"] = m["kernel_ms"] * 1e3 / n
        print(json.dumps({"what": "prefix", **m}), flush=True)
    m = measure(share)
    m["kernel_us_per_tree"] = m["kernel_ms"] * 1e3 / share.n_trees
    print(json.dumps({"what": "share", **m}), flush=True)
    for knob, vals, dflt in (("code_cache", (0,), 1), ("probe", (1,), 2), ("max_row_blocks", (1024, 256), 512)):
        for v in vals:
            ctx.set_tuning(knob, v)
            m = measure(share)
            m["kernel_us_per_tree"] = m["kernel_ms"] * 1e3 / share.n_trees
            print(json.dumps({"what": "share_knob", "knob": knob, "value": v, **m}), flush=True)
        ctx.set_tuning(knob, dflt)
    ctx.set_tuning("chunk_min", 1024)


if __name__ == "__main__":
    main()
