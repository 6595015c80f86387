"""Dead-tree probe mode A/B (sr_set_tuning "probe": 1 = before every chunk, 2 = only before the chunks
after the first): the C2 step, rank 0's 8-rank tree share, the 100k-tree population and a C3-sized
call (31 trees x 100k rows), alternating passes.  One JSON line per (population, mode, pass)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, flatten_trees, gen_random_batch, gen_random_population  # noqa: E402
from sr_amd.distributed import tree_owners  # noqa: E402


def main():
    ctx = sr_amd.get_context()
    opts = Options(**bench.C2_OPS)
    X, y = bench.c2_data(1 << 20, 0)
    ds = Dataset(X, y)
    tb = flatten_trees(gen_random_population(10_000, opts, 5, max_size=30, seed=1), np.float32)
    pops = {"c2": (tb, ds), "share": (tb.take(np.nonzero(tree_owners(tb, 8) == 0)[0]), ds),
            "100k": (gen_random_batch(100_000, opts, 5, max_size=30, seed=4), ds)}
    Xs, ys = bench.c2_data(100_000, 1)
    pops["small"] = (flatten_trees(gen_random_population(31, opts, 5, max_size=30, seed=3), np.float32), Dataset(Xs, ys))
    modes = [int(m) for m in sys.argv[1:]] or [2, 1]
    for pas in range(2):
        for m in modes:
            ctx.set_tuning("probe", m)
            for name, (b, d) in pops.items():
                call, _ = bench.single_gpu_call(ctx, b, d, opts)
                st = {}
                n = 5 if name == "100k" else 20
                dt, _, kms = bench.timed(bench.lib_step(ctx, call, st), n, 3, lambda: None)
                print(json.dumps({"pop": name, "probe": m, "pass": pas, "trees": int(b.n_trees), "ms": dt / n * 1e3,
                                  "kernel_ms": float(np.mean(kms)), "phases": [round(x, 4) for x in ctx.last_phase_ms()]}),
                      flush=True)
    ctx.set_tuning("probe", 2)


if __name__ == "__main__":
    main()
