"""Tree-sharding's per-rank share: rank 0's trees of the C2 population under the 8-rank
owners rule, scored by the single-GPU call over the replicated 1M-row dataset, against the whole
population; per configuration of the probe / exact knobs: ms per call, kernel and busy ms, host phases,
and the implied 8-rank efficiency (t_all / (8 t_share)).  One JSON line per configuration."""
import json
import os
import sys
import time

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
    trees = gen_random_population(10_000, opts, 5, max_size=30, seed=1)
    tb = flatten_trees(trees, np.float32)
    share = tb.take(np.nonzero(tree_owners(tb, 8) == 0)[0])
    knobs = [dict()] + ([dict(probe=1)] if "probe" in sys.argv[1:] else [])
    for kn in knobs:
        for k, v in kn.items():
            ctx.set_tuning(k, v)
        row = {"knobs": kn, "env": {k: v for k, v in os.environ.items() if k.startswith("SR_AMD_")}}
        for name, b in (("all", tb), ("share", share)):
            call, _ = bench.single_gpu_call(ctx, b, ds, opts)
            st = {}
            dt, _, kms = bench.timed(bench.lib_step(ctx, call, st), 20, 5, lambda: None)
            row[name] = {"trees": int(b.n_trees), "ms": dt / 20 * 1e3, "kernel_ms": float(np.mean(kms)),
                         "busy_ms": float(np.mean(st["busy"][-20:])), "phases": ctx.last_phase_ms(),
                         "exact_trees": ctx.last_exact_trees(), "exact_kernel_ms": ctx.last_exact_kernel_ms()}
        row["efficiency_8"] = row["all"]["ms"] / (8 * row["share"]["ms"])
        print(json.dumps(row), flush=True)
        ctx.set_tuning("probe", 2)


if __name__ == "__main__":
    main()
