"""Tree-sharding's per-rank share: rank 0's trees of the C2 population under the 8-rank
owners rule, scored by the single-GPU call over the replicated 1M-row dataset, against the whole
population; per configuration of the probe / exact knobs: ms per call, kernel and busy ms, host phases,
and the implied 8-rank efficiency (t_all / (8 t_share)).  One JSON line per configuration."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SR_AMD_PKG=ab/<name>: another revision's package + library (tools/ab_lib.sh)
sys.path[:0] = [ROOT, os.path.join(ROOT, os.environ["SR_AMD_PKG"]) if os.environ.get("SR_AMD_PKG")
                else os.path.join(ROOT, "symbolicregression.jl_amd")]
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
    # extra settings: "probe" (mode 1), or knob=value arguments (e.g. chunk_min=128), each on its own
    knobs = [dict()] + ([dict(probe=1)] if "probe" in sys.argv[1:] else [])
    knobs += [{a.split("=")[0]: int(a.split("=")[1])} for a in sys.argv[1:] if "=" in a]
    defaults = {"probe": 2, "chunk_min": 1024, "max_row_blocks": 512, "first_chunk": 6}
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
        for k in kn:
            ctx.set_tuning(k, defaults[k])


if __name__ == "__main__":
    main()
