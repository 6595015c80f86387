"""Tree sharding at 8 ranks, measured on one GPU: every rank's share of the C2
population under an owners rule, scored by the single-GPU call over the replicated 1M-row dataset.
Rules: `nodes` (the library's: node count, snake order) and `cost` (a static per-tree cost from the
interpreter's cost model, DESIGN §12, dealt longest-first to the least-loaded rank).  Knob sweeps on
rank 0's share: the two-chunk pipeline's smallest first chunk and row blocks per tree.  One JSON line
per measurement."""
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

# DESIGN §12's cost model (ms per 10k trees x 1M rows): per tree ~2.1, binary ~0.95, cos 6.7, exp 2.6,
# log ~ 3 (its body is ~2/3 of cos's f64 work), leaves ride on their parent's instruction
UNARY_COST = {"cos": 6.7, "sin": 6.7, "exp": 2.6, "log": 3.0}


def static_cost(tb, opts):
    deg, op = tb.degree, tb.op
    names = list(bench.C2_OPS["unary_operators"])
    node = np.zeros(len(deg))
    node[deg == 2] = 0.95
    for i, n in enumerate(names):  # (op is the 1-based operator index)
        node[(deg == 1) & (op == i + 1)] = UNARY_COST.get(n, 1.0)
    cs = np.concatenate([[0], np.cumsum(node)])
    return 2.1 + cs[tb.offsets[1:]] - cs[tb.offsets[:-1]]


def cost_owners(cost, world):
    order = np.argsort(-cost, kind="stable")
    load = np.zeros(world)
    out = np.empty(len(cost), dtype=np.int64)
    for t in order:
        r = int(np.argmin(load))
        out[t] = r
        load[r] += cost[t]
    return out


def main():
    ctx = sr_amd.get_context()
    opts = Options(**bench.C2_OPS)
    X, y = bench.c2_data(1 << 20, 0)
    ds = Dataset(X, y)
    trees = gen_random_population(10_000, opts, 5, max_size=30, seed=1)
    tb = flatten_trees(trees, np.float32)

    def measure(b, n=20, w=5):
        call, _ = bench.single_gpu_call(ctx, b, ds, opts)
        st = {}
        dt, _, kms = bench.timed(bench.lib_step(ctx, call, st), n, w, lambda: None)
        return {"trees": int(b.n_trees), "ms": dt / n * 1e3, "kernel_ms": float(np.mean(kms)),
                "phases": [round(x, 4) for x in ctx.last_phase_ms()], "exact_trees": ctx.last_exact_trees()}

    base = measure(tb)
    print(json.dumps({"what": "all", **base}), flush=True)
    cost = static_cost(tb, opts)
    for rule, own in (("nodes", tree_owners(tb, 8)), ("cost", cost_owners(cost, 8))):
        shares = []
        for r in range(8):
            m = measure(tb.take(np.nonzero(own == r)[0]), 10, 3)
            m["est_cost"] = float(cost[own == r].sum())
            shares.append(m)
            print(json.dumps({"what": f"share_{rule}", "rank": r, **m}), flush=True)
        worst = max(s["ms"] for s in shares)
        print(json.dumps({"what": f"rule_{rule}", "max_share_ms": worst, "rank0_ms": shares[0]["ms"],
                          "efficiency_max": base["ms"] / (8 * worst),
                          "efficiency_rank0": base["ms"] / (8 * shares[0]["ms"]),
                          "kernel_ms": [round(s["kernel_ms"], 3) for s in shares]}), flush=True)
    share = tb.take(np.nonzero(tree_owners(tb, 8) == 0)[0])
    for knob, vals, dflt in (("chunk_min", (1024, 256, 128), 1024), ("max_row_blocks", (512, 1024, 2048), 512)):
        for v in vals:
            ctx.set_tuning(knob, v)
            m = measure(share)
            a = measure(tb, 10, 3)
            print(json.dumps({"what": "knob", "knob": knob, "value": v, "share": m, "all_ms": a["ms"],
                              "efficiency_rank0": a["ms"] / (8 * m["ms"])}), flush=True)
        ctx.set_tuning(knob, dflt)


if __name__ == "__main__":
    main()
