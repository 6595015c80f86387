"""The gradient kernel's bench workload (bench.py grad_roofline: the C5 search's final members with
constants, sr_eval_grad_batch over the full 100k rows in Float64) in a process of its own, so a
rocprofv3 kernel trace / PMC pass of it holds those launches only (2 warm-up + 5 timed calls).

  python3 tools/c5_grad_profile.py --save OUT.npz    # run the C5 search (bench.py's options, seed 0)
  python3 tools/c5_grad_profile.py --load OUT.npz    # the roofline calls alone (profile this one)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

FIELDS = ("offsets", "degree", "op", "feature", "constant", "val")


def c5_setup():
    from sr_amd import Options

    rng = np.random.default_rng(11)
    X3 = rng.uniform(0.5, 2.0, (5, 100_000)).astype(np.float32)
    y3 = (X3[0] * X3[1] * X3[2] / (X3[3] * X3[4] ** 2 + 1)).astype(np.float32)
    o5 = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"], populations=32,
                 should_optimize_constants=True)
    return X3.astype(np.float64), y3.astype(np.float64), o5


def main():
    from sr_amd import equation_search, flatten_trees
    from sr_amd.node import TreeBatch

    X, y, o = c5_setup()
    if sys.argv[1] == "--save":
        res = equation_search(X, y, niterations=int(os.environ.get("C5_ITERS", "40")), options=o, seed=0)
        trees = [m.tree for p in res.populations for m in p if m.tree.count_constants() > 0]
        tb = flatten_trees(trees, np.float64)
        np.savez(sys.argv[2], **{f: getattr(tb, f) for f in FIELDS})
        print(json.dumps({"saved_trees": tb.n_trees}))
        return
    import bench

    d = np.load(sys.argv[2])
    tb = TreeBatch(*[d[f] for f in FIELDS])
    print(json.dumps(bench.grad_roofline_batch(tb, X, y, o)))


if __name__ == "__main__":
    main()
