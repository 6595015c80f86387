"""Diagnostic (GPU): the device gradient of the trees where test_grad_f64_many_features_deep_trees_weighted
disagrees with the oracle's finite differences, with the tree, its loss and both gradients."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
from oracle import Oracle  # noqa: E402
from sr_amd import Dataset, Options, eval_grad_batch, flatten_trees, gen_random_population, string_tree  # noqa: E402

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "sin"])
rng = np.random.default_rng(12)
nf = 10
X = rng.standard_normal((nf, 1500))
y = np.cos(X[0]) + X[1] * X[2]
w = rng.uniform(0.5, 2.0, 1500)
trees = gen_random_population(300, opts, nf, max_size=30, seed=13)
tb = flatten_trees(trees, np.float64)
for weights in (w, None):
    loss, g, comp = eval_grad_batch(tb, Dataset(X, y, weights=weights), opts)
    g_fd, lo, comp_o, fd_err = Oracle.from_options(opts).loss_grad_fd(tb, X, y, weights, with_error=True)
    co = tb.constant_offsets()
    for t in np.nonzero(comp)[0]:
        a, b, e = g[co[t]:co[t + 1]], g_fd[co[t]:co[t + 1]], fd_err[co[t]:co[t + 1]]
        if len(a) == 0:
            continue
        scale = max(1.0, float(np.abs(b).max()))
        if np.all(np.abs(a - b) <= 2e-5 * scale):
            continue
        print("weighted" if weights is not None else "unweighted", t, string_tree(tb.tree(int(t)), opts.operators),
              "loss", loss[t], lo[t], "dev", a, "fd", b, "err", e, "depth", tb.tree(int(t)).count_depth())
