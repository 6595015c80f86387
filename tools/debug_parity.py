"""Debug helper (GPU box): locate trees whose GPU loss differs from the oracle and show the rows."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import sr_amd
from sr_amd import *
from oracle import Oracle
from parity_util import well_conditioned, rel

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
n, nt, seed = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (4096, 3000, 1)
rng = np.random.default_rng(seed)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (2 * np.cos(X[3].astype(np.float64)) + X[0].astype(np.float64) ** 2 - 2
     + 0.1 * np.random.default_rng(seed + 1).standard_normal(n)).astype(np.float32)
tb = flatten_trees(gen_random_population(nt, opts, 5, max_size=30, seed=seed), np.float32)
loss, comp = eval_loss_batch(tb, Dataset(X, y), opts)
orc = Oracle.from_options(opts)
good, ol, oc = well_conditioned(orc, tb, X, y)
r = rel(loss, ol)
r[~good] = 0
worst = np.argsort(-r)[:5]
out, pc = eval_tree_array_batch(tb.subset(worst), Dataset(X), opts)
for j, k in enumerate(worst):
    print("tree", k, "rel", r[k], "gpu", loss[k], "oracle", ol[k])
    print("  ", string_tree(tb.tree(k), opts.operators))
    o, c = orc.eval_tree_array(tb, k, X)
    o64, _ = orc.eval_tree_array(tb.astype(np.float64), k, X.astype(np.float64))
    d = np.abs(out[j].astype(np.float64) - o)
    rows = np.argsort(-d)[:4]
    for i in rows:
        print("    row", i, "x", X[:, i], "gpu", out[j][i], "orc32", o[i], "orc64", o64[i], "y", y[i])
