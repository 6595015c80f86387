"""Debug helper (GPU box): f64 population — trees whose GPU complete flag differs from the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
from sr_amd import *
from sr_amd import _lib
from oracle import Oracle
import ctypes

opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
rng = np.random.default_rng(5)
n = 3000
X = rng.standard_normal((5, n))
y = 2 * np.cos(X[3]) + X[0] ** 2 - 2
tb = flatten_trees(gen_random_population(1500, opts, 5, max_size=30, dtype=np.float64, seed=5), np.float64)
ds = Dataset(X, y)
loss, comp = eval_loss_batch(tb, ds, opts)
orc = Oracle.from_options(opts)
ol, oc = orc.eval_loss_batch(tb, X, y, accum="f64", n_threads=8)
bad = np.nonzero(comp != oc)[0]
print("mismatches", len(bad), "gpu complete", comp.sum(), "oracle complete", oc.sum())
from sr_amd.distributed import gpu_partials
sums, flags = gpu_partials(tb, ds, opts, n)
for k in bad[:8]:
    print("tree", k, "gpu", comp[k], loss[k], "oracle", oc[k], ol[k], "flags", flags[k], "sum", sums[k])
    print("  ", string_tree(tb.tree(k), opts.operators))
