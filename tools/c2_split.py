"""C2 population split by completeness: kernel time of all / complete-only / incomplete-only trees."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
import sr_amd
from sr_amd import Options, Dataset, flatten_trees, gen_random_population, eval_loss_batch

n = 1 << 20
rng = np.random.default_rng(2)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
trees = gen_random_population(10000, opts, 5, seed=1)
tb = flatten_trees(trees, np.float32)
_, comp = eval_loss_batch(tb, ds, opts)
sets = {"all": trees, "complete": [t for t, c in zip(trees, comp) if c],
        "incomplete": [t for t, c in zip(trees, comp) if not c]}
for name, ts in sets.items():
    b = flatten_trees(ts, np.float32)
    eval_loss_batch(b, ds, opts)
    ks = []
    for _ in range(5):
        eval_loss_batch(b, ds, opts)
        ks.append(ctx.last_kernel_ms()[0])
    print(f"{name:11s} trees={b.n_trees:6d} nodes={b.n_nodes:7d} kernel={np.median(ks):.3f} ms", flush=True)
