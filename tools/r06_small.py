"""Round 6: a C3-sized scoring call (31 trees x 100k rows, f32) timed alone, with and without the
in-order fold (analysis only).  usage: python tools/r06_small.py [n_trees] [rows]"""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd")]
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population  # noqa: E402

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 31
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
rng = np.random.default_rng(11)
X = rng.uniform(0.5, 2.0, (5, n)).astype(np.float32)
y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(np.float32)
o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
trees = gen_random_population(nt, o, 5, max_size=20, seed=3)
tb = flatten_trees(trees, np.float32)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
for rf in (1, 0):
    ctx.set_tuning("ref_fold", rf)
    for _ in range(20):
        eval_loss_batch(tb, ds, o)
    t0 = time.perf_counter()
    k = 200
    for _ in range(k):
        loss, comp = eval_loss_batch(tb, ds, o)
    dt = (time.perf_counter() - t0) / k
    print(f"ref_fold {rf}: {dt * 1e6:.1f} us per call, complete {int(comp.sum())}/{nt}, fold {ctx.last_ref_fold()}",
          flush=True)
