"""Throughput of the batched forward-mode gradient (sr_eval_grad_batch) and of batched BFGS
(optimize_constants_batch) on C5-style data: f64, Feynman-style 5-feature target, 100k rows."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np
import sr_amd
from sr_amd import Dataset, Options, eval_grad_batch, eval_loss_batch, flatten_trees, gen_random_population
from sr_amd import optimize_constants_batch

for dt in (np.float64, np.float32):
    rng = np.random.default_rng(1)
    X = rng.uniform(1, 5, size=(5, 100_000)).astype(dt)
    y = (X[0] * X[1] * X[2] / (X[3] * X[4] ** 2 + 1)).astype(dt)
    ds = Dataset(X, y)
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    tb = flatten_trees(gen_random_population(2000, opts, 5, max_size=20, seed=3, dtype=dt), dt)
    nconst = int(tb.constant_mask().sum())
    ctx = sr_amd.get_context()
    eval_grad_batch(tb, ds, opts)
    t0 = time.perf_counter()
    for _ in range(5):
        l, g, c = eval_grad_batch(tb, ds, opts)
    tg = (time.perf_counter() - t0) / 5
    eval_loss_batch(tb, ds, opts)
    t0 = time.perf_counter()
    for _ in range(5):
        eval_loss_batch(tb, ds, opts)
    tl = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    _, _, improved, evals = optimize_constants_batch(tb, ds, opts, np.random.default_rng(0))
    tb_s = time.perf_counter() - t0
    print(json.dumps({"dtype": np.dtype(dt).name, "trees": tb.n_trees, "nodes": int(tb.n_nodes), "constants": nconst,
                      "rows": X.shape[1], "complete": float(c.mean()), "eval_loss_ms": tl * 1e3,
                      "eval_grad_ms": tg * 1e3,
                      "grad_constant_rows_per_s": nconst * X.shape[1] / tg,
                      "bfgs_s": tb_s, "bfgs_improved": int(np.sum(improved)), "bfgs_loss_evals": float(np.sum(evals))}),
          flush=True)
