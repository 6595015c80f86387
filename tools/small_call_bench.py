"""Latency of small scoring calls (the search's regime: ~20-40 trees x 100 rows per call).

Prints, per configuration, the mean wall time of one sr_eval_loss_batch call and its host-side
phases (sr_last_phase_ms: compile, upload + launch, wait, exact, finalize)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population  # noqa: E402

ctx = sr_amd.get_context()
CONFIGS = ((np.float64, 100, 20), (np.float64, 100, 40), (np.float32, 100_000, 31), (np.float64, 100, 280))
# SMALL_CONFIGS=2 (comma-separated indices) runs a subset
_pick = os.environ.get("SMALL_CONFIGS")
for dt, n_rows, n_trees in ([CONFIGS[int(i)] for i in _pick.split(",")] if _pick else CONFIGS):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((2, n_rows)).astype(dt)
    y = (2 * np.cos(X[1]) + X[0] ** 2 - 2).astype(dt)
    ds = Dataset(X, y)
    opts = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"])
    tb = flatten_trees(gen_random_population(n_trees, opts, 2, max_size=15, seed=1), dt)
    for _ in range(50):
        eval_loss_batch(tb, ds, opts)
    reps = 2000 if n_rows <= 1000 else 300
    ph = np.zeros(5)
    t0 = time.perf_counter()
    for _ in range(reps):
        eval_loss_batch(tb, ds, opts)
        ph += np.array(ctx.last_phase_ms())
    wall = (time.perf_counter() - t0) / reps * 1e6
    ph = ph / reps * 1e3
    print(f"{np.dtype(dt).name} rows={n_rows:7d} trees={n_trees:4d}  {wall:8.1f} us/call  phases(us) "
          f"compile={ph[0]:.1f} upload+launch={ph[1]:.1f} wait={ph[2]:.1f} exact={ph[3]:.1f} final={ph[4]:.1f}",
          flush=True)
