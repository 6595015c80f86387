"""Repeat test_probe_modes_change_nothing's comparison and report, per probe / cache mode and
repetition, how many flags and loss bits differ from the no-probe run (diagnosis of an intermittent
failure)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402
import sr_amd  # noqa: E402
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population  # noqa: E402

dtype = np.float32
rng = np.random.default_rng(12)
n = 1 << 18
X = rng.standard_normal((5, n)).astype(dtype)
X[1, 200_001] = dtype(95.0)
X[3, 150_003] = dtype(0.0)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dtype)
ds = Dataset(X, y)
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
tb = flatten_trees(gen_random_population(4000, opts, 5, seed=6), dtype)
ctx = sr_amd.get_context()
ref = None
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for probe, stress, cache, bal in ((0, 0, 1, 1), (2, 0, 1, 1), (2, 1, 1, 1), (1, 1, 1, 1), (2, 1, 0, 1),
                                      (0, 0, 1, 0), (0, 0, 0, 0)):
        ctx.set_tuning("probe", probe)
        ctx.set_tuning("stress_probe", stress)
        ctx.set_tuning("code_cache", cache)
        ctx.set_tuning("balance", bal)
        l, c = eval_loss_batch(tb, ds, opts)
        if ref is None:
            ref = (l.copy(), c.copy())
            print(f"reference: complete {c.mean():.4f}", flush=True)
            continue
        dc = np.nonzero(c != ref[1])[0]
        both = c & ref[1]
        dl = int(np.sum(l[both].view(np.uint32) != ref[0][both].view(np.uint32)))
        print(f"rep {rep} probe {probe} stress {stress} cache {cache} balance {bal}: flag diffs {len(dc)} "
              f"{[(int(k), bool(c[k]), bool(ref[1][k])) for k in dc[:4]]} loss-bit diffs {dl}", flush=True)
ctx.set_tuning("probe", 2); ctx.set_tuning("stress_probe", 1); ctx.set_tuning("code_cache", 1); ctx.set_tuning("balance", 1)
