"""Per-call step-time jitter on C2 (GPU box): wall time, kernel time and host phases of 60
consecutive eval_loss_batch calls, then which phase carries the spread."""
import os, sys, time
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
tb = flatten_trees(gen_random_population(10000, opts, 5, seed=1), np.float32)
for _ in range(3):
    eval_loss_batch(tb, ds, opts)
rows = []
for _ in range(60):
    t0 = time.perf_counter()
    eval_loss_batch(tb, ds, opts)
    wall = (time.perf_counter() - t0) * 1e3
    rows.append([wall, ctx.last_kernel_ms()[0]] + ctx.last_phase_ms())
a = np.array(rows)
names = ["wall", "kernel", "compile", "launch", "wait", "exact", "final"]
for i, nm in enumerate(names):
    c = np.corrcoef(a[:, 0], a[:, i])[0, 1] if i else 1.0
    print(f"{nm:8s} p10={np.percentile(a[:, i], 10):7.3f} p50={np.median(a[:, i]):7.3f} "
          f"p90={np.percentile(a[:, i], 90):7.3f} ms  corr(wall)={c:+.2f}", flush=True)
print("walls:", " ".join(f"{v:.2f}" for v in a[:, 0]))
