"""Large-row evidence (BASELINE C4 per-GPU shard): 100k C2-distribution trees x 8M rows (= 64M rows
over 8 GPUs) f32 on one GPU.  Prints one JSON line: node-evals/s, interpreter ms, algorithmic
HBM bytes and GB/s (same conventions as bench.py)."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), ROOT]
import numpy as np
import sr_amd
from sr_amd import Dataset, Options, eval_loss_batch, flatten_trees, gen_random_population
from bench import chunk_groups

ap = argparse.ArgumentParser()
ap.add_argument("--trees", type=int, default=100_000)
ap.add_argument("--rows", type=int, default=1 << 23)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
tb = flatten_trees(gen_random_population(args.trees, opts, 5, seed=4), np.float32)
rng = np.random.default_rng(2)
X = rng.standard_normal((5, args.rows), dtype=np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * rng.standard_normal(args.rows, dtype=np.float32)).astype(np.float32)
ds = Dataset(X, y)
ctx = sr_amd.get_context()
eval_loss_batch(tb, ds, opts)  # warm-up (upload, compile)
ks, launches = [], []
t0 = time.perf_counter()
for _ in range(args.steps):
    loss, comp = eval_loss_batch(tb, ds, opts)
    ks.append(ctx.last_kernel_ms()[0])
    launches.append(ctx.last_launches())
dt = (time.perf_counter() - t0) / args.steps
k = float(np.mean(ks))
n_passes = sum(-(-c // g) for c, g in chunk_groups(tb.n_trees, args.rows, launches[-1]))
alg_bytes = float(n_passes) * 6 * args.rows * 4
print(json.dumps({"config": f"C4 per-GPU shard: {args.trees} trees x {args.rows} rows x 5 features f32",
                  "node_evals_per_s": float(tb.n_nodes) * args.rows / dt, "ms_per_step": dt * 1e3,
                  "kernel_ms": k, "launches": launches[-1], "fraction_complete": float(comp.mean()),
                  "algorithmic_bytes_per_step": alg_bytes, "algorithmic_GBps": alg_bytes / (k * 1e-3) / 1e9,
                  "flops_per_step": float(args.rows) * (tb.n_operator_nodes + 3 * tb.n_trees),
                  "achieved_TFLOPs": float(args.rows) * (tb.n_operator_nodes + 3 * tb.n_trees) / (k * 1e-3) / 1e12}),
      flush=True)
